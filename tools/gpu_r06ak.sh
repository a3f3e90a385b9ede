#!/bin/bash
# Round 6: quarter-channel conv with the transform store and the staging arithmetic between the
# MFMAs of their groups (AZ_PART_MIX=1, the default build) against diag/libaz_mix0.so -- part-kernel
# bit-identity, then the 64- and 128-position steps interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "part_workgroup or output_channel_split" > gpurun_out/r06ak_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for r in 1 2 3; do
  for v in mix1 mix0; do
    L=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so; [ $v = mix0 ] && L=$GRAFT_REPO_ROOT/diag/libaz_mix0.so
    for b in 64 128; do
      AZ_LIB=$L timeout -k 10 120 python -u bench.py --train-child --train-steps 20 --train-batch $b > gpurun_out/r06ak_${v}_b${b}_r$r.json 2>&1 || { echo "$v $b failed"; exit 1; }
    done
  done
done
echo r06ak-ok
