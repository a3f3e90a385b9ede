#!/bin/bash
# Round 6: finalize kernels as 16-channel workgroups (coalesced partial rows, LDS butterfly) plus the
# batched partial-sum loads, against the previous source (diag/libaz_old.so): training GPU tests, 512-
# and 64-position steps interleaved four times, then kernel stats at 64 and 512
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06ao_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for r in 1 2 3 4; do
  for v in new old; do
    L=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so; [ $v = old ] && L=$GRAFT_REPO_ROOT/diag/libaz_old.so
    for b in 512 64; do
      AZ_LIB=$L timeout -k 10 150 python -u bench.py --train-child --train-steps 20 --train-batch $b > gpurun_out/r06ao_${v}_b${b}_r$r.json 2>&1 || { echo "$v $b failed"; exit 1; }
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ao_prof64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 8 64 > $GRAFT_REPO_ROOT/gpurun_out/r06ao_prof64.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ao_prof512 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 8 > $GRAFT_REPO_ROOT/gpurun_out/r06ao_prof512.log 2>&1 || exit 1
echo r06ao-ok
