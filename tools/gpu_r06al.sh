#!/bin/bash
# Round 6: batched loads in the per-channel partial sums (part_sums / part_m2: bn_board_var,
# finalize_bnback, finalize_* and bn_local) against the previous source (diag/libaz_old.so):
# training GPU tests, then 512- and 64-position steps interleaved, then kernel stats at 512
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06al_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for r in 1 2 3; do
  for v in new old; do
    L=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so; [ $v = old ] && L=$GRAFT_REPO_ROOT/diag/libaz_old.so
    for b in 512 64; do
      AZ_LIB=$L timeout -k 10 150 python -u bench.py --train-child --train-steps 20 --train-batch $b > gpurun_out/r06al_${v}_b${b}_r$r.json 2>&1 || { echo "$v $b failed"; exit 1; }
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06al_prof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 8 > $GRAFT_REPO_ROOT/gpurun_out/r06al_prof.log 2>&1 || exit 1
echo r06al-ok
