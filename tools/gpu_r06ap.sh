#!/bin/bash
# Round 6: the weight grad's split reduction (reduce_out) with the splits' loads batched 2 / 4 at a
# time (diag/libaz_rb{2,4}.so, AZ_RED_BATCH) against one at a time (default): kernel stats at 512
# and the 512-position step, interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp
for v in rb1 rb2 rb4; do
  L=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so; [ $v != rb1 ] && L=$GRAFT_REPO_ROOT/diag/libaz_$v.so
  AZ_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ap_$v -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 4 > $GRAFT_REPO_ROOT/gpurun_out/r06ap_$v.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in rb1 rb2 rb4; do
    L=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so; [ $v != rb1 ] && L=$GRAFT_REPO_ROOT/diag/libaz_$v.so
    AZ_LIB=$L timeout -k 10 150 python -u bench.py --train-child --train-steps 20 --train-batch 512 > gpurun_out/r06ap_${v}_r$r.json 2>&1 || { echo "$v failed"; exit 1; }
  done
done
echo r06ap-ok
