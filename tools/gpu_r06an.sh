#!/bin/bash
# Round 6: batched loads in the per-channel partial sums and the generic split reduce (weight grad's
# reduce_out unchanged) against the previous source (diag/libaz_old.so): 512- and 64-position steps
# interleaved four times, then kernel stats at 64
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  for v in new old; do
    L=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so; [ $v = old ] && L=$GRAFT_REPO_ROOT/diag/libaz_old.so
    for b in 512 64; do
      AZ_LIB=$L timeout -k 10 150 python -u bench.py --train-child --train-steps 20 --train-batch $b > gpurun_out/r06an_${v}_b${b}_r$r.json 2>&1 || { echo "$v $b failed"; exit 1; }
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06an_prof64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 8 64 > $GRAFT_REPO_ROOT/gpurun_out/r06an_prof64.log 2>&1 || exit 1
echo r06an-ok
