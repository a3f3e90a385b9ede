#!/bin/bash
# Round 6: the persistent training convs' weight-ring prefetch (AZ_TRAIN_PF / AZ_TRAIN_LA builds in
# diag/) at 512 positions, interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in base tpf4 tpf4la2; do
    lib=$GRAFT_REPO_ROOT/diag/libaz_$v.so
    [ $v = base ] && lib=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so
    AZ_LIB=$lib timeout -k 10 120 python -u bench.py --train-child --train-steps 20 > gpurun_out/r06ag_${v}_r$r.json 2>&1 || { echo "$v failed"; exit 1; }
  done
done
echo r06ag-ok
