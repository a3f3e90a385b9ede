#!/bin/bash
# Round 6: C2 (6x64) Winograd weight-ring prefetch depth (AZ_WINO64_PF builds in diag/): C2 steady state
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in 2 4 8; do
    lib=$GRAFT_REPO_ROOT/diag/libaz_w64pf$v.so
    [ $v = 2 ] && lib=$GRAFT_REPO_ROOT/alphazero-chess_amd/azchess/libaz.so
    AZ_LIB=$lib timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --bf16-steps 0 --games-leg 0 --train-steps 0 --no-cpu-baseline --c2-steps 20 > gpurun_out/r06af_pf${v}_r$r.json 2>&1 || { echo "pf $v failed"; exit 1; }
  done
done
echo r06af-ok
