#!/bin/bash
# Round 6: quarter-channel convs with the deeper weight-ring prefetch: depth 16 vs 8 at 64 positions,
# and quarters (AZ_TRAIN_HALF=4) vs halves (2) vs one board (0) at 128 / 192 / 256 positions
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for pf in 8 16; do
    AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_pf$pf.so timeout -k 10 120 python -u bench.py --train-child --train-steps 20 --train-batch 64 > gpurun_out/r06ad_pf${pf}_r$r.json 2>&1 || { echo "pf $pf failed"; exit 1; }
  done
done
for b in 128 192 256; do
  timeout -k 10 300 python -u tools/train_ab.py $b 10 2 'q4:AZ_TRAIN_HALF=4' 'h2:AZ_TRAIN_HALF=2' 'one:AZ_TRAIN_HALF=0' > gpurun_out/r06ad_ab_parts_b$b.txt 2>&1 || { echo "ab $b failed"; exit 1; }
done
echo r06ad-ok
