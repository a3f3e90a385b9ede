#!/bin/bash
# Round 6: the half-channel convs' weight-ring prefetch depth (AZ_PART_PF2 builds in diag/): halves vs
# one board at 192 / 256 positions per depth
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 4 8; do
  for b in 192 256; do
    AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_h$v.so timeout -k 10 300 python -u tools/train_ab.py $b 10 2 'h2:AZ_TRAIN_HALF=2' 'one:AZ_TRAIN_HALF=0' 'q4:AZ_TRAIN_HALF=4' > gpurun_out/r06ae_h${v}_b$b.txt 2>&1 || { echo "ab $v $b failed"; exit 1; }
  done
done
echo r06ae-ok
