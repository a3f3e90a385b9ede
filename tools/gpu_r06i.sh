#!/bin/bash
# Round 6: where quarter-channel conv workgroups stop paying: B = 192 and 256 (q4 vs one board).
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 192 256; do
  timeout -k 10 300 python -u tools/train_ab.py $b 10 3 'q4:AZ_TRAIN_HALF=4' 'one:AZ_TRAIN_HALF=0' > gpurun_out/r06i_ab_parts_b$b.txt 2>&1 || { echo "ab b$b failed"; exit 1; }
done
echo r06i-ok
