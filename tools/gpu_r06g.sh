#!/bin/bash
# Round 6: quarter-channel conv workgroups (4 per board) for the 64-position shard: bit-identity
# tests, then interleaved A/Bs at B = 64 and 128 (4 / 2 / 1 workgroups per board).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "part or round6 or bn_staging or sharded_world1" > gpurun_out/r06g_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
for b in 64 128; do
  timeout -k 10 300 python -u tools/train_ab.py $b 10 3 'q4:AZ_TRAIN_HALF=4' 'h2:AZ_TRAIN_HALF=2' 'one:AZ_TRAIN_HALF=0' > gpurun_out/r06g_ab_parts_b$b.txt 2>&1 || { echo "ab b$b failed"; exit 1; }
done
echo r06g-ok
