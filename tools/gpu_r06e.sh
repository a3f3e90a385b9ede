#!/bin/bash
# Round 6: half-channel conv workgroups at small per-rank batches: bit-identity tests, then
# interleaved A/Bs of the step at B = 64 / 128 / 256 (auto = half when 2B <= 256).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "half or round6 or bn_staging or multi_split or sharded or oracle" > gpurun_out/r06e_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
for b in 64 128; do
  timeout -k 10 300 python -u tools/train_ab.py $b 10 3 'half:AZ_TRAIN_HALF=-1' 'one:AZ_TRAIN_HALF=0' > gpurun_out/r06e_ab_half_b$b.txt 2>&1 || { echo "ab b$b failed"; exit 1; }
done
timeout -k 10 300 python -u tools/train_ab.py 256 10 3 'half:AZ_TRAIN_HALF=1' 'one:AZ_TRAIN_HALF=0' > gpurun_out/r06e_ab_half_b256.txt 2>&1 || { echo "ab b256 failed"; exit 1; }
echo r06e-ok
