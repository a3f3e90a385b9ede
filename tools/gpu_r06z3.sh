#!/bin/bash
# Round 6: the weight grad's output channels over four workgroups (AZ_TRAIN_WGRAD_COSPLIT4) vs two
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "channel_split" > gpurun_out/r06z3_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for b in 64 128; do
  timeout -k 10 300 python -u tools/train_ab.py $b 10 3 "c4:AZ_TRAIN_WGRAD_COSPLIT4=$b" 'c2:AZ_TRAIN_WGRAD_COSPLIT4=0' > gpurun_out/r06z3_ab_b$b.txt 2>&1 || { echo "ab $b failed"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
AZ_TRAIN_WGRAD_COSPLIT4=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06z3_prof64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 4 64 > $GRAFT_REPO_ROOT/gpurun_out/r06z3_prof64.log 2>&1 || exit 1
echo r06z3-ok
