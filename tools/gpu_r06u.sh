#!/bin/bash
# Round 6: the one-wave-per-SIMD weight grad as the default -- training GPU tests, A/B against the
# 8-wave kernel at B = 512 / 64, kernel stats, the bench's training legs
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06u_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 512 10 3 'w4:AZ_TRAIN_WGRAD4=1' 'w8:AZ_TRAIN_WGRAD4=0' > gpurun_out/r06u_ab_b512.txt 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 64 10 3 'w4:AZ_TRAIN_WGRAD4=1' 'w8:AZ_TRAIN_WGRAD4=0' > gpurun_out/r06u_ab_b64.txt 2>&1 || { echo "ab failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06u_prof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 > $GRAFT_REPO_ROOT/gpurun_out/r06u_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --train-child --train-steps 20 > gpurun_out/r06u_train_child.txt 2>&1 && timeout -k 10 300 python -u bench.py --train-child --train-steps 20 --train-mode sharded >> gpurun_out/r06u_train_child.txt 2>&1 || { echo "train child failed"; exit 1; }
echo r06u-ok
