#!/bin/bash
# Round 6: training tests (ORC bit-identity, adaptive weight-grad splits), interleaved A/Bs of the
# training step (ORC on / off at B = 512; split size at B = 64, the per-rank shard of a world-8
# sharded step), rocprof kernel stats of 6 training steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06b_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 512 10 3 'orc:AZ_TRAIN_ORC=1' 'noorc:AZ_TRAIN_ORC=0' > gpurun_out/r06b_ab_orc.txt 2>&1 || { echo "ab orc failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 64 10 3 'adaptive:AZ_TRAIN_WGRAD_ROWS=0' 'rows512:AZ_TRAIN_WGRAD_ROWS=512' > gpurun_out/r06b_ab_b64.txt 2>&1 || { echo "ab b64 failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06b_prof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 > $GRAFT_REPO_ROOT/gpurun_out/r06b_prof.log 2>&1 || exit 1
echo r06b-ok
