#!/bin/bash
# Round 6: the changed training paths first (one global replay buffer, merged exchanges, >1024
# positions), then the whole -m gpu suite and smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06a_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --deselect tests/test_gpu_train.py --deselect tests/test_gpu_dist_train.py > gpurun_out/r06a_gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a_smoke.log 2>&1 || exit 1
echo r06a-ok
