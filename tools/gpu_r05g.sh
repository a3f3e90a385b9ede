set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "sharded" > gpurun_out/r05g_gputests.log 2>&1 || { tail -40 gpurun_out/r05g_gputests.log; exit 1; }
tail -6 gpurun_out/r05g_gputests.log
