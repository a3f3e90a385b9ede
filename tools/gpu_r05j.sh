set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "train_loop_sharded or full_loop" > gpurun_out/r05j_gputests.log 2>&1 || { tail -40 gpurun_out/r05j_gputests.log; exit 1; }
tail -4 gpurun_out/r05j_gputests.log
