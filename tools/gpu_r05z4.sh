set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05z4_tests.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/r05z4_tests.log; exit 1; }
tail -3 gpurun_out/r05z4_tests.log
