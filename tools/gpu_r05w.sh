set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "bn_staging_matches" > gpurun_out/r05w_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r05w_tests.log; exit 1; }
tail -4 gpurun_out/r05w_tests.log
