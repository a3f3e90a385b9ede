set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05a_gputests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r05a_gputests.log; exit 1; }
tail -3 gpurun_out/r05a_gputests.log
timeout -k 10 300 python -u bench.py --train-child --train-steps 10 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank > gpurun_out/r05a_train.log 2>&1 && timeout -k 10 300 python -u bench.py --train-child --train-steps 10 --train-batch 512 --blocks 20 --filters 256 --train-mode sharded >> gpurun_out/r05a_train.log 2>&1
cat gpurun_out/r05a_train.log | tail -4
