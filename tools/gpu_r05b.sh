set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05b_gputests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r05b_gputests.log; exit 1; }
tail -3 gpurun_out/r05b_gputests.log
timeout -k 10 300 python -u bench.py --train-child --train-steps 10 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank > gpurun_out/r05b_train.log 2>&1 && timeout -k 10 300 python -u bench.py --train-child --train-steps 10 --train-batch 512 --blocks 20 --filters 256 --train-mode sharded >> gpurun_out/r05b_train.log 2>&1
tail -4 gpurun_out/r05b_train.log
timeout -k 10 120 ./tools/select_chain_repro > gpurun_out/r05b_select_chain.log 2>&1; echo "repro rc $?" >> gpurun_out/r05b_select_chain.log
timeout -k 10 120 ./tools/wgrad_dbg > gpurun_out/r05b_wgrad_dbg.log 2>&1; echo "wgrad_dbg rc $?" >> gpurun_out/r05b_wgrad_dbg.log
tail -5 gpurun_out/r05b_select_chain.log gpurun_out/r05b_wgrad_dbg.log
