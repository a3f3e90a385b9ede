set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -k "half_workgroup or multi_split or winograd_training or grads_losses" > gpurun_out/r05l_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r05l_tests.log; exit 1; }
tail -3 gpurun_out/r05l_tests.log
T="python -u bench.py --train-child --train-steps 20 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank"
for r in 1 2; do
  for v in 1 0; do
    echo "half=$v $(AZ_TRAIN_HALF=$v timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05l_train.log || exit 1
  done
done
cat gpurun_out/r05l_train.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05l_prof -o p -- python -u tools/train_prof.py 6 > gpurun_out/r05l_prof.log 2>&1 || exit 1
echo done
