set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in wg_mid wg_end; do
  AZ_LIB=$PWD/abvar/$v/libaz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -k "multi_split or winograd_training or grads_losses" > gpurun_out/r05h_tests_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 gpurun_out/r05h_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r05h_tests_$v.log)"
done
T="python -u bench.py --train-child --train-steps 20 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank"
for r in 1 2; do
  for v in wg_base wg_single wg_mid wg_end; do
    echo "$v $(AZ_LIB=$PWD/abvar/$v/libaz.so timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05h_train.log || exit 1
  done
done
cat gpurun_out/r05h_train.log
for v in wg_base wg_mid wg_end; do
  AZ_LIB=$PWD/abvar/$v/libaz.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05h_prof_$v -o p -- python -u tools/train_prof.py 6 > gpurun_out/r05h_prof_$v.log 2>&1 || exit 1
done
echo done
