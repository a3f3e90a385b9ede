set -o pipefail
cd $GRAFT_REPO_ROOT
AZ_LIB=abvar/trace/libaz.so timeout -k 10 300 python -u tools/train_trace.py 3 > gpurun_out/r05m_trace_half.txt 2>&1 || exit 1
AZ_TRAIN_HALF=0 AZ_LIB=abvar/trace/libaz.so timeout -k 10 300 python -u tools/train_trace.py 3 > gpurun_out/r05m_trace_one.txt 2>&1 || exit 1
tail -3 gpurun_out/r05m_trace_half.txt gpurun_out/r05m_trace_one.txt
AZ_LIB=$PWD/abvar/late/libaz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -k "half_workgroup" > gpurun_out/r05m_tests_late.log 2>&1 || { echo "late TESTS FAILED"; tail -30 gpurun_out/r05m_tests_late.log; exit 1; }
tail -1 gpurun_out/r05m_tests_late.log
T="python -u bench.py --train-child --train-steps 20 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank"
for r in 1 2; do
  echo "half $(timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05m_train.log || exit 1
  echo "late $(AZ_LIB=$PWD/abvar/late/libaz.so timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05m_train.log || exit 1
  echo "one  $(AZ_TRAIN_HALF=0 timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05m_train.log || exit 1
done
cat gpurun_out/r05m_train.log
