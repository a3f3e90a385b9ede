set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/grads_dump.py /tmp/g_new.npy 80 > gpurun_out/r05z3_dump.log 2>&1 || exit 1
AZ_LIB=$PWD/abvar/base/libaz.so timeout -k 10 200 python -u tools/grads_dump.py /tmp/g_base.npy 80 >> gpurun_out/r05z3_dump.log 2>&1 || exit 1
python -c "import numpy as np; a=np.load('/tmp/g_base.npy'); b=np.load('/tmp/g_new.npy'); print('bit-identical', np.array_equal(a,b), np.abs(a-b).max())"
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z3_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r05z3_tests.log; exit 1; }
tail -1 gpurun_out/r05z3_tests.log
T="python -u bench.py --train-child --train-steps 20 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank"
for r in 1 2 3; do
  echo "base $(AZ_LIB=$PWD/abvar/base/libaz.so timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05z3_train.log || exit 1
  echo "hp   $(timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05z3_train.log || exit 1
done
cat gpurun_out/r05z3_train.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05z3_prof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 > $GRAFT_REPO_ROOT/gpurun_out/r05z3_prof.log 2>&1 || exit 1
echo ok
