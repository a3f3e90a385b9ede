set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/grads_dump.py /tmp/g_base.npy 80 > gpurun_out/r05r_dump.log 2>&1 || exit 1
for v in wred4 wtile; do
  AZ_LIB=$PWD/abvar/$v/libaz.so timeout -k 10 200 python -u tools/grads_dump.py /tmp/g_$v.npy 80 >> gpurun_out/r05r_dump.log 2>&1 || exit 1
  python -c "import numpy as np; a=np.load('/tmp/g_base.npy'); b=np.load('/tmp/g_$v.npy'); print('$v bit-identical', np.array_equal(a,b), np.abs(a-b).max())"
done
T="python -u bench.py --train-child --train-steps 20 --train-batch 512 --blocks 20 --filters 256 --train-mode per-rank"
for r in 1 2 3; do
  echo "base  $(timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05r_train.log || exit 1
  for v in wred4 wtile; do
    echo "$v $(AZ_LIB=$PWD/abvar/$v/libaz.so timeout -k 10 300 $T | tail -1)" >> gpurun_out/r05r_train.log || exit 1
  done
done
cat gpurun_out/r05r_train.log
cd /tmp && export TMPDIR=/tmp
for v in wred4 wtile; do
AZ_LIB=$GRAFT_REPO_ROOT/abvar/$v/libaz.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05r_prof_$v -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 > $GRAFT_REPO_ROOT/gpurun_out/r05r_prof.log 2>&1 || exit 1
done
echo ok
