set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05d_gputests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r05d_gputests.log; exit 1; }
tail -2 gpurun_out/r05d_gputests.log
T="python -u bench.py --train-child --train-steps 20 --train-batch 512 --blocks 20 --filters 256"
for cfg in "1 1" "0 1" "1 0" "0 0" "1 1" "0 1"; do
  set -- $cfg
  echo "streams=$1 fuse=$2 $(AZ_TRAIN_STREAMS=$1 AZ_TRAIN_FUSE_BN=$2 timeout -k 10 300 $T --train-mode per-rank | tail -1)" >> gpurun_out/r05d_train.log || exit 1
done
cat gpurun_out/r05d_train.log
AZ_TRAIN_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05d_prof0 -o r05d -- python -u tools/train_prof.py 12 > gpurun_out/r05d_prof0.log 2>&1
AZ_TRAIN_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05d_prof1 -o r05d -- python -u tools/train_prof.py 12 > gpurun_out/r05d_prof1.log 2>&1
tail -1 gpurun_out/r05d_prof0.log gpurun_out/r05d_prof1.log
