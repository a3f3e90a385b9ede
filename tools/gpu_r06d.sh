#!/bin/bash
# Round 6: sharded exchanges as gathers (rank-order sums), the end-of-board barrier of the
# persistent training convs removed: the training tests (bit-identity and sharded parity), an
# interleaved A/B of the step (AZ_TRAIN_ENDBAR=1 restores the barrier), the training legs of the
# bench (plain and sharded over a 1-rank RCCL communicator, exchange counts and times).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r06d_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 512 10 4 'nobar:AZ_TRAIN_ENDBAR=0' 'endbar:AZ_TRAIN_ENDBAR=1' > gpurun_out/r06d_ab_endbar.txt 2>&1 || { echo "ab failed"; exit 1; }
for m in per-rank sharded; do
  timeout -k 10 200 python -u bench.py --train-child --rank 0 --world 1 --device 0 --uid - --blocks 20 --filters 256 --train-steps 20 --train-batch 512 --train-mode $m > gpurun_out/r06d_train_$m.json 2>&1 || { echo "train leg $m failed"; exit 1; }
done
echo r06d-ok
