#!/bin/bash
# Round 6: rehearsal of the N > 1 bench path on a 1-GPU box (--same-device: every rank on device 0,
# RCCL training leg skipped) -- both the self-launch and the driver's torchrun form
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py --gpus 2 --same-device --steps 3 --warmup 1 --games-leg 0 --train-steps 3 > gpurun_out/r06y_bench_n2_self.json 2> gpurun_out/r06y_bench_n2_self.err || { echo "self-launch failed"; exit 1; }
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --same-device --steps 3 --warmup 1 --games-leg 0 --train-steps 3 > gpurun_out/r06y_bench_n2_torchrun.json 2> gpurun_out/r06y_bench_n2_torchrun.err || { echo "torchrun failed"; exit 1; }
echo r06y-ok
