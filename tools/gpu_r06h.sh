#!/bin/bash
# Round 6: the weight grad's X operand by LDS-DMA (the point's distinct squares only): bit-identity
# tests, then interleaved A/Bs of the step at B = 512 and 64.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "round6 or multi_split or oracle or sharded_world1" > gpurun_out/r06h_train_tests.log 2>&1 || { echo "train tests failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 512 10 3 'glds:AZ_TRAIN_WGRAD_GLDS=1' 'regs:AZ_TRAIN_WGRAD_GLDS=0' > gpurun_out/r06h_ab_glds_b512.txt 2>&1 || { echo "ab 512 failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 64 10 3 'glds:AZ_TRAIN_WGRAD_GLDS=1' 'regs:AZ_TRAIN_WGRAD_GLDS=0' > gpurun_out/r06h_ab_glds_b64.txt 2>&1 || { echo "ab 64 failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06h_prof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 > $GRAFT_REPO_ROOT/gpurun_out/r06h_prof.log 2>&1 || exit 1
echo r06h-ok
