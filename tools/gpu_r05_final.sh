#!/bin/bash
# Round-5 evidence: tools/gpu_final.sh (full -m gpu suite, smoke, C3 + C2 bench, tower PMC, rocprof of
# the C3 bench) + the training kernels' PMC passes and kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r05 || { echo "gpu_final rc $?"; exit 1; }
timeout -k 10 700 bash tools/pmc_train.sh gpurun_out/r05_pmc_train 2 || { echo "pmc_train failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05_trainprof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 12 > $GRAFT_REPO_ROOT/gpurun_out/r05_trainprof.log 2>&1 || exit 1
echo final-ok
