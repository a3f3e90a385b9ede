#!/bin/bash
# Round-6 evidence: tools/gpu_final.sh (full -m gpu suite, smoke, C3 + C2 bench, tower PMC, rocprof of
# the C3 bench) + rocprof kernel stats of the training step at 512 and at 64 positions.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r06 || { echo "gpu_final rc $?"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06_trainprof -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 > $GRAFT_REPO_ROOT/gpurun_out/r06_trainprof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06_trainprof64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 64 > $GRAFT_REPO_ROOT/gpurun_out/r06_trainprof64.log 2>&1 || exit 1
echo final-ok
