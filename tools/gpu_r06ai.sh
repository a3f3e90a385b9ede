#!/bin/bash
# Round 6: pricing the small-batch weight grad's load latency -- a build whose weight-grad loads all
# read board 0 (cache-hot, wrong results) against the real one, kernel stats at 64 positions
set -o pipefail
cd /tmp && export TMPDIR=/tmp
AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_hot.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ai_hot64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 4 64 > $GRAFT_REPO_ROOT/gpurun_out/r06ai_hot64.log 2>&1 || exit 1
AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_hot.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ai_hot512 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 4 > $GRAFT_REPO_ROOT/gpurun_out/r06ai_hot512.log 2>&1 || exit 1
echo r06ai-ok
