#!/bin/bash
# Round 6: kernel stats of the 64-position step after the quarter convs' deep prefetch
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ah_prof64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 64 > $GRAFT_REPO_ROOT/gpurun_out/r06ah_prof64.log 2>&1 || exit 1
echo r06ah-ok
