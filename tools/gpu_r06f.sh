#!/bin/bash
# Round 6: where the step's time goes at 64 positions (a world-8 rank's shard): rocprof kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06f_prof64 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 6 64 > $GRAFT_REPO_ROOT/gpurun_out/r06f_prof64.log 2>&1 || exit 1
echo r06f-ok
