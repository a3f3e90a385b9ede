#!/bin/bash
# Round 6: the weight grad's output-channel split at the full batch (AZ_TRAIN_WGRAD_COSPLIT=512)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/train_ab.py 512 10 3 'cs:AZ_TRAIN_WGRAD_COSPLIT=512' 'one:AZ_TRAIN_WGRAD_COSPLIT=0' > gpurun_out/r06z_ab_b512.txt 2>&1 || { echo "ab failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
AZ_TRAIN_WGRAD_COSPLIT=512 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06z_prof512 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 4 > $GRAFT_REPO_ROOT/gpurun_out/r06z_prof512.log 2>&1 || exit 1
echo r06z2-ok
