#!/bin/bash
# Round 6: phase stamps of the part (quarter-channel) convs at 64 positions (trace build in diag/)
set -o pipefail
cd $GRAFT_REPO_ROOT
AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_trace.so timeout -k 10 300 python -u tools/train_trace.py 3 64 > gpurun_out/r06aj_trace64.txt 2>&1 || { echo "trace failed"; exit 1; }
echo r06aj-ok
