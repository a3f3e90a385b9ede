#!/bin/bash
# Round 6: default bench with the C2 steady-state leg
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u bench.py > gpurun_out/r06aa_bench.json 2> gpurun_out/r06aa_bench.err || { echo "bench failed"; exit 1; }
echo r06aa-ok
