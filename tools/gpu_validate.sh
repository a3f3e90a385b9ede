#!/bin/bash
# GPU box: full -m gpu suite, smoke(), default C3 bench and the C2 bench; logs under gpurun_out/<tag>_*.
TAG=${1:-val}
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || exit 1
timeout -k 10 200 python -u bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || exit 1
