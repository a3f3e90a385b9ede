#!/bin/bash
# Round 6, closing check of the in-tree build: full -m gpu suite, smoke, default C3 bench (driver command).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r06v8_gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06v8_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06v8_bench_c3.json 2> gpurun_out/r06v8_bench_c3.err || { echo "bench failed"; exit 1; }
echo val8-ok
