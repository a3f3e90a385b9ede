#!/bin/bash
# GPU box: tests + benches + A/B (base vs new) + rocprof kernel trace of the default bench.
TAG=${1:-val}
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_validate.sh $TAG || exit 1
GAMES=256 BLOCKS=6 FILTERS=64 bash tools/ab_run.sh gpurun_out/${TAG}_ab_c2.log 800 build_var/base/libaz.so build_var/new/libaz.so || exit 1
bash tools/ab_run.sh gpurun_out/${TAG}_ab_c3.log 64 build_var/base/libaz.so build_var/new/libaz.so || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --cache 0 --no-cpu-baseline --train-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
