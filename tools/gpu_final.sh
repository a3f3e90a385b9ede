#!/bin/bash
# GPU box, round-end evidence in one call: the full -m gpu suite, smoke(), the default C3 bench and
# the C2 bench (tools/gpu_validate.sh), then rocprofv3 kernel stats of the C3 bench command and the
# PMC passes over the headline tower (tools/pmc_run.sh).  Logs under gpurun_out/<tag>_*.
# Usage (repo root on the box): bash tools/gpu_final.sh <tag>
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/gpu_validate.sh $TAG || exit $?
timeout -k 10 240 bash tools/pmc_run.sh gpurun_out/${TAG}_pmc_tower32w 2048 8 f32 || exit 5
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_tower32w tower32w_kernel 32 > gpurun_out/${TAG}_pmc_tower32w_summary.json || exit 6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_c3prof -o c3 -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --train-steps 0 --games-leg 0 --bf16-steps 0 \
    > $R/gpurun_out/${TAG}_c3prof.json 2> $R/gpurun_out/${TAG}_c3prof.err || exit 7
