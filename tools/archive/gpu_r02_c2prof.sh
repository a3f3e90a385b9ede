# round-2: rocprofv3 kernel stats of the C2 bench command (f32 headline leg + bf16 leg)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c2prof -o c2 -- python3 $R/bench.py --games 256 --blocks 6 --filters 64 --steps 4 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/c2prof.json 2> $R/gpurun_out/c2prof.err || exit $?
tail -1 $R/gpurun_out/c2prof.json | cut -c1-300
f=$(find $R/gpurun_out/c2prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-6
