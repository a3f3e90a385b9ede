# round 3 (session 2) final evidence on HEAD: GPU suite, smoke, default bench, rocprof stats of the
# C2 bench command
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputests_final.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputests_final.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_final.log 2>&1 || exit 2
tail -1 gpurun_out/r03_smoke_final.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_final.json 2> gpurun_out/r03_bench_final.err || exit 3
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_final.json')); r=d['roofline']; t=d['training']; print('C3', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['tower']['share_of_step'], d['games_per_hr_measured']['value'], t['ms_per_step'], t['frac'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_profc2 -o c2 -- python3 $R/bench.py --games 256 --blocks 6 --filters 64 --steps 10 --warmup 2 --no-cpu-baseline --train-steps 0 --games-leg 0 --bf16-steps 0 > $R/gpurun_out/r03_profc2.json 2> $R/gpurun_out/r03_profc2.err || exit 4
head -6 $R/gpurun_out/r03_profc2/c2_kernel_stats.csv | cut -c1-150
