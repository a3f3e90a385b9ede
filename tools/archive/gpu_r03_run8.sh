# round 3 (session 2) evidence on the current build: default bench, C2 bench, PMC passes of the C3
# tower (tools/pmc_run.sh), rocprof kernel stats of the C3 bench command
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_8.log 2>&1 || exit 2
tail -1 gpurun_out/r03_smoke_8.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_8.json 2> gpurun_out/r03_bench_8.err || exit 3
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_8.json')); r=d['roofline']; t=d['training']; print('C3', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['tower']['share_of_step'], d['games_per_hr_measured']['value'], t['ms_per_step'], t['frac'])"
timeout -k 10 300 python -u bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 --games-leg 0 > gpurun_out/r03_bench_c2_8.json 2> gpurun_out/r03_bench_c2_8.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_c2_8.json')); r=d['roofline']; print('C2', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['bf16_mode']['value'])"
timeout -k 10 240 bash tools/pmc_run.sh gpurun_out/r03_pmc_c3_8 2048 8 f32 || exit 5
python3 tools/pmc_summary.py gpurun_out/r03_pmc_c3_8 tower32w_kernel 32 > gpurun_out/r03_pmc_c3_8_summary.json
grep -E "l2_hit|traffic_bytes|mfma_busy|effective_clock|SQ_INSTS_MFMA\"|SQ_INSTS_VALU\"|lds_conflict" gpurun_out/r03_pmc_c3_8_summary.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_prof8 -o c3 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --train-steps 0 --games-leg 0 --bf16-steps 0 > $R/gpurun_out/r03_prof8_c3.json 2> $R/gpurun_out/r03_prof8_c3.err || exit 6
head -4 $R/gpurun_out/r03_prof8/c3_kernel_stats.csv | cut -c1-160
