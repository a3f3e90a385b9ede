# round 3 (session 2): evidence on HEAD (Winograd wgrad + v_mov_b64 zeroing build): GPU suite,
# smoke, default bench, rocprof kernel stats, PMC passes
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputests_5.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputests_5.log | tail -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_5.log 2>&1 || exit 3
tail -1 gpurun_out/r03_smoke_5.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_5.json 2> gpurun_out/r03_bench_5.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_5.json')); r=d['roofline']; print('C3', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['games_per_hr_measured']['value'], d['training'])"
timeout -k 10 240 bash tools/pmc_run.sh gpurun_out/r03_pmc_c3_5 2048 8 f32 || exit 5
python3 tools/pmc_summary.py gpurun_out/r03_pmc_c3_5 tower32w_kernel 32 > gpurun_out/r03_pmc_c3_5_summary.json
grep -E "l2_hit|traffic_bytes|mfma_busy|effective_clock|SQ_INSTS_MFMA\"" gpurun_out/r03_pmc_c3_5_summary.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_prof5 -o c3 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --train-steps 0 --games-leg 0 --bf16-steps 0 > $R/gpurun_out/r03_prof5_c3.json 2> $R/gpurun_out/r03_prof5_c3.err || exit 6
head -4 $R/gpurun_out/r03_prof5/c3_kernel_stats.csv | cut -c1-160
