# round 3: A/B of the no-chunk-barrier timing bound, then the full evidence set for the stripped
# build: GPU suite, smoke, default bench, rocprof kernel stats, PMC passes (incl. L2 hit/miss)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab2_nobar_c3.log 32 build_var/base/libaz.so build_var/nobar/libaz.so || exit $?
grep best gpurun_out/r03_ab2_nobar_c3.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputests_2.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputests_2.log | tail -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_2.log 2>&1 || exit 3
tail -1 gpurun_out/r03_smoke_2.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_2.json 2> gpurun_out/r03_bench_2.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_2.json')); r=d['roofline']; print('C3', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['games_per_hr_measured']['value'])"
timeout -k 10 240 bash tools/pmc_run.sh gpurun_out/r03_pmc_c3 2048 8 f32 || exit 5
python3 tools/pmc_summary.py gpurun_out/r03_pmc_c3 tower32w_kernel 32 > gpurun_out/r03_pmc_c3_summary.json
grep -E "l2_hit|traffic_bytes|mfma_busy|effective_clock|SQ_INSTS_MFMA\"" gpurun_out/r03_pmc_c3_summary.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_prof -o c3 -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --train-steps 0 --games-leg 0 --bf16-steps 0 > $R/gpurun_out/r03_prof_c3.json 2> $R/gpurun_out/r03_prof_c3.err || exit 6
head -4 $R/gpurun_out/r03_prof/c3_kernel_stats.csv | cut -c1-160
