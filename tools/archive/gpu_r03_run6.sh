# round 3 (session 2): tail transform + chunk-0 pre-transform + xres in registers (defaults):
# stamps, A/B against the previous build (build_var/base), GPU suite, smoke, default bench
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/tr/libaz.so gpurun_out/r03_tower_trace_run6.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_run6.bin 20 > gpurun_out/r03_tower_trace_run6.txt; head -7 gpurun_out/r03_tower_trace_run6.txt
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab_wino_run6_c3.log 32 build_var/head0/libaz.so build_var/base/libaz.so alphazero-chess_amd/azchess/libaz.so || exit 3
grep -E "best" gpurun_out/r03_ab_wino_run6_c3.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputests_6.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputests_6.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_6.log 2>&1 || exit 4
tail -1 gpurun_out/r03_smoke_6.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_6.json 2> gpurun_out/r03_bench_6.err || exit 5
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_6.json')); r=d['roofline']; t=d['training']; print('C3', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['games_per_hr_measured']['value'], t['ms_per_step'], t['frac'])"
