# round 3 (session 2): GPU suite, smoke, default (C3) bench with the instrumented profile pass moved
# out of the timed window, C2 bench (6x64, 256 games)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputests_7.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputests_7.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_7.log 2>&1 || exit 4
tail -1 gpurun_out/r03_smoke_7.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_7.json 2> gpurun_out/r03_bench_7.err || exit 5
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_7.json')); r=d['roofline']; t=d['training']; print('C3', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['tower']['share_of_step'], d['games_per_hr_measured']['value'], t['ms_per_step'], t['frac'])"
timeout -k 10 300 python -u bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 --games-leg 0 > gpurun_out/r03_bench_c2_7.json 2> gpurun_out/r03_bench_c2_7.err || exit 6
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_c2_7.json')); r=d['roofline']; print('C2', d['value'], d['ms_per_step'], r['frac'], r['avg_ms_per_launch'], d['bf16_mode']['value'])"
GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_c2pk.log 800 build_var/c2x/libaz.so alphazero-chess_amd/azchess/libaz.so || exit 7
grep best gpurun_out/r03_ab_c2pk.log
