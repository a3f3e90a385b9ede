# round 3, first GPU call: full GPU suite (new: callback evaluator, run_sims chunks, C5 at 20x256,
# the 2-rank bench on one GPU), the f32 Winograd smoke, and the default bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputests_1.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputests_1.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_1.log 2>&1 || { tail -20 gpurun_out/r03_smoke_1.log; exit 3; }
tail -1 gpurun_out/r03_smoke_1.log
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_1.json 2> gpurun_out/r03_bench_1.err || { tail -20 gpurun_out/r03_bench_1.err; exit 4; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_1.json')); r=d['roofline']; print('C3', d['value'], d['ms_per_step'], d['config']['sims_per_step'], r['frac'], r['algorithmic_tflops'], d['games_per_hr_measured'])"
