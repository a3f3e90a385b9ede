# re-entry check on the current tree: full GPU suite + the driver's default bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests_check.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_check.log | tail -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_check.json')); print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['executed_frac'], d['bf16_mode']['value'])"
