# round-2 close: smoke() and the driver's default bench command on the final HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_head.log 2>&1 || { tail -20 gpurun_out/smoke_head.log; exit 1; }
tail -1 gpurun_out/smoke_head.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_c3_head.json 2> gpurun_out/bench_c3_head.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c3_head.json')); r=d['roofline']; print('C3', d['value'], r['avg_ms_per_launch'], r['executed_frac'], r['traffic'], d['bf16_mode']['value'], d['cpu_baseline']['value'])"
