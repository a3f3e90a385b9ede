# persistent per-game simulation kernel (k_sims32w): parity tests, then C2 bench with it off / on
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_configs.py -x -v --timeout 150 --timeout-method thread -k "persistent or c2_search or fused_step or synthetic" > gpurun_out/persist_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/persist_tests.log | tail -n 15; [ $rc -ne 0 ] && exit $rc
for p in 0 1; do
  AZ_PERSIST=$p timeout -k 10 300 python3 bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 > gpurun_out/bench_c2_persist$p.json 2> gpurun_out/bench_c2_persist$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_persist$p.json')); print('C2 persist=$p', d['value'], d['ms_per_step'], d['bf16_mode']['value'])"
done
