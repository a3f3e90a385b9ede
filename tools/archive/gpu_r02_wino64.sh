# round-2: Winograd f32 tower for F = 64 / 128 -- parity tests, then the C2 f32 bench (Winograd vs direct)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_configs.py -x -v -k "f32 or winograd or 64" --timeout 200 --timeout-method thread > gpurun_out/wino64_tests.log 2>&1
rc=$?; tail -5 gpurun_out/wino64_tests.log; [ $rc -ne 0 ] && exit $rc
for wg in 1 0; do
  AZ_WINOGRAD=$wg timeout -k 10 200 python -u bench.py --games 256 --blocks 6 --filters 64 --steps 10 --warmup 2 --train-steps 0 --no-cpu-baseline > gpurun_out/c2_f32_w$wg.json 2> gpurun_out/c2_f32_w$wg.err || exit $?
  tail -1 gpurun_out/c2_f32_w$wg.json
done
