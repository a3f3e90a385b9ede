# round-2: F = 64 Winograd (point halves) -- f32 parity tests, C2 A/B (XH 1 vs 2), coarse trace
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_configs.py -x -q -k "f32 or winograd or 64" --timeout 200 --timeout-method thread > gpurun_out/w64_tests.log 2>&1
rc=$?; tail -3 gpurun_out/w64_tests.log; [ $rc -ne 0 ] && exit $rc
DTYPES=f32 LIBS="build_var/xh1/libaz.so build_var/xh2/libaz.so" timeout -k 10 300 bash tools/gpu_r02_ab.sh w64xh || exit $?
AZ_TOWER_TRACE_FILE=gpurun_out/w64trace.bin DTYPE=f32 GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 200 bash tools/ab_run.sh gpurun_out/w64trace.log 64 build_var/wtrace/libaz.so || exit $?
python tools/wino_coarse.py gpurun_out/w64trace.bin 6
