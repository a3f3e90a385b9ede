# pk2 (v_mov_b64 accumulator zeroing, leaner patch addressing): Winograd GPU tests, then C3 and C2 A/B vs base / pk
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wino or persistent or headline or oracle or run_sims" > gpurun_out/r03_pk2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_pk2_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_pk2_c3.log 32 build_var/base/libaz.so build_var/pk/libaz.so build_var/pk2/libaz.so || exit $?
grep best gpurun_out/r03_ab_pk2_c3.log
GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_pk2_c2.log 200 build_var/base/libaz.so build_var/pk/libaz.so build_var/pk2/libaz.so || exit $?
grep best gpurun_out/r03_ab_pk2_c2.log
