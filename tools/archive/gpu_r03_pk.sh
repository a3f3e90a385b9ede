# packed-f32 Winograd transforms + zero-padded ACT: the Winograd/persistent/training GPU tests, then C3 A/B vs base
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_train.py tests/test_gpu_search.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_pk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/r03_pk_tests.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_pk_c3.log 32 build_var/base/libaz.so build_var/pk/libaz.so || exit $?
grep best gpurun_out/r03_ab_pk_c3.log
