# round-2: Winograd f32 tower -- parity tests, then C3 A/B direct vs Winograd (PF 2 / 4)
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wino_net.log 2>&1
rc=$?; tail -3 gpurun_out/wino_net.log; [ $rc -ne 0 ] && exit $rc
DTYPE=f32 timeout -k 10 400 bash tools/ab_run.sh gpurun_out/ab_wino_c3.log 16 ${LIBS} || exit $?
cat gpurun_out/ab_wino_c3.log
