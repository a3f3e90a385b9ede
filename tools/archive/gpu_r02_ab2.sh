# Winograd tower A/B (session 7): Winograd/direct parity tests on the default build, then
# tools/tower_ab over build_var/* (C3, 2048 games x 16 sims, 3 interleaved rounds)
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab2_net.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab2_net.log; [ $rc -ne 0 ] && exit $rc
DTYPE=f32 timeout -k 10 500 bash tools/ab_run.sh gpurun_out/ab2_c3.log 16 ${LIBS} || exit $?
grep best gpurun_out/ab2_c3.log
