# C2 (256 games, 6x64 f32) A/B of Winograd F=64 variants: parity of each variant library
# (tests/test_gpu_net.py + the persistent-kernel test), then tools/tower_ab
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
for L in ${LIBS}; do
  AZ_LIB=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py -x -q --timeout 200 --timeout-method thread -k "winograd or persistent or oracle" > gpurun_out/ab64_tests.log 2>&1
  rc=$?; echo "$L: $(tail -n 1 gpurun_out/ab64_tests.log)"; [ $rc -ne 0 ] && exit $rc
done
GAMES=256 BLOCKS=6 FILTERS=64 DTYPE=f32 timeout -k 10 500 bash tools/ab_run.sh gpurun_out/ab64_c2.log 64 ${LIBS} || exit $?
grep best gpurun_out/ab64_c2.log
