# timing bounds of the C3 Winograd tower: no weight traffic / one conv's weights for all convs / no chunk barriers
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab3_bounds_c3.log 32 build_var/base/libaz.so build_var/nowt/libaz.so build_var/samew/libaz.so build_var/nobar/libaz.so || exit $?
grep best gpurun_out/r03_ab3_bounds_c3.log
