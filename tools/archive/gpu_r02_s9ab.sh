# C3 A/B: the session-7 build (2006575) vs the current build, f32 and bf16 towers, interleaved
# rounds on one box (tools/tower_ab: 2048 games x 32 sims x 1 move, engine HIP-event tower time)
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
DTYPE=f32 timeout -k 10 400 bash tools/ab_run.sh gpurun_out/s9ab_c3_f32.log 32 build_var/s7/libaz.so build_var/pq0/libaz.so || exit $?
grep best gpurun_out/s9ab_c3_f32.log
DTYPE=bf16 timeout -k 10 300 bash tools/ab_run.sh gpurun_out/s9ab_c3_bf16.log 32 build_var/s7/libaz.so build_var/pq0/libaz.so || exit $?
grep best gpurun_out/s9ab_c3_bf16.log
