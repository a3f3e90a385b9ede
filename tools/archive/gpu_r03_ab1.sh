# A/B of the F=256 Winograd tower variants (tools/tower_ab: 2048 games x 32 sims, 3 interleaved rounds)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab1_c3.log 32 build_var/old/libaz.so build_var/dt_s1r4/libaz.so build_var/dt_s0r4/libaz.so build_var/dt_s2r4/libaz.so
rc=$?; grep best gpurun_out/r03_ab1_c3.log; exit $rc
