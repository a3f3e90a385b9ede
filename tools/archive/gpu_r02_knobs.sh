# C3 f32 Winograd knob sweep (tools/tower_ab, 3 interleaved rounds, 2048 games x 32 sims x 1 move):
# patch-read step (TLOAD), read->transform distance (TSPLIT), second-wave stagger (TSTAG), B lookahead (LA)
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
DTYPE=f32 timeout -k 10 600 bash tools/ab_run.sh gpurun_out/knobs_c3.log 32 ${LIBS} || exit $?
grep best gpurun_out/knobs_c3.log
