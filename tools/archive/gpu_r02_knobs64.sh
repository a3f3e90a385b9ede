# C2 f32 (256 games x 800 sims, 6x64) Winograd F=64 knob sweep: tools/tower_ab move timing, 3 interleaved rounds
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
GAMES=256 BLOCKS=6 FILTERS=64 DTYPE=f32 timeout -k 10 600 bash tools/ab_run.sh gpurun_out/knobs_c2.log 64 ${LIBS} || exit $?
grep best gpurun_out/knobs_c2.log
