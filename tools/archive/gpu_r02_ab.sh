# GPU box: A/B of build_var/old vs build_var/new at C2 (bf16, f32) -- tools/tower_ab through the C-ABI
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
TAG=${1:-ab}
for dt in ${DTYPES:-bf16 f32}; do
DTYPE=$dt GAMES=256 BLOCKS=6 FILTERS=64 bash tools/ab_run.sh gpurun_out/${TAG}_c2_$dt.log 800 ${LIBS:-build_var/old/libaz.so build_var/new/libaz.so} || exit $?
grep best gpurun_out/${TAG}_c2_$dt.log; grep "round 2" gpurun_out/${TAG}_c2_$dt.log
done
