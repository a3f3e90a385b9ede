# PMC passes of the f32 Winograd tower on the round's final build (TSPLIT=2): FETCH/WRITE/SQ/cycles,
# then the summary bench.py's roofline.traffic reads
set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 500 bash tools/pmc_run.sh gpurun_out/pmc_s9 2048 8 f32 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_s9 tower32w 32 > gpurun_out/pmc_s9_summary.json || exit $?
cat gpurun_out/pmc_s9_summary.json
