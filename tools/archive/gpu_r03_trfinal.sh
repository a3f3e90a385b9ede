# round 3: phase stamps of the final build (C3 and C2 shapes), PMC passes of the C2 tower
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32'); A.random_weights(6, 64, seed=42).tofile('/tmp/w6x64.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/tr/libaz.so gpurun_out/r03_tower_trace_final_c3.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_final_c3.bin 20 > gpurun_out/r03_tower_trace_final_c3.txt; cat gpurun_out/r03_tower_trace_final_c3.txt
timeout -k 10 120 tools/tower_trace 256 64 6 64 /tmp/w6x64.f32 build_var/tr/libaz.so gpurun_out/r03_tower_trace_final_c2.bin || exit 3
python3 tools/tower_trace64.py gpurun_out/r03_tower_trace_final_c2.bin 6 > gpurun_out/r03_tower_trace_final_c2.txt; cat gpurun_out/r03_tower_trace_final_c2.txt
BLOCKS=6 FILTERS=64 timeout -k 10 240 bash tools/pmc_run.sh gpurun_out/r03_pmc_c2 256 64 f32 || exit 4
python3 tools/pmc_summary.py gpurun_out/r03_pmc_c2 k_sims32w 32 > gpurun_out/r03_pmc_c2_summary.json
grep -E "mfma_busy|l2_hit|SQ_INSTS_MFMA\"|effective_clock|wait_frac" gpurun_out/r03_pmc_c2_summary.json
