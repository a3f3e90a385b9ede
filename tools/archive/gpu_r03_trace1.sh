# round 3: phase stamps of the f32 Winograd tower (AZ_TOWER_TRACE build), C3 shape
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/trace/libaz.so gpurun_out/r03_tower_trace.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace.bin 20 | tee gpurun_out/r03_tower_trace.txt
