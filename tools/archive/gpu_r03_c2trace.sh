# round 3: phase stamps of the C2 tower (6x64 f32 Winograd, persistent per-game kernel, 256 games)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(6, 64, seed=42).tofile('/tmp/w6x64.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 256 64 6 64 /tmp/w6x64.f32 build_var/tr/libaz.so gpurun_out/r03_tower_trace_c2.bin || exit 2
python3 tools/tower_trace64.py gpurun_out/r03_tower_trace_c2.bin 6 | tee gpurun_out/r03_tower_trace_c2.txt
