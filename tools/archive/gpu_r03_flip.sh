# round 3: SIMD-pair priority flips every K steps (AZ_WINO_FLIP=K): phase stamps at K=4, then A/B vs base
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/flip4tr/libaz.so gpurun_out/r03_tower_trace_flip4.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_flip4.bin 20 | tee gpurun_out/r03_tower_trace_flip4.txt
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab_wino_flip_c3.log 32 build_var/base/libaz.so build_var/flip2/libaz.so build_var/flip4/libaz.so build_var/flip8/libaz.so || exit 3
grep -E "round|best" gpurun_out/r03_ab_wino_flip_c3.log
