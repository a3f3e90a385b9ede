# round 3: dependent-chain MFMA order (AZ_WINO_CHAIN): phase stamps, then interleaved A/B vs the base build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/chaintr/libaz.so gpurun_out/r03_tower_trace_chain.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_chain.bin 20 | tee gpurun_out/r03_tower_trace_chain.txt
timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_wino_chain_c3.log 32 build_var/base/libaz.so build_var/chain/libaz.so || exit 3
grep -E "round|best" gpurun_out/r03_ab_wino_chain_c3.log
