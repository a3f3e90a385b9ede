# round 3: F = 64 register (DPP) transform of the next conv's input: GPU net/search/config tests,
# C2 stamps, C2 A/B (persistent per-game kernel) against the session-start build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py tests/test_gpu_configs.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_c2x_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_c2x_tests.log; [ $rc -ne 0 ] && exit $rc
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(6, 64, seed=42).tofile('/tmp/w6x64.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 256 64 6 64 /tmp/w6x64.f32 build_var/tr/libaz.so gpurun_out/r03_tower_trace_c2x.bin || exit 2
python3 tools/tower_trace64.py gpurun_out/r03_tower_trace_c2x.bin 6 | tee gpurun_out/r03_tower_trace_c2x.txt
GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_c2x.log 800 build_var/head0/libaz.so alphazero-chess_amd/azchess/libaz.so || exit 3
cut -c1-160 gpurun_out/r03_ab_c2x.log
