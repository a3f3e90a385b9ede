# round 3: packed input conv + heads with their biases / node record preloaded: full GPU suite, C2
# stamps, C2 and C3 A/B against the previous commit (3cd6311)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_heads_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_heads_tests.log; [ $rc -ne 0 ] && exit $rc
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(6, 64, seed=42).tofile('/tmp/w6x64.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 256 64 6 64 /tmp/w6x64.f32 build_var/tr/libaz.so gpurun_out/r03_tower_trace_c2hd.bin || exit 2
python3 tools/tower_trace64.py gpurun_out/r03_tower_trace_c2hd.bin 6 | tee gpurun_out/r03_tower_trace_c2hd.txt
GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_heads_c2.log 800 build_var/prev/libaz.so alphazero-chess_amd/azchess/libaz.so || exit 3
grep move gpurun_out/r03_ab_heads_c2.log | cut -c1-160
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab_heads_c3.log 32 build_var/prev/libaz.so alphazero-chess_amd/azchess/libaz.so || exit 4
grep move gpurun_out/r03_ab_heads_c3.log | cut -c1-160
