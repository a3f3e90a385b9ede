# round 3: the leading waves' epilogue + chunk-0 pre-transform at issue priority (AZ_WINO_EPRIO=1/3):
# stamps at prio 1, A/B against the default build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/ep1tr/libaz.so gpurun_out/r03_tower_trace_ep1.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_ep1.bin 20 > gpurun_out/r03_tower_trace_ep1.txt; head -6 gpurun_out/r03_tower_trace_ep1.txt
timeout -k 10 500 bash tools/ab_run.sh gpurun_out/r03_ab_eprio_c3.log 32 alphazero-chess_amd/azchess/libaz.so build_var/ep1/libaz.so build_var/ep3/libaz.so alphazero-chess_amd/azchess/libaz.so build_var/ep1/libaz.so build_var/ep3/libaz.so || exit 3
grep move gpurun_out/r03_ab_eprio_c3.log | cut -c1-160
