# round 3: next-chunk transform by the first wave of each SIMD pair after its last step (AZ_WINO_XTAIL):
# stamps, A/B vs base, GPU net/search tests on the variant
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/xtailtr/libaz.so gpurun_out/r03_tower_trace_xtail.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_xtail.bin 20 | tee gpurun_out/r03_tower_trace_xtail.txt
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab_wino_xtail_c3.log 32 build_var/base/libaz.so build_var/xtail/libaz.so build_var/noxf/libaz.so || exit 3
grep -E "best" gpurun_out/r03_ab_wino_xtail_c3.log
cp build_var/xtail/libaz.so alphazero-chess_amd/azchess/libaz.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_xtail_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_xtail_tests.log; exit $rc
