# round 3: no barrier after the last chunk of each Winograd conv (AZ_WINO_NOLASTBAR), flip-8 priority:
# phase stamps, A/B vs base, then the net / persistent-search GPU tests on the nlb build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/nlbtr/libaz.so gpurun_out/r03_tower_trace_nlb.bin || exit 2
python3 tools/tower_trace.py gpurun_out/r03_tower_trace_nlb.bin 20 | tee gpurun_out/r03_tower_trace_nlb.txt
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab_wino_nlb_c3.log 32 build_var/base/libaz.so build_var/nlb/libaz.so build_var/flip8/libaz.so build_var/flip8nlb/libaz.so || exit 3
grep -E "best" gpurun_out/r03_ab_wino_nlb_c3.log
cp build_var/nlb/libaz.so alphazero-chess_amd/azchess/libaz.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_nlb_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_nlb_tests.log; exit $rc
