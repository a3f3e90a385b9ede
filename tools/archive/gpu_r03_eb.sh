# round 3: early B-fragment reads of the trailing waves across the chunk barrier (AZ_WINO_EARLYB):
# C3 A/B against the default build, then the GPU net/search tests on the variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_run.sh gpurun_out/r03_ab_eb_c3.log 32 alphazero-chess_amd/azchess/libaz.so build_var/eb/libaz.so alphazero-chess_amd/azchess/libaz.so build_var/eb/libaz.so || exit 3
grep move gpurun_out/r03_ab_eb_c3.log | cut -c1-160
cp build_var/eb/libaz.so alphazero-chess_amd/azchess/libaz.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_eb_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_eb_tests.log; exit $rc
