# round 3: heads with the value-FC weights requested after the 1x1 conv's MFMAs (AZ_HEADS_LATEWQ):
# C2 and C3 A/B against the default build, then net/search tests on the variant
set -o pipefail
mkdir -p gpurun_out
GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 300 bash tools/ab_run.sh gpurun_out/r03_ab_lwq_c2.log 800 alphazero-chess_amd/azchess/libaz.so build_var/lwq/libaz.so alphazero-chess_amd/azchess/libaz.so build_var/lwq/libaz.so || exit 2
grep move gpurun_out/r03_ab_lwq_c2.log | cut -c1-160
timeout -k 10 500 bash tools/ab_run.sh gpurun_out/r03_ab_lwq_c3.log 32 alphazero-chess_amd/azchess/libaz.so build_var/lwq/libaz.so || exit 3
grep move gpurun_out/r03_ab_lwq_c3.log | cut -c1-160
cp build_var/lwq/libaz.so alphazero-chess_amd/azchess/libaz.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_lwq_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_lwq_tests.log; exit $rc
