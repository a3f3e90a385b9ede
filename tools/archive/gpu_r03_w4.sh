# round 3: 4 waves x 64 output channels per workgroup at F = 256 (one wave per SIMD, accumulators
# in AGPRs; prototype build build_var/w4): C3 A/B against the default build, then net tests on it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_run.sh gpurun_out/r03_ab_w4_c3.log 32 alphazero-chess_amd/azchess/libaz.so build_var/w4/libaz.so alphazero-chess_amd/azchess/libaz.so build_var/w4/libaz.so || exit 3
grep move gpurun_out/r03_ab_w4_c3.log | cut -c1-160
cp build_var/w4/libaz.so alphazero-chess_amd/azchess/libaz.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_w4_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_w4_tests.log; exit $rc
