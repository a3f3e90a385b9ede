# round 3: the tower's inner step in isolation (tools/mfma_loads.hip), 1 and 2 waves per SIMD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/mfma_loads > gpurun_out/r03_mfma_loads.log 2>&1; rc=$?
cat gpurun_out/r03_mfma_loads.log; exit $rc
