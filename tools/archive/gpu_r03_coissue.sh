set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/mfma_coissue > gpurun_out/r03_mfma_coissue.log 2>&1; rc=$?
cat gpurun_out/r03_mfma_coissue.log; exit $rc
