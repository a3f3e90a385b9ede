#!/bin/bash
# Round 6: PMC passes over the training step's kernels (tools/pmc_train.sh, 2 steps at 20x256, B = 512)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 bash tools/pmc_train.sh gpurun_out/r06_pmc_train 2 || { echo "pmc_train failed"; exit 1; }
for k in "conv_wino_train_kernel<false, 1, 1" "conv_wino_train_kernel<false, 2, 2" "conv_wino_train_kernel<true, 2, 2, 1" wino_wgrad_gemm_kernel; do
  n=$(echo "$k" | tr -dc 'a-z0-9_')
  python3 tools/pmc_summary.py gpurun_out/r06_pmc_train "$k" 32 > gpurun_out/r06_pmc_train_$n.json || { echo "summary $k failed"; exit 1; }
done
echo r06m-ok
