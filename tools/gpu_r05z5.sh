set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 bash tools/pmc_train.sh gpurun_out/r05z5_pmc_train 2 || { echo "pmc_train failed"; exit 1; }
for k in "conv_wino_train_kernel<false, 1, 1>" "conv_wino_train_kernel<true, 2, 2>" "conv_wino_train_kernel<false, 2, 2>" "wino_wgrad_gemm_kernel" "wino_wgrad_reduce_out_kernel" "wino_weights_kernel" "wgrad_f32_kernel<9, 2>"; do
  n=$(echo "$k" | tr -cd 'a-z0-9_')
  python3 tools/pmc_summary.py gpurun_out/r05z5_pmc_train "$k" 32 > gpurun_out/r05z5_pmc_train_$n.json || exit 1
done
echo ok
