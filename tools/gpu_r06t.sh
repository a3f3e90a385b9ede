#!/bin/bash
# Round 6: PMC of the one-wave-per-SIMD weight grad, full and without side jobs (diag build d1)
# (AZ_TRAIN_WSPREAD=4 selected the one-wave weight grad while it was opt-in; it is the default since, AZ_TRAIN_WGRAD4=0 the 8-wave kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export AZ_TRAIN_WSPREAD=4
timeout -k 10 400 bash tools/pmc_train.sh gpurun_out/r06t_pmc_w4 2 || { echo "pmc w4 failed"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r06t_pmc_w4 wino_wgrad_gemm4 32 > gpurun_out/r06t_pmc_w4.json || exit 1
AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_d1.so timeout -k 10 400 bash tools/pmc_train.sh gpurun_out/r06t_pmc_d1 2 || { echo "pmc d1 failed"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r06t_pmc_d1 wino_wgrad_gemm4 32 > gpurun_out/r06t_pmc_d1.json || exit 1
echo r06t-ok
