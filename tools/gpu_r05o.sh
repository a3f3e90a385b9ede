set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for h in 0 1; do
  AZ_TRAIN_HALF=$h timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $R/gpurun_out/r05o_h$h -o c -- python3 $R/tools/train_prof.py 2 > $R/gpurun_out/r05o_h$h.log 2>&1 || exit 1
done
echo ok
