# one PMC pass (LDS bank conflicts, instruction counts) of the C3 f32 tower on the in-tree build
set -o pipefail
R=$(pwd)
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
OUT=$R/gpurun_out/pmcsq; mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('$OUT/w.f32')"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES --kernel-trace --output-format csv -d $OUT/sq -o sq -- $R/tools/pmc_driver 2048 8 1 20 256 $OUT/w.f32 f32 > $OUT/sq.log 2>&1 || exit $?
rm -f $OUT/w.f32
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcsq tower32w 32 | grep -E "LDS|conflict"
