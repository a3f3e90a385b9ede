#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over tools/pmc_driver:
# one self-play move of G games x S sims with the BLOCKS x FILTERS net (default 20x256) through the C-ABI, no Python in the
# profiled process.  Usage (GPU box, repo root): bash tools/pmc_run.sh <outdir> [games] [sims] [f32|bf16]
set -e
R=$(pwd)
OUT=$R/$1
G=${2:-2048}
S=${3:-16}
DT=${4:-f32}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(${BLOCKS:-20}, ${FILTERS:-256}, seed=42).tofile('$OUT/w.f32')"
cd /tmp && export TMPDIR=/tmp
CMD="$R/tools/pmc_driver $G $S 1 ${BLOCKS:-20} ${FILTERS:-256} $OUT/w.f32 $DT"
timeout -k 10 60 $CMD > $OUT/plain.log 2>&1
run() { name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o $name -- $CMD > $OUT/$name.log 2>&1; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES
run tcc TCC_HIT_sum TCC_MISS_sum
run cyc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES
rm -f $OUT/w.f32
