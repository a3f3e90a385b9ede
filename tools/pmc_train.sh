#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over tools/train_prof.py:
# a few 20x256 training steps at B = 512.  Summarise per kernel with
#   python3 tools/pmc_summary.py <outdir> <kernel substring> 32
# Usage (GPU box, repo root): bash tools/pmc_train.sh <outdir> [steps]
set -e
R=$(pwd)
OUT=$R/$1
S=${2:-2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { name=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o $name -- python3 $R/tools/train_prof.py $S > $OUT/$name.log 2>&1; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES
run tcc TCC_HIT_sum TCC_MISS_sum
run cyc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES
