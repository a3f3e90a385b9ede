#!/bin/bash
# Round 6: weight-ring prefetch depth of the quarter-channel convs (AZ_PART_PF builds in diag/):
# 64-position step per depth, interleaved twice; part-kernel bit-identity with the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "part_workgroup" > gpurun_out/r06ac_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for r in 1 2; do
  for pf in 2 4 8; do
    AZ_LIB=$GRAFT_REPO_ROOT/diag/libaz_pf$pf.so timeout -k 10 120 python -u bench.py --train-child --train-steps 20 --train-batch 64 > gpurun_out/r06ac_pf${pf}_r$r.json 2>&1 || { echo "pf $pf failed"; exit 1; }
  done
done
echo r06ac-ok
