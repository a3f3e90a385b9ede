#!/bin/bash
# Round 6: the one-wave-per-SIMD weight grad (AZ_TRAIN_WSPREAD=4): bit-identity, A/B, kernel stats
# (AZ_TRAIN_WSPREAD=4 selected the one-wave weight grad while it was opt-in; it is the default since, AZ_TRAIN_WGRAD4=0 the 8-wave kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread -k "load_placement" > gpurun_out/r06s_tests.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 512 10 3 's1:AZ_TRAIN_WSPREAD=1' 'w4:AZ_TRAIN_WSPREAD=4' > gpurun_out/r06s_ab_b512.txt 2>&1 || { echo "ab failed"; exit 1; }
timeout -k 10 300 python -u tools/train_ab.py 64 10 3 's1:AZ_TRAIN_WSPREAD=1' 'w4:AZ_TRAIN_WSPREAD=4' > gpurun_out/r06s_ab_b64.txt 2>&1 || { echo "ab failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
AZ_TRAIN_WSPREAD=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06s_prof4 -o t -- python3 $GRAFT_REPO_ROOT/tools/train_prof.py 4 > $GRAFT_REPO_ROOT/gpurun_out/r06s_prof4.log 2>&1 || exit 1
echo r06s-ok
