# round 3: two boards per workgroup in the training Winograd conv: training GPU tests,
# step time, rocprof stats of the training step
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_train3_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_train3_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/train_prof.py 10 > gpurun_out/r03_train3_ms.log 2>&1 || exit 4
cat gpurun_out/r03_train3_ms.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_train3prof -o tr -- python3 $R/tools/train_prof.py 5 > $R/gpurun_out/r03_train3prof.log 2>&1 || exit 5
head -8 $R/gpurun_out/r03_train3prof/tr_kernel_stats.csv | cut -c1-150
