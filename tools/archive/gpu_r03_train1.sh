# round 3: the Winograd training step -- its GPU tests, then step time (direct vs Winograd) and rocprof stats
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_net.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_train_tests_1.log 2>&1
rc=$?; echo "train tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/r03_train_tests_1.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
AZ_TRAIN_WINOGRAD=0 timeout -k 10 120 python -u tools/train_prof.py 10 > gpurun_out/r03_train_direct.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/train_prof.py 10 > gpurun_out/r03_train_wino.log 2>&1 || exit 4
echo direct $(cat gpurun_out/r03_train_direct.log) wino $(cat gpurun_out/r03_train_wino.log)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_trainprof -o tr -- python3 $R/tools/train_prof.py 5 > $R/gpurun_out/r03_trainprof.log 2>&1 || exit 5
head -12 $R/gpurun_out/r03_trainprof/tr_kernel_stats.csv | cut -c1-150
