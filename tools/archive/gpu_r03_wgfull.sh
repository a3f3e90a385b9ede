# round 3: Winograd weight-grad GEMM with one 256x256 tile per (split, point) workgroup (wino_wgrad_gemm_kernel)
# vs the committed kernel (base): training GPU tests on the in-tree build, then rocprof kernel stats
# of a few training steps per variant
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_wgfull_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_wgfull_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in base full base full; do
  export AZ_LIB=$R/build_var/$v/libaz.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_wgfull_$v -o tr -- python3 $R/tools/train_prof.py 6 > $R/gpurun_out/r03_wgfull_$v.log 2>&1 || exit 5
  echo "== $v $(grep ms/step $R/gpurun_out/r03_wgfull_$v.log)"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$R/gpurun_out/r03_wgfull_$v/tr_kernel_stats.csv')))[:5]:
    print(r['Name'][:44], r['Calls'], r['AverageNs'], r['Percentage'])"
done
unset AZ_LIB; timeout -k 10 120 python -u $R/tools/train_prof.py 10 > $R/gpurun_out/r03_wgfull_ms.log 2>&1 || exit 4
cat $R/gpurun_out/r03_wgfull_ms.log
