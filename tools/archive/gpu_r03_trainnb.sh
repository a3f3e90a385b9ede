# round 3: training Winograd conv, boards per workgroup (base = one, the committed kernel; nb1 /
# nb2 = the multi-board kernel at one / two boards): training GPU tests on the in-tree build, then
# rocprof kernel stats of a few training steps per variant
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_trainnb_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_trainnb_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in base nb1 nb2 base nb2; do
  export AZ_LIB=$R/build_var/$v/libaz.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_trainnb_$v -o tr -- python3 $R/tools/train_prof.py 6 > $R/gpurun_out/r03_trainnb_$v.log 2>&1 || exit 5
  echo "== $v $(grep ms/step $R/gpurun_out/r03_trainnb_$v.log)"
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$R/gpurun_out/r03_trainnb_$v/tr_kernel_stats.csv')):
    if 'conv_wino_train' in r['Name']: print(r['Name'][:44], r['Calls'], r['AverageNs'])"
done
