# round 3: wino_wgrad_gemm_kernel staging depth (rows per LDS stage 16 / 32 / 64) and q-loop unroll
# (2 / 4): rocprof kernel stats of a few training steps per variant
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-base r64 u4 r64u4 r16 base r64}; do
  export AZ_LIB=$R/build_var/$v/libaz.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_wgtune_$v -o tr -- python3 $R/tools/train_prof.py 4 > $R/gpurun_out/r03_wgtune_$v.log 2>&1 || exit 5
  echo "== $v $(python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/r03_wgtune_$v/tr_kernel_stats.csv')):
    if 'wino_wgrad_gemm' in r['Name']: print(r['Calls'], r['AverageNs'])")"
done
