# round 3: timing-only bounds of the training Winograd conv (AZ_TRAIN_NOIO: no row load / no row
# load or store) against the base build; rocprof kernel stats of a few training steps per variant
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in base noio1 noio2; do
  export AZ_LIB=$R/build_var/$v/libaz.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_trainio_$v -o tr -- python3 $R/tools/train_prof.py 4 > $R/gpurun_out/r03_trainio_$v.log 2>&1 || exit 5
  echo "== $v"; grep -E "conv_wino_train" $R/gpurun_out/r03_trainio_$v/tr_kernel_stats.csv | cut -d, -f1,3,4 | cut -c1-40,150-
done
