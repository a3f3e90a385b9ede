# round 3: the next conv's chunk-0 pre-transform split over all 8 waves (each its own item, the
# trailing waves after their epilogue) vs on the 4 leading waves (base), C3 tower A/B; net tests
# on the split build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_run.sh gpurun_out/r03_ab_presplit_c3.log 32 build_var/base/libaz.so build_var/split/libaz.so build_var/base/libaz.so build_var/split/libaz.so || exit 3
cut -c1-150 gpurun_out/r03_ab_presplit_c3.log
export AZ_LIB=$R/build_var/split/libaz.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_presplit_net.log 2>&1
rc=$?; tail -2 gpurun_out/r03_presplit_net.log; exit $rc
