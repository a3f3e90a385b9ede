# C2: point-quarter Winograd F=64 conv (AZ_WINO64_PQ=1, conv_wino_pq) against the one-point-set
# kernel (PQ=0): bitwise comparison of net.forward + one self-play move, the F=64 parity tests on
# the PQ build, tower_ab move timing at C2 f32, then the C2 bench line of the in-tree build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
for V in pq0 pq1; do
  AZ_LIB=$R/build_var/$V/libaz.so timeout -k 10 200 python3 -u tools/wino_bitcheck.py dump gpurun_out/bit_$V.npz || exit $?
done
python3 tools/wino_bitcheck.py cmp gpurun_out/bit_pq0.npz gpurun_out/bit_pq1.npz
AZ_LIB=$R/build_var/pq1/libaz.so timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "winograd or persistent or oracle or c2" > gpurun_out/pq_tests.log 2>&1
rc=$?; echo "pq1 tests: $(tail -n 1 gpurun_out/pq_tests.log)"; [ $rc -ne 0 ] && exit $rc
GAMES=256 BLOCKS=6 FILTERS=64 DTYPE=f32 timeout -k 10 500 bash tools/ab_run.sh gpurun_out/pq_ab_c2.log 64 build_var/pq0/libaz.so build_var/pq1/libaz.so || exit $?
grep best gpurun_out/pq_ab_c2.log
timeout -k 10 300 python3 bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 > gpurun_out/bench_c2_pq.json 2> gpurun_out/bench_c2_pq.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_pq.json')); print('C2', d['value'], d['roofline']['executed_frac'], d['roofline']['avg_ms_per_launch'], d['bf16_mode']['value'])"
