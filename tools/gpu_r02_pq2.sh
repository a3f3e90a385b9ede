# C2 point quarters vs one point set: coarse per-block trace of each (AZ_WINO_TRACE builds) and
# the C2 bench line of each library (AZ_LIB), interleaved
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
for V in pq1t; do
  AZ_TOWER_TRACE_FILE=gpurun_out/tr_$V.bin DTYPE=f32 GAMES=256 BLOCKS=6 FILTERS=64 timeout -k 10 200 bash tools/ab_run.sh gpurun_out/tr_$V.log 64 build_var/$V/libaz.so || exit $?
  echo "== $V"; python3 tools/wino_coarse.py gpurun_out/tr_$V.bin 6 | head -11
done
for r in 1 2; do for V in pq0 pq1; do
  AZ_LIB=$R/build_var/$V/libaz.so timeout -k 10 300 python3 bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 --bf16-steps 0 > gpurun_out/bench_c2_$V.json 2> gpurun_out/bench_c2_$V.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_$V.json')); print('$V C2', d['value'], d['roofline']['avg_ms_per_launch'])"
done; done
