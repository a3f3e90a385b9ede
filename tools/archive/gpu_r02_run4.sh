# round-2 GPU session 4: wave-parallel expansion -- search tests, then C2/C3 A/B serial vs wave
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_search.py tests/test_gpu_configs.py tests/test_gpu_arena.py -v --timeout 300 --timeout-method thread > gpurun_out/gputests4.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests4.log | tail -8
[ $rc -ne 0 ] && exit $rc
for dt in bf16 f32; do
DTYPE=$dt GAMES=256 BLOCKS=6 FILTERS=64 bash tools/ab_run.sh gpurun_out/ab_expand_c2_$dt.log 800 build_var/serial/libaz.so build_var/wave/libaz.so || exit $?
done
cat gpurun_out/ab_expand_c2_*.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o c2 -- python3 $R/bench.py --games 256 --blocks 6 --filters 64 --steps 4 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_c2.json 2> $R/gpurun_out/prof_c2.err || exit $?
head -8 $R/gpurun_out/prof_c2/c2_kernel_stats.csv | cut -c1-160
