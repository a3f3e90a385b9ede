# round-2 final evidence: full GPU suite, the driver bench command (C3), a C2 bench line, rocprof
# kernel stats of the C3 and C2 bench commands, PMC passes of the f32 Winograd tower
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests_final.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_final.log | tail -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['executed_frac'], d['bf16_mode']['value'])"
timeout -k 10 300 python3 bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 > gpurun_out/bench_c2_final.json 2> gpurun_out/bench_c2_final.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_final.json')); print('C2', d['value'], d['roofline']['frac'], d['bf16_mode']['value'])"
timeout -k 10 200 bash tools/pmc_run.sh gpurun_out/pmcw 2048 8 f32 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o c3 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_final_c3.json 2> $R/gpurun_out/prof_final_c3.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o c2 -- python3 $R/bench.py --games 256 --blocks 6 --filters 64 --steps 4 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_final_c2.json 2> $R/gpurun_out/prof_final_c2.err || exit $?
head -4 $R/gpurun_out/prof_final/c3_kernel_stats.csv | cut -c1-150
head -6 $R/gpurun_out/prof_final/c2_kernel_stats.csv | cut -c1-150
