# round-2 evidence run: full GPU suite, driver bench command, rocprof kernel stats of a short bench,
# PMC passes of the f32 Winograd tower
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests_full.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_full.log | tail -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_full.json')); print(d['value'], d['roofline']['frac'], d['roofline']['executed_frac'], d['bf16_mode']['value'])"
timeout -k 10 200 bash tools/pmc_run.sh gpurun_out/pmcw 2048 8 f32 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || exit $?
head -4 $R/gpurun_out/prof_bench/bench_kernel_stats.csv | cut -c1-150
