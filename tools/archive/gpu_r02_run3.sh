# round-2 GPU session 3: full GPU test suite, then rocprofv3 kernel stats of the bench command
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests.log | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || exit $?
find $R/gpurun_out/prof_bench -name "*stats*"
