# round-2 GPU session 2: full GPU test suite, short bench, f32 tower PMC passes
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/gputests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err || exit $?
tail -c 600 gpurun_out/bench_short.json
timeout -k 10 200 bash tools/pmc_run.sh gpurun_out/pmc32 2048 8 f32 || exit $?
echo done
