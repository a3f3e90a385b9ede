set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1
python3 -c "import sys; sys.path.insert(0,'alphazero-chess_amd'); import azchess as A; A.random_weights(20,256,seed=42).tofile('/tmp/w.f32')"
timeout -k 10 300 python -u -m pytest tests/test_gpu_net.py -x -v --timeout 120 --timeout-method thread > gpurun_out/net.log 2>&1
rc=$?; echo "net tests rc=$rc"; tail -3 gpurun_out/net.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 tools/pmc_driver 2048 8 1 20 256 /tmp/w.f32 f32 > gpurun_out/f32drv.log 2>&1 || exit $?
cat gpurun_out/f32drv.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_f32 -o f32 -- $R/tools/pmc_driver 2048 8 1 20 256 /tmp/w.f32 f32 > $R/gpurun_out/prof_f32.log 2>&1 || exit $?
find $R/gpurun_out/prof_f32 -name "*stats*"
