# round 3: chunk-0 pre-transform by waves 0-3 at the conv boundary (AZ_WINO_PRE) on top of the tail
# transform default: stamps (base, pre), A/B, then the GPU net/search/train tests on the pre build
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
for v in basetr pretr; do
  timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/$v/libaz.so gpurun_out/r03_tower_trace_$v.bin || exit 2
  echo "== $v"; python3 tools/tower_trace.py gpurun_out/r03_tower_trace_$v.bin 20 > gpurun_out/r03_tower_trace_$v.txt; head -7 gpurun_out/r03_tower_trace_$v.txt
done
timeout -k 10 400 bash tools/ab_run.sh gpurun_out/r03_ab_wino_pre_c3.log 32 build_var/base/libaz.so build_var/pre/libaz.so || exit 3
grep -E "best" gpurun_out/r03_ab_wino_pre_c3.log
cp build_var/pre/libaz.so alphazero-chess_amd/azchess/libaz.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_search.py tests/test_gpu_train.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03_pre_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_pre_tests.log; exit $rc
