# round 3: phase stamps of timing-only tower variants (AZ_TOWER_TRACE builds): base, second wave of each
# SIMD pair without MFMAs (solo), and both with zero-record weight descriptors (no weight traffic)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')" || exit 1
for v in trace solo tracenw solonw; do
  timeout -k 10 120 tools/tower_trace 2048 8 20 256 /tmp/w20x256.f32 build_var/$v/libaz.so gpurun_out/r03_tower_trace_$v.bin || exit 2
  echo "== $v"; python3 tools/tower_trace.py gpurun_out/r03_tower_trace_$v.bin 20 | tee gpurun_out/r03_tower_trace_$v.txt
done
