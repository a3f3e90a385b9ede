#!/bin/bash
# Round 6: the training step at small per-rank batches (the 512 / world shard of a sharded step):
# Winograd convs (one board per workgroup) against the implicit-GEMM direct convs, interleaved;
# then the default bench (headline, training legs with collective counts).
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in 64 128 256; do
  timeout -k 10 300 python -u tools/train_ab.py $b 10 3 'wino:AZ_TRAIN_WINOGRAD=1' 'direct:AZ_TRAIN_WINOGRAD=0' > gpurun_out/r06c_ab_wd_b$b.txt 2>&1 || { echo "ab b$b failed"; exit 1; }
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06c_bench_c3.json 2> gpurun_out/r06c_bench_c3.err || { echo "bench failed"; exit 1; }
echo r06c-ok
