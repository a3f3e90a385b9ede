# k_sims32w phase trace at C2 (one self-play move, 256 games x 800 sims, 6x64 f32) and the rocprof
# kernel stats of the C2 bench command with the persistent kernel
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
rm -f gpurun_out/sims_trace.bin
AZ_LIB=$R/build_var/strace/libaz.so AZ_SIMS_TRACE_FILE=$R/gpurun_out/sims_trace.bin timeout -k 10 200 python3 -c "
import sys, time; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A
net = A.AlphaZero(6, 64, weights=A.random_weights(6, 64, seed=42), dtype='f32')
sp = A.SelfPlay(net, games=256, sims=800, seed=5, cache_capacity=0); sp.reset()
sp.step(); A_t = time.time(); sp.step(); print('move %.1f ms' % ((time.time() - A_t) * 1e3))
" || exit $?
python3 tools/sims_trace.py gpurun_out/sims_trace.bin 256
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c2prof -o c2 -- python3 $R/bench.py --games 256 --blocks 6 --filters 64 --steps 4 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/c2prof.json 2> $R/gpurun_out/c2prof.err || exit $?
f=$(find $R/gpurun_out/c2prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-7
