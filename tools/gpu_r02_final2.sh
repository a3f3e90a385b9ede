# round-2 final evidence (session 7 build): full GPU suite, the driver bench command (C3), a C2
# bench line, the k_sims32w phase trace at C2, PMC passes of the f32 Winograd tower, rocprof kernel
# stats of the C3 and C2 bench commands
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests_final2.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests_final2.log | tail -n 5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/bench_final2.json 2> gpurun_out/bench_final2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_final2.json')); print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['executed_frac'], d['bf16_mode']['value'], d['training'].get('ms_per_step'))"
timeout -k 10 300 python3 bench.py --games 256 --blocks 6 --filters 64 --no-cpu-baseline --train-steps 0 > gpurun_out/bench_c2_final2.json 2> gpurun_out/bench_c2_final2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_c2_final2.json')); print('C2', d['value'], d['roofline']['executed_frac'], d['bf16_mode']['value'], d['sim_kernels'][:20])"
rm -f gpurun_out/sims_trace.bin
AZ_LIB=$R/build_var/strace/libaz.so AZ_SIMS_TRACE_FILE=$R/gpurun_out/sims_trace.bin timeout -k 10 200 python3 -c "
import sys, time; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A
net = A.AlphaZero(6, 64, weights=A.random_weights(6, 64, seed=42), dtype='f32')
sp = A.SelfPlay(net, games=256, sims=800, seed=5, cache_capacity=0); sp.reset()
sp.step(); t = time.time(); sp.step(); print('C2 move %.1f ms' % ((time.time() - t) * 1e3))
" > gpurun_out/sims_trace_c2.txt || exit $?
python3 tools/sims_trace.py gpurun_out/sims_trace.bin 256 >> gpurun_out/sims_trace_c2.txt && cat gpurun_out/sims_trace_c2.txt
timeout -k 10 200 bash tools/pmc_run.sh gpurun_out/pmcw2 2048 8 f32 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final2 -o c3 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_final2_c3.json 2> $R/gpurun_out/prof_final2_c3.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final2 -o c2 -- python3 $R/bench.py --games 256 --blocks 6 --filters 64 --steps 4 --warmup 1 --no-cpu-baseline --train-steps 0 > $R/gpurun_out/prof_final2_c2.json 2> $R/gpurun_out/prof_final2_c2.err || exit $?
head -4 $R/gpurun_out/prof_final2/c3_kernel_stats.csv | cut -c1-150
head -6 $R/gpurun_out/prof_final2/c2_kernel_stats.csv | cut -c1-150
