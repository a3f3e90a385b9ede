# f32 Winograd headline net: 256 complete self-play games at 800 sims/move (plies per game for bench.py's C3 projection)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/game_length.py 256 gpurun_out/r03_game_length_c3_f32.json f32 > gpurun_out/r03_game_length.log 2>&1
rc=$?; tail -3 gpurun_out/r03_game_length.log; exit $rc
