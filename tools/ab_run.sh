#!/bin/bash
# GPU box: A/B-time libaz.so variants under build_var/ (tools/tower_ab).  Usage: bash tools/ab_run.sh <out.log> [sims] lib...
set -e
R=$(pwd)
OUT=$1; shift
S=$1; shift
mkdir -p $(dirname $OUT)
[ -f /tmp/w20x256.f32 ] || python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights(20, 256, seed=42).tofile('/tmp/w20x256.f32')"
timeout -k 10 300 $R/tools/tower_ab 2048 $S 20 256 /tmp/w20x256.f32 "$@" > $OUT 2>&1
