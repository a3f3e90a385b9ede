#!/bin/bash
# GPU box: A/B-time libaz.so variants under build_var/ (tools/tower_ab).
# Usage: [GAMES=2048 BLOCKS=20 FILTERS=256] bash tools/ab_run.sh <out.log> <sims> lib...
set -e
R=$(pwd)
OUT=$1; shift
S=$1; shift
G=${GAMES:-2048}; B=${BLOCKS:-20}; F=${FILTERS:-256}
mkdir -p $(dirname $OUT)
W=/tmp/w${B}x${F}.f32
[ -f $W ] || python3 -c "import sys; sys.path.insert(0, '$R/alphazero-chess_amd'); import azchess as A; A.random_weights($B, $F, seed=42).tofile('$W')"
timeout -k 10 300 $R/tools/tower_ab $G $S $B $F $W "$@" > $OUT 2>&1
