#!/bin/bash
# Register use / spills of the tower kernels for a set of -D knobs (device-only compile of tower.hip).
# Usage: bash tools/kinfo.sh [-DAZ_...=N ...]   (prints .vgpr_count / spills per tower32w kernel;
# the disassembly is left in /tmp/kinfo/t.dis)
set -e
R=$(cd $(dirname $0)/.. && pwd)
D=/tmp/kinfo; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 --cuda-device-only -O3 -std=c++17 -ffp-contract=off "$@" -c -o $D/t.co $R/alphazero-chess_amd/csrc/tower.hip
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$D/t.co --targets=hipv4-amdgcn-amd-amdhsa-unknown-gfx950 --output=$D/t.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $D/t.elf | grep -E "^\s+\.name:|vgpr_count|vgpr_spill|agpr_count" | paste - - - - | grep tower32w | sed 's/_ZN3azi15//; s/EEEvPKf.*SearchOutE//'
/opt/rocm/lib/llvm/bin/llvm-objdump -d $D/t.elf > $D/t.dis
echo "scratch instructions: $(grep -c scratch_ $D/t.dis || true)"
