#!/bin/bash
# Build kernel variants of libaz.so for tools/tower_ab: each arg is name=FLAGS (FLAGS space-separated
# -D knobs, use ',' between them), output build_var/<name>/libaz.so.
set -e
R=$(cd $(dirname $0)/.. && pwd)
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}; flags=${flags//,/ }
  mkdir -p $R/build_var/$name
  make -s -C $R/alphazero-chess_amd/csrc OUT=$R/build_var/$name/libaz.so OBJDIR=$R/build_var/$name/obj EXTRA="$flags" > $R/build_var/$name/build.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
