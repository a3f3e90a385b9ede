# round 3: A/B tail-only (base) vs + pre-transform with xres read from LDS (xlds) vs + xres in registers (cur)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_run.sh gpurun_out/r03_ab_wino_ab7_c3.log 32 build_var/base/libaz.so build_var/xlds/libaz.so build_var/cur/libaz.so build_var/base/libaz.so build_var/xlds/libaz.so build_var/cur/libaz.so || exit 3
cut -c1-150 gpurun_out/r03_ab_wino_ab7_c3.log
