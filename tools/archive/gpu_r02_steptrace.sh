set -o pipefail
mkdir -p gpurun_out
make -s -C tools > gpurun_out/tools_build.log 2>&1 || exit 1
for dt in bf16 f32; do
rm -f gpurun_out/step_trace_$dt.bin
AZ_STEP_TRACE_FILE=gpurun_out/step_trace_$dt.bin DTYPE=$dt GAMES=256 BLOCKS=6 FILTERS=64 bash tools/ab_run.sh gpurun_out/trace_c2_$dt.log 800 build_var/trace/libaz.so || exit $?
python3 tools/step_trace.py gpurun_out/step_trace_$dt.bin 256
done
