# round-2 GPU session 5: full GPU suite after the scalar-load fixes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests5.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gputests5.log | tail -8
exit $rc
