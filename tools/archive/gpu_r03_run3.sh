set -o pipefail
bash tools/gpu_r03_ab3.sh || exit $?
bash tools/gpu_r03_train1.sh
