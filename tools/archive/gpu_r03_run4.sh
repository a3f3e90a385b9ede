# pk2 A/B (C3, C2) then the training tests + step time with the Winograd weight grads
set -o pipefail
bash tools/gpu_r03_pk2.sh || exit $?
bash tools/gpu_r03_train1.sh
