set -o pipefail
cd $GRAFT_REPO_ROOT
for v in trace tracefake; do
  for h in 1 0; do
    AZ_TRAIN_HALF=$h AZ_LIB=abvar/$v/libaz.so timeout -k 10 300 python -u tools/train_trace.py 3 > gpurun_out/r05n_${v}_h$h.txt 2>&1 || exit 1
    echo "$v half=$h"; tail -2 gpurun_out/r05n_${v}_h$h.txt
  done
done
