set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for i in 1 2; do
AZ_LIB=$R/abvar/base/libaz.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05t2_prof_base$i -o t -- python3 $R/tools/train_prof.py 6 > $R/gpurun_out/r05t2_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05t2_prof_mask$i -o t -- python3 $R/tools/train_prof.py 6 >> $R/gpurun_out/r05t2_prof.log 2>&1 || exit 1
done
echo ok
