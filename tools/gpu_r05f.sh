set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05f
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || { tail -20 gpurun_out/${TAG}_bench_c3.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench_c3.json'))
print(d['value'], d['roofline']['frac'], d['roofline']['avg_ms_per_launch'])
t=d['training']; print('train', t.get('ms_per_step'), t.get('frac'), 'sharded', (t.get('sharded_batch') or {}).get('ms_per_step'))
print(json.dumps(d['cpu_baseline'])[:600])"
