set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t1_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/t1_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 150 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/t1_bench$i.log 2>&1 || exit 1
python3 -c "
import json;j=json.loads(open('gpurun_out/t1_bench$i.log').read().strip().splitlines()[-1]);r=j['roofline'];a=j['roofline_aux']
print('step',round(j['ms_per_step'],3),'trmm',r['avg_launch_ms'],r['achieved'],r['frac'],'potrf',a['potrf_inv']['avg_call_ms'])"; done
