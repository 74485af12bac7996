set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload fit > gpurun_out/fit_bench.log 2>&1; rc=$?; tail -1 gpurun_out/fit_bench.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
MCS="4096 8192" bash tools/job_c3chunk.sh > /dev/null 2>&1 || true
: > gpurun_out/c4chunk2.log
for rep in 1 2; do for mc in 4096 8192; do
  timeout -k 10 200 python bench.py --workload c4 --m-chunk $mc --steps 5 --warmup 2 > gpurun_out/_c4.log 2>&1 || exit 1
  python3 -c "
import json;j=json.loads(open('gpurun_out/_c4.log').read().strip().splitlines()[-1]);r=j['roofline']
print('c4 m_chunk $mc', round(j['ms_per_step'],3), 'ms', round(j['value']/1e6,2), 'M/s trmm', r['avg_launch_ms'], r['achieved'])" >> gpurun_out/c4chunk2.log
done; done
cat gpurun_out/c4chunk2.log
