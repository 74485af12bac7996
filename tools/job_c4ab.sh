set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
: > gpurun_out/c4libs.log
for rep in 1 2; do for tag in "$@"; do
  timeout -k 10 200 env GPFIT_LIB_AB=$PWD/_ab/lib_$tag.so python bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/_c4.log 2>&1 || { tail -5 gpurun_out/_c4.log; exit 1; }
  python3 -c "
import json;j=json.loads(open('gpurun_out/_c4.log').read().strip().splitlines()[-1]);r=j['roofline']
print('$tag', round(j['ms_per_step'],3), 'ms', round(j['value']/1e6,2), 'M/s trmm', r['avg_launch_ms'], r['achieved'])" >> gpurun_out/c4libs.log
done; done
cat gpurun_out/c4libs.log
