set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
: > gpurun_out/c3chunk.log
for rep in 1 2; do for mc in ${MCS:-4096 8192}; do
  timeout -k 10 200 python bench.py --m-chunk $mc --no-cpu --steps 10 --warmup 3 > gpurun_out/_c3.log 2>&1 || { tail -5 gpurun_out/_c3.log; exit 1; }
  python3 -c "
import json;j=json.loads(open('gpurun_out/_c3.log').read().strip().splitlines()[-1]);r=j['roofline']
print('m_chunk $mc', round(j['ms_per_step'],3), 'ms trmm', r['avg_launch_ms'], r['launches'], r['achieved'], 'TF/s trmm/step', j['roofline_aux']['trmm_ms_per_step'])" >> gpurun_out/c3chunk.log
done; done
cat gpurun_out/c3chunk.log
