#!/bin/bash
# Same-box A/B of the column-resident fused prediction (trmm_res_kernel) against the
# cross-covariance + pair-TRMM path (GPFIT_TRMM_RES=0) on C5, two interleaved rounds.
#   tools/ab_res.sh TAG   -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for res in 0 1; do
    GPFIT_TRMM_RES=$res timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']; ph=l['phases_ms']
print('GPFIT_TRMM_RES=$res c5 step %.3f ms  %.2fM pred/s  predict %.3f ms  trmm %.4f ms/launch x %d (%.1f TF/s, frac %.4f)' % (l['ms_per_step'], l['value']/1e6, ph['predict'], r['avg_launch_ms'], r['launches'], r['achieved'], r['frac']))
" >> gpurun_out/$TAG.log || exit 1
  done
done
cat gpurun_out/$TAG.log
