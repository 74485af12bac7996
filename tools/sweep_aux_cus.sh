#!/bin/bash
# C3: CUs the cross-covariance stream leaves to the factorisation (gp_ctx aux_free_cus, FRS)
# and the factorisation step fraction it starts at (cross_start, CSS; -1 = library default),
# two interleaved rounds on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sweep_aux_cus}
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for fr in ${FRS:-0 16 32 48 64}; do
   for cs in ${CSS:--1}; do
    timeout -k 10 200 python bench.py --aux-free-cus $fr --cross-start $cs --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']; a=l['roofline_aux']
print('c3 aux_free_cus $fr cross_start $cs: step %.3f ms  %.3fM pred/s  trmm %.4f ms/launch  potrf %.4f ms  cross %.3f ms/step' % (l['ms_per_step'], l['value']/1e6, r['avg_launch_ms'], a['potrf_inv']['avg_call_ms'], a['cross']['ms_per_step']))
" >> gpurun_out/$TAG.log || exit 1
    tail -1 gpurun_out/$TAG.log
   done
  done
done
