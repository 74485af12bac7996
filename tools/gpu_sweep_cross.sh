#!/bin/bash
# GPU box job: C3 step time vs the cross-covariance placement (gp_ctx cross_start / CUs left
# free to the factorisation), two rounds so box drift shows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sweepx}
mkdir -p gpurun_out
: > gpurun_out/${TAG}.log
for rep in 1 2; do
  for cfg in ${CFGS:-"0.4 128" "0.4 96" "0.4 64" "0.4 32" "0.4 0"}; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu --cross-start $1 --aux-free-cus $2 > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json,sys
l=json.loads(open('gpurun_out/${TAG}_one.log').read().strip().splitlines()[-1])
a=l['roofline_aux']
print('cross_start=$1 free=$2 step %.3f ms potrf %.3f cross %.3f trmm %.3f' % (l['ms_per_step'], a['potrf_inv']['avg_call_ms'], a['cross']['ms_per_step'], a['trmm_ms_per_step']))
" >> gpurun_out/${TAG}.log || exit 1
  done
done
cat gpurun_out/${TAG}.log
