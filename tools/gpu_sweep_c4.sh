#!/bin/bash
# GPU box job: C4 step time, gp_predict (cross-covariance then TRMM per chunk, one stream) vs
# gp_fit_predict on a gp_ctx (cross-covariance of every chunk on the CU-masked aux stream, each
# chunk's TRMM waiting for its own chunk) at several aux CU masks; two rounds so drift shows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sweepc4}
mkdir -p gpurun_out
: > gpurun_out/${TAG}.log
for rep in 1 2; do
  for cfg in ${CFGS:-"predict -1" "fit_predict 0" "fit_predict 128" "fit_predict 192" "fit_predict 224"}; do
    set -- $cfg
    timeout -k 10 180 python bench.py --workload c4 --steps 5 --warmup 2 --c4-path $1 --aux-free-cus $2 > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads(open('gpurun_out/${TAG}_one.log').read().strip().splitlines()[-1])
print('path=$1 free=$2 step %.3f ms  %.2fM pred/s  trmm %.3f ms/launch  potrf %.3f ms/step' % (l['ms_per_step'], l['value']/1e6, l['roofline']['avg_launch_ms'], l['roofline_aux']['potrf_inv_ms_per_step']))
" >> gpurun_out/${TAG}.log || exit 1
  done
done
cat gpurun_out/${TAG}.log
