#!/bin/bash
# C3: chunks whose cross-covariance runs beside the factorisation (gp_ctx_set_aux_chunks),
# A B B A A B B A order.
#   tools/ab_c3_aux_chunks.sh TAG A B   -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; A=$2; B=$3
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for ax in $A $B $B $A $A $B $B $A; do
  timeout -k 10 200 python bench.py --aux-chunks $ax --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
  python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('aux_chunks %3s: step %.3f ms  trmm %.4f ms/launch  head (step - 7 trmm) %.3f ms' % ('$ax', l['ms_per_step'], r['avg_launch_ms'], l['ms_per_step'] - 7 * r['avg_launch_ms']))
" >> gpurun_out/$TAG.log || exit 1
done
cat gpurun_out/$TAG.log
