#!/bin/bash
# C3: cross_start A/B in ABBA order (cancels the slow drift of the TRMM's clock over a run).
#   tools/ab_cross_start.sh TAG A B      -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; A=$2; B=$3
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for cs in $A $B $B $A $A $B $B $A; do
  timeout -k 10 200 python bench.py --cross-start $cs --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
  python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']; a=l['roofline_aux']
print('cross_start %s: step %.3f ms  trmm %.4f ms/launch  head (step - 7 trmm) %.3f ms  potrf %.4f ms  cross %.3f ms/step' % ('$cs', l['ms_per_step'], r['avg_launch_ms'], l['ms_per_step'] - 7 * r['avg_launch_ms'], a['potrf_inv']['avg_call_ms'], a['cross']['ms_per_step']))
" >> gpurun_out/$TAG.log || exit 1
done
cat gpurun_out/$TAG.log
