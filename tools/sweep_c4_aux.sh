#!/bin/bash
# C4 on gp_fit_predict: test-point chunk x chunks whose cross-covariance runs beside the
# batched factorisation, two interleaved rounds (second round in reverse order).
#   tools/sweep_c4_aux.sh TAG "chunk:aux chunk:aux ..."   -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; CFGS=$2
REV=$(echo $CFGS | tr ' ' '\n' | tac | tr '\n' ' ')
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for cfg in $CFGS $REV; do
  ch=${cfg%%:*}; ax=${cfg#*:}
  timeout -k 10 200 python bench.py --workload c4 --steps 5 --warmup 2 --m-chunk $ch --aux-chunks $ax --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
  python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('chunk %5s aux %s: %.2f M/s  %.3f ms/step  trmm %.4f ms/launch (frac %.4f)' % ('$ch', '$ax', l['value']/1e6, l['ms_per_step'], r['avg_launch_ms'], r['frac']))
" >> gpurun_out/$TAG.log || exit 1
done
cat gpurun_out/$TAG.log
