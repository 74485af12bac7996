#!/bin/bash
# Test-point chunk sizes for C3 and C4 on one box (ms per step), interleaved.
#   tools/sweep_chunks.sh TAG -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for spec in "c4 4096" "c4 8192" "c4 2048" "c3 16384" "c3 12544" "c3 25088"; do
    set -- $spec
    st=10; [ $1 = c4 ] && st=5
    timeout -k 10 200 python bench.py --workload $1 --m-chunk $2 --steps $st --warmup 2 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('$1 chunk $2: step %.3f ms  %.2fM pred/s  trmm %.4f ms/launch (frac %.4f)' % (l['ms_per_step'], l['value']/1e6, r['avg_launch_ms'], r['frac']))
" >> gpurun_out/$TAG.log || exit 1
  done
done
cat gpurun_out/$TAG.log
