#!/bin/bash
# C4 with small test-point chunks (the batch's cross-covariance slab near the Infinity Cache
# size) against the 8192 default, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sweep_c4_small}
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for ch in 512 1024 2048 8192; do
    timeout -k 10 200 python bench.py --workload c4 --m-chunk $ch --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('c4 chunk $ch: step %.3f ms  %.2fM pred/s  trmm %.4f ms/launch x %d (frac %.4f)' % (l['ms_per_step'], l['value']/1e6, r['avg_launch_ms'], r['launches'], r['frac']))
" >> gpurun_out/$TAG.log || exit 1
    tail -1 gpurun_out/$TAG.log
  done
done
