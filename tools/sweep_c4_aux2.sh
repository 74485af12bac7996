# C4 test-point chunk sweep (the library caps a batch's cross-covariance slab at 2 GB by
# default, i.e. 8192 points at 32 x 1024; explicit m_chunk overrides): 2 interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r05_c4_aux.log
for rep in 1 2 3; do
  for mc in 8192; do
    for ac in 0 1 2 3 4; do
    timeout -k 10 200 python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --m-chunk $mc --aux-chunks $ac > gpurun_out/r05_c4_one.log 2>&1 || { tail -5 gpurun_out/r05_c4_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/r05_c4_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('m_chunk %5d aux %d: %.3f ms/step  %.2f M pred/s  trmm %.4f ms/launch' % ($mc, $ac, l['ms_per_step'], l['value']/1e6, r['avg_launch_ms']))
" >> gpurun_out/r05_c4_aux.log || exit 1
    done
  done
done
cat gpurun_out/r05_c4_aux.log
