# C3 aux-chunk re-sweep on the round-5 library (three interleaved rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r05_c3_aux.log
for rep in 1 2 3; do
  for ac in -1 6 4 2; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --aux-chunks $ac > gpurun_out/r05_c3_one.log 2>&1 || { tail -5 gpurun_out/r05_c3_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/r05_c3_one.log').read().splitlines() if x.startswith('{')][-1])
r=l['roofline']
print('aux %2d: %.3f ms/step  %.3f M pred/s  trmm %.4f ms/launch' % ($ac, l['ms_per_step'], l['value']/1e6, r['avg_launch_ms']))
" >> gpurun_out/r05_c3_aux.log || exit 1
  done
done
cat gpurun_out/r05_c3_aux.log
