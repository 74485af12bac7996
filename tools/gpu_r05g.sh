set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05g_prof_pca.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r05g_ev.log 2>&1 || exit 1
  GPFIT_BENCH_NOEVENTS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r05g_noev.log 2>&1 || exit 1
  python3 -c "
import json
f=lambda p: json.loads([x for x in open(p).read().splitlines() if x.startswith('{')][-1])['ms_per_step']
print('events %.3f ms  no events %.3f ms' % (f('gpurun_out/r05g_ev.log'), f('gpurun_out/r05g_noev.log')))" | tee -a gpurun_out/r05g_events_ab.log
done
timeout -k 10 900 bash tools/sweep_c4_aux.sh r05g_c4aux "8192:4 8192:7 8192:13" || exit 1
