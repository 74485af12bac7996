set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/ab_xcd_queues.py > gpurun_out/r05f_xcd_queues.log 2>&1 || { cat gpurun_out/r05f_xcd_queues.log; exit 1; }
cat gpurun_out/r05f_xcd_queues.log
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05f_prof_pca.log 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_bench_libs.sh r05f_ab _ab/libgpfit_pk_new.so _ab/libgpfit_tabexp_ts.so _ab/libgpfit_fs.so _ab/libgpfit_xq.so || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r05f_ev.log 2>&1 || exit 1
  GPFIT_BENCH_NOEVENTS=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r05f_noev.log 2>&1 || exit 1
  python3 -c "
import json
f=lambda p: json.loads([x for x in open(p).read().splitlines() if x.startswith('{')][-1])['ms_per_step']
print('events %.3f ms  no events %.3f ms' % (f('gpurun_out/r05f_ev.log'), f('gpurun_out/r05f_noev.log')))" | tee -a gpurun_out/r05f_events_ab.log
done
timeout -k 10 900 bash tools/sweep_c4_aux.sh r05f_c4aux "8192:4 8192:7 8192:13" || exit 1
