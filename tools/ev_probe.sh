cd $GRAFT_REPO_ROOT
for r in 1 2; do
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ev_a.log 2>&1 || exit 1
GPFIT_BENCH_NOEVENTS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ev_b.log 2>&1 || exit 1
python3 -c "
import json
for f in ('gpurun_out/ev_a.log','gpurun_out/ev_b.log'):
    x=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(x['ms_per_step'],3))
"
done
