#!/bin/bash
# Same-box A/B of environment settings: each arg is "tag:VAR=val,VAR2=val" (tag alone = defaults);
# BENCH_ARGS adds bench.py options.  C3 bench per variant, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
OUT=gpurun_out/ab_vars.log; : > $OUT
for rep in $(seq 1 ${REPS:-2}); do for spec in "$@"; do
  tag=${spec%%:*}; vars=""; [ "$spec" != "$tag" ] && vars=$(echo "${spec#*:}" | tr ',' ' ')
  timeout -k 10 200 env GPFIT_X=0 $vars python bench.py --no-cpu --steps 10 --warmup 3 $BENCH_ARGS > gpurun_out/_ab.log 2>&1 || { echo "FAIL $tag" >> $OUT; tail -5 gpurun_out/_ab.log >> $OUT; cat $OUT; exit 1; }
  python3 - "$tag" >> $OUT <<'PY'
import json, sys
j = json.loads(open("gpurun_out/_ab.log").read().strip().splitlines()[-1])
r, a = j["roofline"], j.get("roofline_aux", {})
p = a.get("potrf_inv", {}).get("avg_call_ms", a.get("potrf_inv_ms_per_step"))
print(f"{sys.argv[1]:20s} step {j['ms_per_step']:7.3f} ms  trmm {r['avg_launch_ms']:.4f} ms/launch ({r['achieved']:.1f} TF/s, frac {r['frac']})  potrf {p}")
PY
done; done
cat $OUT
