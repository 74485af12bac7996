#!/bin/bash
# Same-box A/B of library builds (_ab/lib_<tag>.so via GPFIT_LIB_AB): C3 bench per variant, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
OUT=gpurun_out/ab_libs.log; : > $OUT
for rep in $(seq 1 ${REPS:-2}); do for tag in "$@"; do
  timeout -k 10 150 env GPFIT_LIB_AB=$PWD/_ab/lib_$tag.so python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/_ab.log 2>&1 || { echo "FAIL $tag" >> $OUT; tail -5 gpurun_out/_ab.log >> $OUT; exit 1; }
  python3 - "$tag" >> $OUT <<'PY'
import json, sys
j = json.loads(open("gpurun_out/_ab.log").read().strip().splitlines()[-1])
r, a = j["roofline"], j["roofline_aux"]
print(f"{sys.argv[1]:20s} step {j['ms_per_step']:7.3f} ms  trmm {r['avg_launch_ms']:.4f} ms/launch ({r['achieved']:.1f} TF/s, frac {r['frac']})  potrf {a['potrf_inv']['avg_call_ms']:.3f} ms")
PY
done; done
cat $OUT
