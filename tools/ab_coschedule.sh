#!/bin/bash
# A/B of TRMM occupancy (dynamic LDS pad -> 1 TRMM block per CU) with and without cross-step
# pipelining (next step's factorisation co-resident beside the TRMM).  One line per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_cosched.log
: > $OUT
run() {
  local tag=$1; shift
  timeout -k 10 150 env "$@" python bench.py --no-cpu --steps 10 --warmup 3 $EXTRA > gpurun_out/_ab.log 2>&1 || { echo "FAIL $tag" >> $OUT; tail -5 gpurun_out/_ab.log >> $OUT; exit 1; }
  python3 - "$tag" >> $OUT <<'PY'
import json, sys
j = json.loads(open("gpurun_out/_ab.log").read().strip().splitlines()[-1])
r, a = j["roofline"], j["roofline_aux"]
print(f"{sys.argv[1]:34s} step {j['ms_per_step']:7.3f} ms  trmm {r['avg_launch_ms']:.4f} ms/launch "
      f"({r['achieved']:.1f} TF/s)  potrf {a['potrf_inv']['avg_call_ms']:.3f} ms  cross {a['cross']['ms_per_step']:.3f}")
PY
}
for rep in 1 2; do
EXTRA="" run "base" GPFIT_X=0
EXTRA="" run "base hwq8" GPU_MAX_HW_QUEUES=8
EXTRA="--pipeline" run "pipe" GPFIT_X=0
EXTRA="--pipeline" run "pipe hwq8" GPU_MAX_HW_QUEUES=8
EXTRA="--pipeline" run "pipe hwq8 nomask" GPU_MAX_HW_QUEUES=8 GPFIT_AUX_FREE_CUS=0
EXTRA="--pipeline" run "pipe hwq8 cross0" GPU_MAX_HW_QUEUES=8 GPFIT_CROSS_START=0
done
cat $OUT
