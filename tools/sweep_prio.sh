#!/bin/bash
# GPU box job: C3 step time vs gp_fit_predict stream priorities (GPFIT_FP_PRIO = fact,aux,pred;
# -1 high, 0 normal, 1 low), with and without two alternating caller streams (--pipeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_prio.log
: > $OUT
for cfg in ${CFGS:-"0,0,0:" "0,0,0:--pipeline" "-1,0,0:--pipeline" "-1,0,1:--pipeline" "-1,-1,1:--pipeline" "0,0,1:--pipeline" "-1,0,0:"}; do
  pr=${cfg%%:*}; a=${cfg#*:}
  GPFIT_FP_PRIO=$pr timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/_b.log 2>&1 || { cat gpurun_out/_b.log; exit 1; }
  python3 - "$pr $a" >> $OUT <<'PY'
import json, sys
x = json.loads(open("gpurun_out/_b.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:22s} {x['ms_per_step']:7.2f} ms/step  {x['value']/1e6:6.3f} M/s  trmm {x['roofline']['avg_launch_ms']:.3f} ms/launch  potrf {x['roofline_aux']['potrf_inv']['avg_call_ms']:.2f} ms")
PY
  tail -1 $OUT
done
