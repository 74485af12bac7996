#!/bin/bash
# GPU box job: C3 step time vs the spatial split of gp_fit_predict (CUs reserved for the
# factorisation stream while two alternating caller streams pipeline consecutive problems).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/sweep_split.log
: > $OUT
for a in "" "--pipeline" ${SPLITS:-"--fact-cus 8" "--fact-cus 16" "--fact-cus 24" "--fact-cus 32"}; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/_b.log 2>&1 || { cat gpurun_out/_b.log; exit 1; }
  python3 - "$a" >> $OUT <<'PY'
import json, sys
x = json.loads(open("gpurun_out/_b.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1] or 'default':18s} {x['ms_per_step']:7.2f} ms/step  {x['value']/1e6:6.3f} M/s  trmm {x['roofline']['avg_launch_ms']:.3f} ms/launch  potrf {x['roofline_aux']['potrf_inv']['avg_call_ms']:.2f} ms")
PY
  tail -1 $OUT
done
