#!/bin/bash
# GPU box job: A/B of bench.py C3 step time under environment settings, interleaved runs.
#   ENVS="A=1 B=2|A=0" tools/ab_env.sh   (| separates variants; "-" = no extra env)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS='|' read -ra V <<< "${ENVS:--}"
for r in 1 2; do
  for v in "${V[@]}"; do
    e=""; [ "$v" != "-" ] && e="$v"
    env $e timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} > gpurun_out/_ab.log 2>&1 || { tail -5 gpurun_out/_ab.log; exit 1; }
    python3 - "$v" <<'PY'
import json, sys
x = json.loads(open("gpurun_out/_ab.log").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} {x['ms_per_step']:7.3f} ms/step  trmm {x['roofline']['avg_launch_ms']:.4f} ms/launch  potrf {x['roofline_aux']['potrf_inv']['avg_call_ms']:.3f} ms", flush=True)
PY
  done
done | tee gpurun_out/ab_env.log
