#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for order in 0 3; do
  for mc in 4096 8192; do
    r=$(GPFIT_TRMM_ORDER=$order timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu --m-chunk $mc | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['roofline']['achieved'], d['roofline_aux']['trmm_ms_per_step'])") || exit 1
    echo "c3 order=$order mc=$mc ms/step,trmmTF,trmm_ms: $r"
    r=$(GPFIT_TRMM_ORDER=$order timeout -k 10 120 python bench.py --workload c4 --steps 3 --warmup 1 --m-chunk $mc | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['roofline']['achieved'])") || exit 1
    echo "c4 order=$order mc=$mc ms/step,trmmTF: $r"
  done
done
