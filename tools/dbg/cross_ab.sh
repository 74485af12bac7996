#!/bin/bash
# GPU box job (debug): prediction parity tests, then the C3 step with the cross-covariance run
# after the factorisation on all CUs (its standalone time) and in the default placement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-x1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c3.py tests/test_gpu_c4.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1.0 0" "0.4 128" "0.4 64"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu --cross-start $1 --aux-free-cus $2 > gpurun_out/${TAG}_b.log 2>&1 || exit 1
  python - "$1" "$2" "gpurun_out/${TAG}_b.log" <<'PY'
import json, sys
l = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
a = l["roofline_aux"]
print(f"cross_start={sys.argv[1]} free={sys.argv[2]} step {l['ms_per_step']:.3f} ms cross "
      f"{a['cross']['ms_per_step']:.3f} ms ({a['cross']['achieved']} GB/s) potrf {a['potrf_inv']['avg_call_ms']:.3f}")
PY
done
