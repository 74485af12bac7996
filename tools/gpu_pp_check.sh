#!/bin/bash
# Factorisation iteration job: the factorisation-facing GPU tests, per-part timings, the
# dataflow trace (trace build) and the C3 / C4 benches.  First failure ends the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pp}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_faults.py tests/test_gpu_largebatch.py tests/test_gpu_c3.py tests/test_gpu_c4.py tests/test_gpu_mcmc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/prof_parts.py > gpurun_out/${TAG}_parts.log 2>&1 || exit 1
cat gpurun_out/${TAG}_parts.log
timeout -k 10 120 python tools/dbg/pp_trace.py 4096 > gpurun_out/${TAG}_pptrace.txt 2>&1 || exit 1
head -3 gpurun_out/${TAG}_pptrace.txt | tail -2
grep "chain mean" gpurun_out/${TAG}_pptrace.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/${TAG}_c4.log 2>&1 || exit 1
for f in gpurun_out/${TAG}_bench.log gpurun_out/${TAG}_c4.log; do grep '^{' $f | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j.get('roofline_aux',{}).get('potrf_inv', j.get('roofline_aux')))"; done
