#!/bin/bash
# GPU box job: factorisation parity tests, then potrf timing (persistent vs the blocked
# sweep) at the C3, C4 and fit shapes.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pp}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu -k "cholesky or potrf or trtri or loglik or nll" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/${TAG}_time.log
for shape in "4096 6 1" "1024 6 32" "512 6 8" "2048 6 1"; do
  timeout -k 10 120 python tools/prof_potrf.py $shape | tail -1 | sed "s/^/pp    /" >> gpurun_out/${TAG}_time.log || exit 1
  GPFIT_POTRF_SWEEP=1 timeout -k 10 120 python tools/prof_potrf.py $shape | tail -1 | sed "s/^/sweep /" >> gpurun_out/${TAG}_time.log || exit 1
done
cat gpurun_out/${TAG}_time.log
