#!/bin/bash
# GPU box job: factorisation parity tests, then potrf timing (persistent vs sweep) and a
# kernel trace of the persistent path.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
TAG=${1:-pp}
mkdir -p gpurun_out
GPFIT_PP_WATCHDOG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu -k "cholesky or potrf or trtri or loglik or nll" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/prof_potrf.py 4096 8 > gpurun_out/${TAG}_time_pp.log 2>&1 || exit 1
GPFIT_POTRF_SWEEP=1 timeout -k 10 120 python tools/prof_potrf.py 4096 8 > gpurun_out/${TAG}_time_sweep.log 2>&1 || exit 1
tail -3 gpurun_out/${TAG}_time_pp.log gpurun_out/${TAG}_time_sweep.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_kt -o run --output-format csv -- python3 $R/tools/prof_potrf.py 4096 5 > $R/gpurun_out/${TAG}_kt.log 2>&1 || exit 1
head -6 $R/gpurun_out/${TAG}_kt/run_kernel_stats.csv | cut -c1-160
