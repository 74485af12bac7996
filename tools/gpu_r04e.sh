#!/bin/bash
# Round 4: the persistent factorisation with its task families as calls (353 registers, room for
# three cross-covariance waves per SIMD) against the inlined default (462, room for one):
# correctness of the new default, then same-box A/B of the factorisation alone, the C3 / C4
# benches and the fit.
#   tools/gpu_r04e.sh TAG      (needs _ab/libgpfit_calls.so, _ab/libgpfit_inline.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04e}
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest_sub
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c3.py tests/test_gpu_c4.py tests/test_gpu_faults.py tests/test_gpu_largebatch.py -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest_sub.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest_sub.log; [ $rc -ne 0 ] && exit $rc
step ab_potrf
timeout -k 10 300 python tools/ab_libs.py _ab/libgpfit_calls.so _ab/libgpfit_inline.so > gpurun_out/${TAG}_ab_potrf.log 2>&1 || { cat gpurun_out/${TAG}_ab_potrf.log; exit 1; }
cat gpurun_out/${TAG}_ab_potrf.log
step ab_bench
bash tools/ab_bench_libs.sh ${TAG}_ab_bench _ab/libgpfit_calls.so _ab/libgpfit_inline.so > /dev/null || exit 1
cat gpurun_out/${TAG}_ab_bench.log
step ab_fit
bash tools/ab_fit_libs.sh ${TAG}_ab_fit _ab/libgpfit_calls.so _ab/libgpfit_inline.so > /dev/null || exit 1
cat gpurun_out/${TAG}_ab_fit.log
step pca
timeout -k 10 300 python tools/prof_pca.py > gpurun_out/${TAG}_prof_pca.log 2>&1 || exit 1
tail -15 gpurun_out/${TAG}_prof_pca.log
step end
