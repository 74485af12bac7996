#!/bin/bash
# Round 4: the persistent chain's 16 x 16 leaf blocked four columns at a time (PP_LEAF_BLOCKED:
# 0 = one MFMA per column, 1 = blocked with LDS shuffles, 3 = blocked lane-local) -- same-box A/B
# of the factorisation, the C3 / C4 benches and the fit, then the GPU tests on the blocked build.
#   tools/gpu_r04f.sh TAG    (needs _ab/libgpfit_leaf{0,1,3}.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04f}
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step ab_potrf
timeout -k 10 300 python tools/ab_libs.py _ab/libgpfit_leaf0.so _ab/libgpfit_leaf1.so _ab/libgpfit_leaf3.so > gpurun_out/${TAG}_ab_potrf.log 2>&1 || { cat gpurun_out/${TAG}_ab_potrf.log; exit 1; }
cat gpurun_out/${TAG}_ab_potrf.log
step ab_fit
bash tools/ab_fit_libs.sh ${TAG}_ab_fit _ab/libgpfit_leaf0.so _ab/libgpfit_leaf3.so > /dev/null || exit 1
cat gpurun_out/${TAG}_ab_fit.log
step ab_bench
bash tools/ab_bench_libs.sh ${TAG}_ab_bench _ab/libgpfit_leaf0.so _ab/libgpfit_leaf3.so > /dev/null || exit 1
cat gpurun_out/${TAG}_ab_bench.log
step pytest_leaf3
cp gladsgp_amd/libgpfit.so gpurun_out/.keep_main.so
cp _ab/libgpfit_leaf3.so gladsgp_amd/libgpfit.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c3.py tests/test_gpu_c4.py tests/test_gpu_mcmc.py tests/test_gpu_faults.py tests/test_gpu_fitside.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest_leaf3.log 2>&1
rc=$?
cp gpurun_out/.keep_main.so gladsgp_amd/libgpfit.so
tail -3 gpurun_out/${TAG}_pytest_leaf3.log
step end
exit $rc
