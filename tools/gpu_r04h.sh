#!/bin/bash
# Round 4: the last inverse row's early sums beside leaf 3 (diag micro + same-box potrf A/B,
# bit-identity of L^-1), the kernel tests on it, and a cross_start re-sweep now that the
# factorisation ends 0.15 ms sooner.
#   tools/gpu_r04h.sh TAG   (needs _ab/libgpfit_{prev,new}.so, tools/dbg/diag_micro_{nr1,r3})
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04h}
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step micro
for v in nr1 r3; do timeout -k 10 60 tools/dbg/diag_micro_$v > gpurun_out/${TAG}_micro_$v.log 2>&1 || exit 1; echo "$v $(grep -h "rep 3" gpurun_out/${TAG}_micro_$v.log | cut -c1-46 | tr "\n" " ")"; done
step ab_potrf
timeout -k 10 300 python tools/ab_libs.py _ab/libgpfit_prev.so _ab/libgpfit_new.so > gpurun_out/${TAG}_ab_potrf.log 2>&1 || { cat gpurun_out/${TAG}_ab_potrf.log; exit 1; }
cat gpurun_out/${TAG}_ab_potrf.log
step pytest
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c3.py tests/test_gpu_mcmc.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
step sweep_cs
FRS="0" CSS="0 0.2 0.4" bash tools/sweep_aux_cus.sh ${TAG}_sweep_cs > /dev/null || exit 1
cat gpurun_out/${TAG}_sweep_cs.log
step end
