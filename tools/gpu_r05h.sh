set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fitside.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05h_pytest_fitside.log 2>&1
rc=$?; tail -3 gpurun_out/r05h_pytest_fitside.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05h_prof_pca.log 2>&1 || exit 1
grep -E "gemm\(" gpurun_out/r05h_prof_pca.log | head -4
cp gladsgp_amd/libgpfit.so gpurun_out/.keep.so && cp _ab/libgpfit_xq.so gladsgp_amd/libgpfit.so
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05h_prof_pca_old.log 2>&1; rc=$?
cp gpurun_out/.keep.so gladsgp_amd/libgpfit.so; [ $rc -ne 0 ] && exit $rc
grep -E "gemm\(" gpurun_out/r05h_prof_pca_old.log | head -4
