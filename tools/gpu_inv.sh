set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_libs.py _ab/lib_pre.so _ab/lib_inv.so > gpurun_out/ab_inv.log 2>&1 || { cat gpurun_out/ab_inv.log; exit 1; }
cat gpurun_out/ab_inv.log
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/i1_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/i1_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_fit_libs.sh ab_inv_fit _ab/lib_pre.so _ab/lib_inv.so
