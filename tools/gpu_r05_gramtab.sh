# Gram with the table exp: Gram / likelihood / prediction GPU tests, then fit and C3 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mcmc.py tests/test_gpu_dropin.py tests/test_gpu_c3.py tests/test_gpu_emulator.py > gpurun_out/r05_gramtab_pytest.log 2>&1 || { tail -40 gpurun_out/r05_gramtab_pytest.log; exit 1; }
tail -2 gpurun_out/r05_gramtab_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash tools/ab_fit_libs.sh r05_gramtab_fit _ab/gr_old.so _ab/gr_new.so > /dev/null || exit 1
cat gpurun_out/r05_gramtab_fit.log
AB_WORKLOADS=c3 bash tools/ab_bench_libs.sh r05_gramtab_c3 _ab/gr_old.so _ab/gr_new.so > /dev/null || exit 1
cat gpurun_out/r05_gramtab_c3.log
