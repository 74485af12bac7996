# Omega read as drawn (float32 in place): fit-side GPU tests, PCA profile, fit bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fitside.py tests/test_gpu_emulator.py tests/test_gpu_dropin.py tests/test_gpu_mcmc.py > gpurun_out/r05_tsfast2_pytest.log 2>&1 || { tail -40 gpurun_out/r05_tsfast2_pytest.log; exit 1; }
tail -2 gpurun_out/r05_tsfast2_pytest.log
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05_tsfast2_pca.log 2>&1 || exit 1
grep -E "init_model|5.791 GB|randomized_svd" gpurun_out/r05_tsfast2_pca.log
timeout -k 10 300 python bench.py --workload fit > gpurun_out/r05_tsfast2_fit.log 2>&1 || exit 1
grep '^{' gpurun_out/r05_tsfast2_fit.log | cut -c1-120
grep -o '"breakdown.*' gpurun_out/r05_tsfast2_fit.log | cut -c1-300
