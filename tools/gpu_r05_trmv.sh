# gp_loglik's trmv with its loop unrolled: likelihood GPU tests, then the fit A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mcmc.py tests/test_gpu_dropin.py tests/test_gpu_kernels.py > gpurun_out/r05_tv_pytest.log 2>&1 || { tail -40 gpurun_out/r05_tv_pytest.log; exit 1; }
tail -2 gpurun_out/r05_tv_pytest.log
bash tools/ab_fit_libs.sh r05_tv_fit _ab/tv_base.so _ab/tv_unroll.so
