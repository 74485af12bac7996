# Sampler kernels with parallel proposals / log-posterior terms: sampler GPU tests, fit A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mcmc.py tests/test_gpu_faults.py tests/test_gpu_emulator.py tests/test_capi.py > gpurun_out/r05_mc_pytest.log 2>&1 || { tail -40 gpurun_out/r05_mc_pytest.log; exit 1; }
tail -2 gpurun_out/r05_mc_pytest.log
bash tools/ab_fit_libs.sh r05_mc_fit _ab/mc_base.so _ab/mc_par.so
