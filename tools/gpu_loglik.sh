set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mcmc.py tests/test_gpu_faults.py tests/test_capi.py tests/test_gpu_dropin.py -x -v --timeout 200 --timeout-method thread > gpurun_out/m3_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/m3_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_mcmc_spec.sh ab_spec2 2 3 4
