set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fitside.py tests/test_gpu_emulator.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05l_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05l_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05l_prof_pca.log 2>&1 || exit 1
grep -E "gemm\(|init_model|randomized" gpurun_out/r05l_prof_pca.log | head -14
