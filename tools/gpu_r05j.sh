set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fitside.py tests/test_gpu_emulator.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05j_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r05j_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05j_prof_pca.log 2>&1 || exit 1
grep -E "gemm\(|init_model|randomized" gpurun_out/r05j_prof_pca.log | head -8
timeout -k 10 200 python tools/dbg/ts_probe.py > gpurun_out/r05j_ts_probe.log 2>&1 || exit 1
cat gpurun_out/r05j_ts_probe.log
