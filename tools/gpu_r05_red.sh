set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fitside.py tests/test_gpu_emulator.py > gpurun_out/r05_red_pytest.log 2>&1 || { tail -30 gpurun_out/r05_red_pytest.log; exit 1; }
tail -2 gpurun_out/r05_red_pytest.log
timeout -k 10 200 python tools/dbg/ts_probe.py > gpurun_out/r05_red_ts.log 2>&1 || exit 1
cat gpurun_out/r05_red_ts.log
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05_red_pca.log 2>&1 || exit 1
tail -25 gpurun_out/r05_red_pca.log
