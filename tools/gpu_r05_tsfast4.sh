# Tall-skinny products' unmasked fast path: fit-side GPU tests, then the probe A/B (old / new)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fitside.py tests/test_gpu_emulator.py > gpurun_out/r05_tsfast4_pytest.log 2>&1 || { tail -40 gpurun_out/r05_tsfast4_pytest.log; exit 1; }
tail -2 gpurun_out/r05_tsfast4_pytest.log
TS_LIBS="_ab/ts_old.so _ab/ts_new.so" bash tools/gpu_tsm.sh > /dev/null || exit 1
cp gpurun_out/r05w_ts.log gpurun_out/r05_tsfast4_ab.log
grep -E "==|padded\]" gpurun_out/r05_tsfast4_ab.log
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05_tsfast4_pca.log 2>&1 || exit 1
grep -E "init_model|5.791 GB" gpurun_out/r05_tsfast4_pca.log
