set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05b_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/dbg/trmv_micro > gpurun_out/r05b_trmv_micro.log 2>&1 || exit 1
cat gpurun_out/r05b_trmv_micro.log
timeout -k 10 300 python tools/prof_bcast_contention.py > gpurun_out/r05b_bcast.log 2>&1 || exit 1
cat gpurun_out/r05b_bcast.log
