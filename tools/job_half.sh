set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/half_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/half_pytest.log; [ $rc -ne 0 ] && exit $rc
REPS=3 bash tools/ab_libs.sh cur half
