set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
GPFIT_TRMM_RING=1 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ring_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ring_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_vars.sh pair ring:GPFIT_TRMM_RING=1 || exit 1
cp gpurun_out/ab_vars.log gpurun_out/ab_ring_c3.log
BENCH_ARGS="--workload c4 --steps 5 --warmup 2" bash tools/ab_vars.sh c4pair c4ring:GPFIT_TRMM_RING=1
