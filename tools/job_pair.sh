set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3.py -x -q -s -m gpu --timeout 120 --timeout-method thread > gpurun_out/c3t_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/c3t_pytest.log; grep "C3 sample" gpurun_out/c3t_pytest.log; [ $rc -ne 0 ] && exit $rc
GPFIT_TRMM_PAIR=1 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pair_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/pair_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_vars.sh base pair:GPFIT_TRMM_PAIR=1 || exit 1
cp gpurun_out/ab_vars.log gpurun_out/ab_pair_c3.log
BENCH_ARGS="--workload c4 --steps 5 --warmup 2" bash tools/ab_vars.sh c4base c4pair:GPFIT_TRMM_PAIR=1
