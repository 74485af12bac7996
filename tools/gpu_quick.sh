set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/g1_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/g1_smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/g1_bench.log 2>&1 || exit 1
tail -1 gpurun_out/g1_bench.log | cut -c1-600
