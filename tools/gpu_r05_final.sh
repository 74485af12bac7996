# Round-5 closing check on the final tree: the whole GPU suite, smoke, C3 bench (no CPU leg)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05z2_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r05z2_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z2_smoke.log 2>&1 || { tail -5 gpurun_out/r05z2_smoke.log; exit 1; }
tail -1 gpurun_out/r05z2_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r05z2_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/r05z2_bench.log | cut -c1-400
timeout -k 10 400 python bench.py --workload fit > gpurun_out/r05z2_bench_fit.log 2>&1 || exit 1
grep '^{' gpurun_out/r05z2_bench_fit.log | cut -c1-200
