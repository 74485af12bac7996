# Round-5 evidence, part 2: C4 PMC + rocprof (library default), GPU suite, smoke, broadcast
# contention + scaling projection, the default bench (CPU baseline included), C4 and fit benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R0=$(pwd)
step() { echo "== $1 $(date +%T)"; }
step pmc_c4
bash tools/pmc_traffic.sh c4 > gpurun_out/r05o_pmc_c4.log 2>&1 || { tail -5 gpurun_out/r05o_pmc_c4.log; exit 1; }
tail -1 gpurun_out/r05o_pmc_c4.log
step pytest
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05o_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r05o_pytest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05o_smoke.log 2>&1 || { tail -5 gpurun_out/r05o_smoke.log; exit 1; }
tail -2 gpurun_out/r05o_smoke.log
step bcast
timeout -k 10 400 python tools/prof_bcast_contention.py > gpurun_out/r05o_bcast.log 2>&1 || exit 1
R=$(grep "worst prediction slowdown" gpurun_out/r05o_bcast.log | sed 's/.*x//')
step projection
timeout -k 10 300 python tools/project_scaling.py $R > gpurun_out/r05o_proj.log 2>&1 || exit 1
cat gpurun_out/r05o_proj.log
step bench_c3
timeout -k 10 400 python bench.py > gpurun_out/r05o_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/r05o_bench.log | cut -c1-300
step bench_c4
timeout -k 10 400 python bench.py --workload c4 > gpurun_out/r05o_bench_c4.log 2>&1 || exit 1
grep '^{' gpurun_out/r05o_bench_c4.log | cut -c1-300
step bench_fit
timeout -k 10 400 python bench.py --workload fit > gpurun_out/r05o_bench_fit.log 2>&1 || exit 1
grep '^{' gpurun_out/r05o_bench_fit.log | cut -c1-300
step rocprof_c4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05o_prof_c4 -o run --output-format csv -- python3 $R0/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $R0/gpurun_out/r05o_prof_c4.log 2>&1 || exit 1
step end
