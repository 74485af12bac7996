# Round-5 final evidence on the final library: GPU suite, smoke, PMC traffic (C3, C4), MFMA busy,
# rocprofv3 stats + timeline, broadcast contention + projection, C3 (CPU baseline included),
# C4, fit, PCA profile, latency harness
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R0=$(pwd)
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05x_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r05x_pytest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05x_smoke.log 2>&1 || { tail -5 gpurun_out/r05x_smoke.log; exit 1; }
tail -1 gpurun_out/r05x_smoke.log
step pmc
bash tools/pmc_traffic.sh c3 > gpurun_out/r05x_pmc_c3.log 2>&1 || exit 1
cp gpurun_out/pmc_traffic.json gpurun_out/r05x_pmc_traffic.json
bash tools/pmc_traffic.sh c4 > gpurun_out/r05x_pmc_c4.log 2>&1 || exit 1
cp gpurun_out/pmc_traffic_c4.json gpurun_out/r05x_pmc_traffic_c4.json
bash tools/pmc_mfma.sh c3 > gpurun_out/r05x_pmc_mfma_c3.txt 2>&1 || exit 1
grep -E "pp_kernel|trmm" gpurun_out/r05x_pmc_mfma_c3.txt
step rocprof_c3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05x_prof -o run --output-format csv -- python3 $R0/bench.py --steps 5 --warmup 2 --no-cpu > $R0/gpurun_out/r05x_prof.log 2>&1 || exit 1
python3 $R0/tools/step_timeline.py $R0/gpurun_out/r05x_prof/run_kernel_trace.csv > $R0/gpurun_out/r05x_timeline.txt || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05x_prof_c4 -o run --output-format csv -- python3 $R0/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $R0/gpurun_out/r05x_prof_c4.log 2>&1 || exit 1
cd $R0
step bcast
timeout -k 10 400 python tools/prof_bcast_contention.py > gpurun_out/r05x_bcast.log 2>&1 || exit 1
R=$(grep "worst prediction slowdown" gpurun_out/r05x_bcast.log | sed 's/.*x//')
timeout -k 10 300 python tools/project_scaling.py $R > gpurun_out/r05x_proj.log 2>&1 || exit 1
tail -3 gpurun_out/r05x_proj.log
step bench_c3
timeout -k 10 400 python bench.py > gpurun_out/r05x_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/r05x_bench.log | cut -c1-250
step bench_c4
timeout -k 10 400 python bench.py --workload c4 > gpurun_out/r05x_bench_c4.log 2>&1 || exit 1
grep '^{' gpurun_out/r05x_bench_c4.log | cut -c1-250
step bench_fit
timeout -k 10 400 python bench.py --workload fit > gpurun_out/r05x_bench_fit.log 2>&1 || exit 1
grep '^{' gpurun_out/r05x_bench_fit.log | cut -c1-250
step pca
timeout -k 10 200 python tools/prof_pca.py > gpurun_out/r05x_prof_pca.log 2>&1 || exit 1
step latency
timeout -k 10 400 python bench.py --workload latency > gpurun_out/r05x_bench_latency.log 2>&1 || exit 1
grep '^{' gpurun_out/r05x_bench_latency.log | cut -c1-250
step end
