set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r05c_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05c_pytest.log; [ $rc -ne 0 ] && exit $rc
step bcast
timeout -k 10 400 python tools/prof_bcast_contention.py > gpurun_out/r05c_bcast.log 2>&1 || exit 1
cat gpurun_out/r05c_bcast.log
R=$(grep "worst prediction slowdown" gpurun_out/r05c_bcast.log | sed 's/.*x//')
step projection
timeout -k 10 300 python tools/project_scaling.py $R > gpurun_out/r05c_proj.log 2>&1 || exit 1
cat gpurun_out/r05c_proj.log
step bench
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r05c_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/r05c_bench.log | cut -c1-400
step rocprof_c3
R0=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05c_prof -o run --output-format csv -- python3 $R0/bench.py --steps 5 --warmup 2 --no-cpu > $R0/gpurun_out/r05c_prof.log 2>&1 || exit 1
python3 $R0/tools/step_timeline.py $R0/gpurun_out/r05c_prof/run_kernel_trace.csv > $R0/gpurun_out/r05c_timeline.txt || exit 1
head -20 $R0/gpurun_out/r05c_timeline.txt
step end
