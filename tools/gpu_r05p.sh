set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R0=$(pwd)
timeout -k 10 700 python -u -m pytest tests/test_gpu_sched.py tests/test_gpu_c3.py tests/test_gpu_c4.py tests/test_gpu_rccl.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r05p_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r05p_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab_bench_libs.sh r05p_ab _ab/libgpfit_cur.so _ab/libgpfit_hop.so || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R0/gpurun_out/r05p_prof -o run --output-format csv -- python3 $R0/bench.py --steps 5 --warmup 2 --no-cpu > $R0/gpurun_out/r05p_prof.log 2>&1 || exit 1
python3 $R0/tools/step_timeline.py $R0/gpurun_out/r05p_prof/run_kernel_trace.csv > $R0/gpurun_out/r05p_timeline.txt || exit 1
cat $R0/gpurun_out/r05p_timeline.txt
