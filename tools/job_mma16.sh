set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/mma16_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/mma16_pytest.log; [ $rc -ne 0 ] && exit $rc
REPS=3 bash tools/ab_libs.sh cur mma16 || exit 1
bash tools/pmc_lds.sh > gpurun_out/pmc_lds_mma16.txt 2>&1; grep "chol_" gpurun_out/pmc_lds_mma16.txt | cut -c1-150
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/potrf_tl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_potrf.py 4096 5 > $GRAFT_REPO_ROOT/gpurun_out/potrf_tl.log 2>&1 && python3 $GRAFT_REPO_ROOT/tools/potrf_timeline.py $GRAFT_REPO_ROOT/gpurun_out/potrf_tl/run_kernel_trace.csv | tail -3
