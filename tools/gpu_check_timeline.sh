#!/bin/bash
# GPU box job: parity tests, bench, rocprofv3 kernel trace of a short bench run, and the
# per-step timeline of the last step (tools/step_timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-run}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu ${BENCH_ARGS} > $R/gpurun_out/${TAG}_prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
python3 $R/tools/step_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv | tee $R/gpurun_out/${TAG}_timeline.txt
