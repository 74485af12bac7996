#!/bin/bash
# rocprofv3 kernel trace of a short C3 bench and its step timeline, with the inter-step gap
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-gap}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 $R/tools/step_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv > $R/gpurun_out/${TAG}_timeline.txt || exit 1
cat $R/gpurun_out/${TAG}_timeline.txt
tail -1 $R/gpurun_out/${TAG}_prof.log | cut -c1-200
