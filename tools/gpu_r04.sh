#!/bin/bash
# Round 4 GPU job: new tests first (RCCL world 1, full-size C3 on the bench's context path, the
# sweep hook), then the whole GPU suite + smoke, the C3 bench, and rocprofv3 kernel trace +
# stats of the bench through the one-rank RCCL path (--force-nccl).  Each step has its own
# time limit; the first failure ends the job.
#   tools/gpu_r04.sh TAG [quick]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04a}
R=$(pwd)
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest_new
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_c3.py tests/test_gpu_largebatch.py -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest_new.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_new.log; [ $rc -ne 0 ] && exit $rc
if [ "$2" != "quick" ]; then
step pytest
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
fi
step bench
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
step bench_nccl
timeout -k 10 300 python bench.py --force-nccl --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_bench_nccl.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench_nccl.log | cut -c1-400
step rocprof_nccl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof_nccl -o run --output-format csv -- python3 $R/bench.py --force-nccl --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof_nccl.log 2>&1 || exit 1
cd $R
f=$(find gpurun_out/${TAG}_prof_nccl -name '*kernel_stats.csv' | head -1)
grep -i -E "nccl|rccl" "$f" | cut -c1-160 | head -20
step end
