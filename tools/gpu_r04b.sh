#!/bin/bash
# Round 4 evidence job: the whole GPU suite + smoke, the C3 bench (CPU baseline included),
# C4 bench, rocprofv3 kernel + RCCL API trace of the bench through the one-rank RCCL path
# (--force-nccl), the C3 kernel trace + step timeline, the factorisation's dataflow trace, and
# the PCA profile.  Each step has its own time limit; the first failure ends the job.
#   tools/gpu_r04b.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r04b}
R=$(pwd)
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
step bench
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-300
step c4
timeout -k 10 300 python bench.py --workload c4 --steps 5 --warmup 2 > gpurun_out/${TAG}_c4.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_c4.log | cut -c1-250
step fit
timeout -k 10 300 python bench.py --workload fit > gpurun_out/${TAG}_fit.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_fit.log | cut -c1-250
step rocprof_c3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 $R/tools/step_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv > $R/gpurun_out/${TAG}_timeline.txt || exit 1
step rocprof_rccl
timeout -k 10 400 rocprofv3 --rccl-trace --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof_nccl -o run --output-format csv -- python3 $R/bench.py --force-nccl --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof_nccl.log 2>&1 || exit 1
cd $R
ls gpurun_out/${TAG}_prof_nccl/
step pptrace
timeout -k 10 120 python tools/dbg/pp_trace.py 4096 > gpurun_out/${TAG}_pptrace.txt 2>&1 || exit 1
step potrf_modes
timeout -k 10 120 python tools/prof_potrf_modes.py > gpurun_out/${TAG}_potrf_modes.log 2>&1 || exit 1
cat gpurun_out/${TAG}_potrf_modes.log
step pca
timeout -k 10 120 python tools/prof_pca.py > gpurun_out/${TAG}_prof_pca.log 2>&1 || exit 1
head -3 gpurun_out/${TAG}_prof_pca.log
step end
