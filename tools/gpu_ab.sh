#!/bin/bash
# Same-box A/B evidence job for a predict-side change: the GPU suite on the current library,
# the C3 / C4 benches with each library in turn (tools/ab_bench_libs.sh), the one-GPU scaling
# projection with each, and a rocprofv3 kernel trace + step timeline of the current library.
#   tools/gpu_ab.sh TAG old.so new.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; OLD=$2; NEW=$3
R=$(pwd)
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
cp "$NEW" gladsgp_amd/libgpfit.so
step pytest
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
step ab_bench
timeout -k 10 900 bash tools/ab_bench_libs.sh ${TAG}_ab "$OLD" "$NEW" || exit 1
for lib in "$OLD" "$NEW"; do
  step "projection $(basename $lib)"
  cp "$lib" gladsgp_amd/libgpfit.so
  timeout -k 10 300 python tools/project_scaling.py > gpurun_out/${TAG}_proj_$(basename $lib .so).log 2>&1 || exit 1
  cat gpurun_out/${TAG}_proj_$(basename $lib .so).log
done
cp "$NEW" gladsgp_amd/libgpfit.so
step rocprof_c3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 $R/tools/step_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv > $R/gpurun_out/${TAG}_timeline.txt || exit 1
cat $R/gpurun_out/${TAG}_timeline.txt | head -20
step end
