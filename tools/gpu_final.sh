#!/bin/bash
# GPU box job: parity tests, bench (C3, with CPU baseline), rocprofv3 kernel trace + stats of a
# short bench run with its step timeline, the standalone potrf timeline, and the PMC traffic
# passes (FETCH_SIZE, WRITE_SIZE; separate runs).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-final}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 $R/tools/step_timeline.py $R/gpurun_out/${TAG}_prof/run_kernel_trace.csv > $R/gpurun_out/${TAG}_timeline.txt || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/potrf_tl -o run --output-format csv -- python3 $R/tools/prof_potrf.py 4096 5 > $R/gpurun_out/potrf_tl.log 2>&1 || exit 1
python3 $R/tools/potrf_timeline.py $R/gpurun_out/potrf_tl/run_kernel_trace.csv > $R/gpurun_out/${TAG}_potrf_timeline.txt || exit 1
bash $R/tools/pmc_traffic.sh > $R/gpurun_out/${TAG}_pmc.txt 2>&1 || exit 1
tail -12 $R/gpurun_out/${TAG}_pmc.txt
bash $R/tools/pmc_mfma.sh > $R/gpurun_out/${TAG}_pmc_mfma.txt 2>&1 || exit 1
bash $R/tools/pmc_lds.sh > $R/gpurun_out/${TAG}_pmc_lds.txt 2>&1 || exit 1
grep "trmm" $R/gpurun_out/${TAG}_pmc_mfma.txt $R/gpurun_out/${TAG}_pmc_lds.txt | cut -c1-200
