#!/bin/bash
# GPU box job: kernel trace of tools/prof_potrf.py (gram + potrf_inv at n = 4096) and its
# per-step timeline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/potrf_tl -o run --output-format csv -- python3 $R/tools/prof_potrf.py 4096 5 > $R/gpurun_out/potrf_tl.log 2>&1 || { tail -5 $R/gpurun_out/potrf_tl.log; exit 1; }
python3 $R/tools/potrf_timeline.py $R/gpurun_out/potrf_tl/run_kernel_trace.csv > $R/gpurun_out/potrf_timeline.txt
tail -4 $R/gpurun_out/potrf_tl.log; tail -4 $R/gpurun_out/potrf_timeline.txt
