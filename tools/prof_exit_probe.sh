#!/bin/bash
# GPU box job: does the rocprofv3-wrapped bench exit cleanly with / without the CU-masked
# cross-covariance stream?
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for v in 0 64; do
  GPFIT_AUX_FREE_CUS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pe_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/pe_$v.log 2>&1
  echo "GPFIT_AUX_FREE_CUS=$v rc=$?"
done
