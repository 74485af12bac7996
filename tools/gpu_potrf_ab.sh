#!/bin/bash
# GPU box job: potrf_inv timing, persistent (default) vs sweep (GPFIT_POTRF_SWEEP=1), at the C3
# (n=4096, batch 1), C4 (n=1024, batch 32) and fit (n=512, batch 8) shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pab}
mkdir -p gpurun_out
for shape in "4096 8 1" "1024 8 32" "512 8 8" "1024 8 8" "512 8 64"; do
  timeout -k 10 120 python tools/prof_potrf.py $shape | tail -1 | sed 's/^/pp    /' >> gpurun_out/${TAG}.log || exit 1
  GPFIT_POTRF_SWEEP=1 timeout -k 10 120 python tools/prof_potrf.py $shape | tail -1 | sed 's/^/sweep /' >> gpurun_out/${TAG}.log || exit 1
done
cat gpurun_out/${TAG}.log
