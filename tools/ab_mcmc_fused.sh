#!/bin/bash
# Same-box A/B of the fused sweep kernels (GPFIT_MCMC_FUSED=1) against the tensor-op sweep (=0)
# on the fit workload, spec 2, interleaved.   tools/ab_mcmc_fused.sh TAG -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for fu in 0 1; do
    GPFIT_MCMC_FUSED=$fu timeout -k 10 300 python bench.py --workload fit > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
b=l['breakdown']
print('fused=$fu fit %.3f s  pca %.3f s  mcmc %.3f s  %.3f ms/sweep' % (l['value'], b['pca_s'], b['mcmc_s'], b['mcmc_ms_per_sweep']))
" >> gpurun_out/$TAG.log || exit 1
  done
done
cat gpurun_out/$TAG.log
