#!/bin/bash
# Same-box A/B of the Metropolis sweep's speculative group size (GPFIT_MCMC_SPEC = updates per
# batched gp_loglik) on the fit workload, interleaved: fit seconds, MCMC seconds, ms per sweep.
#   tools/ab_mcmc_spec.sh TAG spec...   -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
mkdir -p gpurun_out
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for sp in "$@"; do
    GPFIT_MCMC_SPEC=$sp timeout -k 10 300 python bench.py --workload fit > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
b=l['breakdown']
print('spec=$sp fit %.3f s  mcmc %.3f s  %.3f ms/sweep' % (l['value'], b['mcmc_s'], b['mcmc_ms_per_sweep']))
" >> gpurun_out/$TAG.log || exit 1
  done
done
cat gpurun_out/$TAG.log
