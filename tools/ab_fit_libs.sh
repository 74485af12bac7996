#!/bin/bash
# Same-box A/B of whole library builds on the fit workload (MCMC ms per sweep), interleaved.
#   tools/ab_fit_libs.sh TAG lib1.so lib2.so ...   -> gpurun_out/TAG.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
mkdir -p gpurun_out
cp gladsgp_amd/libgpfit.so gpurun_out/.libgpfit_keep3.so
: > gpurun_out/$TAG.log
for rep in 1 2; do
  for lib in "$@"; do
    cp "$lib" gladsgp_amd/libgpfit.so
    timeout -k 10 300 python bench.py --workload fit --no-cpu > gpurun_out/${TAG}_one.log 2>&1 || { cat gpurun_out/${TAG}_one.log; cp gpurun_out/.libgpfit_keep3.so gladsgp_amd/libgpfit.so; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/${TAG}_one.log').read().splitlines() if x.startswith('{')][-1])
b=l['breakdown']
print('%-16s fit %.3f s  mcmc %.3f s  %.3f ms/sweep' % ('$(basename $lib)', l['value'], b['mcmc_s'], b['mcmc_ms_per_sweep']))
" >> gpurun_out/$TAG.log || exit 1
  done
done
cp gpurun_out/.libgpfit_keep3.so gladsgp_amd/libgpfit.so
cat gpurun_out/$TAG.log
