# MCMC block graphs: GPU tests of the sampler, then the fit with 1 vs 16 sweeps per replay
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mcmc.py tests/test_gpu_faults.py tests/test_gpu_emulator.py > gpurun_out/r05_block_pytest.log 2>&1 || { tail -40 gpurun_out/r05_block_pytest.log; exit 1; }
tail -2 gpurun_out/r05_block_pytest.log
: > gpurun_out/r05_block_fit.log
for rep in 1 2; do
  for B in 1 16 32; do
    GPFIT_MCMC_BLOCK=$B timeout -k 10 300 python bench.py --workload fit > gpurun_out/r05_block_one.log 2>&1 || { cat gpurun_out/r05_block_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/r05_block_one.log').read().splitlines() if x.startswith('{')][-1])
b=l['breakdown']
print('block %2d  fit %.3f s  mcmc %.3f s  %.3f ms/sweep' % ($B, l['value'], b['mcmc_s'], b['mcmc_ms_per_sweep']))
" >> gpurun_out/r05_block_fit.log || exit 1
  done
done
cat gpurun_out/r05_block_fit.log
