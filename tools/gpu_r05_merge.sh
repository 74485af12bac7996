# Sampler: decide + next prep in one launch (gp_mcmc_group_step) vs two: GPU tests, fit A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mcmc.py tests/test_gpu_faults.py tests/test_gpu_emulator.py > gpurun_out/r05_merge_pytest.log 2>&1 || { tail -40 gpurun_out/r05_merge_pytest.log; exit 1; }
tail -2 gpurun_out/r05_merge_pytest.log
: > gpurun_out/r05_merge_fit.log
for rep in 1 2; do
  for M in 0 1; do
    GPFIT_MCMC_MERGE=$M timeout -k 10 300 python bench.py --workload fit > gpurun_out/r05_merge_one.log 2>&1 || { cat gpurun_out/r05_merge_one.log; exit 1; }
    python -c "
import json
l=json.loads([x for x in open('gpurun_out/r05_merge_one.log').read().splitlines() if x.startswith('{')][-1])
b=l['breakdown']
print('merge %s  fit %.3f s  mcmc %.3f s  %.3f ms/sweep' % ('$M', l['value'], b['mcmc_s'], b['mcmc_ms_per_sweep']))
" >> gpurun_out/r05_merge_fit.log || exit 1
  done
done
cat gpurun_out/r05_merge_fit.log
