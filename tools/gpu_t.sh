#!/bin/bash
# GPU suite + smoke + C3 bench, then (optional 'pmc') the TRMM traffic passes for C3 and C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-t}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
if [ "$2" = pmc ]; then
  bash tools/pmc_traffic.sh c3 > gpurun_out/${TAG}_pmc.txt 2>&1 || exit 1
  tail -1 gpurun_out/${TAG}_pmc.txt
  bash tools/pmc_traffic.sh c4 > gpurun_out/${TAG}_pmc_c4.txt 2>&1 || exit 1
  tail -1 gpurun_out/${TAG}_pmc_c4.txt
fi
