#!/bin/bash
# GPU box job: parity tests, then the bench (each step time-limited; stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_bench.log | cut -c1-1500
exit $rc
