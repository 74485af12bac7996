#!/bin/bash
# Round 3, first GPU job: the whole GPU suite (new: fault path, large-batch parity, package
# sharding), smoke, default bench, the self-launched --gpus 2 bench on the one GPU, the
# latency harness, and the group-size A/B.  Each step has its own limit; the first failure ends
# the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r03a}
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
step bench
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
step bench_n2
timeout -k 10 400 python bench.py --gpus 2 --share-gpu --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_bench_n2.log 2>&1 || exit 1
grep '^{' gpurun_out/${TAG}_bench_n2.log | cut -c1-300
step latency
timeout -k 10 400 python bench.py --workload latency --latency-points 10 --warmup 2 > gpurun_out/${TAG}_latency.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_latency.log | cut -c1-600
step ab_group
timeout -k 10 400 python tools/ab_group.py > gpurun_out/${TAG}_ab_group.log 2>&1 || exit 1
step done
