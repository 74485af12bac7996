#!/bin/bash
# GPU box job: parity tests, bench, then a rocprofv3 kernel-trace of a short bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-run}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu ${BENCH_ARGS} > $R/gpurun_out/${TAG}_prof.log 2>&1
rc=$?
python3 - "$R/gpurun_out/${TAG}_prof/run_kernel_stats.csv" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(f"{x['Name'][:60]:60s} {x['Calls']:>6s} {float(x['AverageNs'])/1e3:10.1f} us {x['Percentage'][:5]}%")
PY
exit $rc
