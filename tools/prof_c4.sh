#!/bin/bash
# rocprofv3 kernel stats of a short C4 bench (per-kernel time split of the batched predict path)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-c4prof}
CH=${2:-0}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG} -o run --output-format csv -- python3 $R/bench.py --workload c4 --m-chunk $CH --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/${TAG}.log 2>&1 || exit 1
python3 - $R/gpurun_out/${TAG}/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(f"{r['Name'][:60]:60s} calls {int(r['Calls']):5d} total {float(r['TotalDurationNs'])/1e6:9.3f} ms avg {float(r['AverageNs'])/1e3:9.1f} us")
PY
tail -1 $R/gpurun_out/${TAG}.log | cut -c1-200
