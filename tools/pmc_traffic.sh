#!/bin/bash
# HBM traffic per kernel from PMC counters (separate passes: FETCH_SIZE, WRITE_SIZE).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_$c.log 2>&1 || exit 1
done
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{R}/gpurun_out/pmc_{c}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counter csv for", c, glob.glob(f"{R}/gpurun_out/pmc_{c}/**/*", recursive=True)); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(list)
    for r in rows:
        agg[r["Kernel_Name"][:50]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f"{c:11s} {k:50s} n={len(v):4d} mean={sum(v)/len(v):14.1f} (KB per dispatch)")
PY
