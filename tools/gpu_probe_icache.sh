#!/bin/bash
# GPU box job: instruction-cache counters for tools/probe_update (n = 2048).
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU -d $R/gpurun_out/pi -o run --output-format csv -- $R/tools/probe_update 2048 > $R/gpurun_out/pi.log 2>&1
echo rc=$?
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
f = glob.glob(f"{R}/gpurun_out/pi/**/*counter_collection.csv", recursive=True)
if not f:
    print(open(f"{R}/gpurun_out/pi.log").read()[-3000:]); sys.exit()
rows = list(csv.DictReader(open(f[0])))
by = collections.defaultdict(dict)
for r in rows:
    by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    by[int(r["Dispatch_Id"])]["name"] = r["Kernel_Name"][:45]
ups = [d for k, d in sorted(by.items()) if "chol_update" in d["name"]]
# 5 k values x 5 modes x 11 reps
for i in range(0, len(ups), 11):
    d = ups[i + 5]
    kk, mode = divmod(i // 11, 5)
    print(f"k-index {kk} mode {mode}: " + " ".join(f"{c}={int(v)}" for c, v in d.items() if c != "name"))
PY
