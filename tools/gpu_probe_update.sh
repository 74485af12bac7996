#!/bin/bash
# GPU box job: tools/probe_update under a kernel trace, then one SQ counter pass.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pu_kt -o run --output-format csv -- $R/tools/probe_update > $R/gpurun_out/pu_kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES -d $R/gpurun_out/pu_pmc -o run --output-format csv -- $R/tools/probe_update > $R/gpurun_out/pu_pmc.log 2>&1 || exit 1
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(f"{R}/gpurun_out/pu_kt/**/run_kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ups = [r for r in rows if "chol_update" in r["Kernel_Name"]]
# 5 k values x 3 modes x 11 reps, in order
out = collections.defaultdict(list)
for i, r in enumerate(ups):
    kk, rem = divmod(i, 33); mode = rem // 11
    out[(kk, mode)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (kk, mode), v in sorted(out.items()):
    v = sorted(v)[1:-1]
    print(f"k-index {kk} mode {mode}: median {v[len(v)//2]:7.1f} us")
f = glob.glob(f"{R}/gpurun_out/pu_pmc/**/*counter_collection.csv", recursive=True)
if f:
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(k, {c: round(sum(v)/len(v)) for c, v in d.items()})
PY
