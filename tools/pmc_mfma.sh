#!/bin/bash
# MFMA busy fraction and effective clock of the bench's kernels (one --pmc pass of its own).
#   tools/pmc_mfma.sh [c3|c4]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
WL=${1:-c3}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_mfma -o run --output-format csv -- python3 $R/bench.py --workload $WL --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_mfma.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/pmc_mfma_kt -o run --output-format csv -- python3 $R/bench.py --workload $WL --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_mfma_kt.log 2>&1 || exit 1
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
def key(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
f = glob.glob(f"{R}/gpurun_out/pmc_mfma/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
kt = glob.glob(f"{R}/gpurun_out/pmc_mfma_kt/**/*kernel_trace.csv", recursive=True)[0]
dur = collections.defaultdict(list)
for r in csv.DictReader(open(kt)):
    dur[key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    d = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
    line = f"{k:40s} n={len(c['GRBM_GUI_ACTIVE']):4d} dur={d/1e3:9.1f} us"
    if "GRBM_GUI_ACTIVE" in m and d == d:
        clk = m["GRBM_GUI_ACTIVE"] / 8 / (d * 1e-9) / 1e9
        line += f" eff_clock={clk:5.2f} GHz"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            # MFMA busy cycles summed over SIMDs (1024) vs the kernel's GPU cycles
            busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
            line += f" mfma_busy={busy:6.3f}"
    print(line)
PY
