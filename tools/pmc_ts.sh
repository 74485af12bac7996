#!/bin/bash
# Counters of the tall-skinny products on tools/dbg/ts_probe.py: MFMA busy + clock, then LDS
# conflicts / waits (separate --pmc passes), then a kernel trace for the durations.
#   bash tools/pmc_ts.sh   -> gpurun_out/pmc_ts.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/dbg/ts_probe.py"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_ts1 -o run --output-format csv -- $P > $R/gpurun_out/pmc_ts1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES -d $R/gpurun_out/pmc_ts2 -o run --output-format csv -- $P > $R/gpurun_out/pmc_ts2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/pmc_ts_kt -o run --output-format csv -- $P > $R/gpurun_out/pmc_ts_kt.log 2>&1 || exit 1
python3 - "$R" <<'PY' | tee $R/gpurun_out/pmc_ts.txt
import csv, glob, sys, collections
R = sys.argv[1]
def key(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:44]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("pmc_ts1", "pmc_ts2"):
    f = glob.glob(f"{R}/gpurun_out/{d}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        agg[key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
kt = glob.glob(f"{R}/gpurun_out/pmc_ts_kt/**/*kernel_trace.csv", recursive=True)[0]
dur = collections.defaultdict(list)
for r in csv.DictReader(open(kt)):
    dur[key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, c in agg.items():
    if "ts" not in k and "reduce" not in k:
        continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    d = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    li = m.get("SQ_LDS_IDX_ACTIVE", 0) or 1
    clk = m["GRBM_GUI_ACTIVE"] / 8 / (d * 1e-9) / 1e9 if d == d else float("nan")
    print(f"{k:44s} n={len(dur[k]):3d} dur={d/1e3:8.1f} us clk={clk:4.2f} "
          f"mfma_busy={m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * m['GRBM_GUI_ACTIVE'] / 8):5.3f} "
          f"wait_any/wave={m.get('SQ_WAIT_ANY',0)/wc:5.3f} wait_lds/wave={m.get('SQ_WAIT_INST_LDS',0)/wc:5.3f} "
          f"bank_conf/idx={m.get('SQ_LDS_BANK_CONFLICT',0)/li:5.3f} waves={m.get('SQ_WAVES',0):.0f}")
PY
