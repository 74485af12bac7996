#!/bin/bash
# Counters of the prediction kernels on tools/dbg/res_probe.py (C5 shape): MFMA busy / clock,
# then wait / issue buckets and instruction counts, then LDS (separate --pmc passes), then a
# kernel trace for the durations.   bash tools/pmc_res.sh TAG  -> gpurun_out/TAG.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pmc_res}
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/dbg/res_probe.py"
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_kt -o run --output-format csv -- $P > $R/gpurun_out/${TAG}_kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/${TAG}_1 -o run --output-format csv -- $P > $R/gpurun_out/${TAG}_1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES -d $R/gpurun_out/${TAG}_2 -o run --output-format csv -- $P > $R/gpurun_out/${TAG}_2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum -d $R/gpurun_out/${TAG}_3 -o run --output-format csv -- $P > $R/gpurun_out/${TAG}_3.log 2>&1 || echo "pass 3 failed (counter names?)"
python3 - "$R" "$TAG" <<'PY' | tee $R/gpurun_out/$TAG.txt
import csv, glob, sys, collections
R, TAG = sys.argv[1], sys.argv[2]
def key(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:44]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in (f"{TAG}_1", f"{TAG}_2", f"{TAG}_3"):
    fs = glob.glob(f"{R}/gpurun_out/{d}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("no counters for", d); continue
    for r in csv.DictReader(open(fs[0])):
        agg[key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
kt = glob.glob(f"{R}/gpurun_out/{TAG}_kt/**/*kernel_trace.csv", recursive=True)[0]
dur = collections.defaultdict(list)
for r in csv.DictReader(open(kt)):
    dur[key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, c in agg.items():
    if not dur.get(k) or sum(dur[k]) / len(dur[k]) < 50e3:
        continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    d = sum(dur[k]) / len(dur[k])
    print(f"== {k}  dur {d/1e3:.1f} us")
    if "GRBM_GUI_ACTIVE" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        print(f"  eff_clock {cyc / (d * 1e-9) / 1e9:.2f} GHz  mfma_busy "
              f"{m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * cyc):.3f}")
    wc = m.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            print(f"  {n:24s} {m.get(n, 0) / wc:.3f} of wave cycles")
    for n, v in sorted(m.items()):
        print(f"  {n:32s} {v:16.1f}")
PY
