#!/bin/bash
# LDS conflicts and wait breakdown of the C3 kernels (one --pmc pass, 8 SQ counters).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d $R/gpurun_out/pmc_lds -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_lds.log 2>&1 || exit 1
python3 - "$R" <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
def key(n):
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:32]
f = glob.glob(f"{R}/gpurun_out/pmc_lds/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    agg[key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    li = m.get("SQ_LDS_IDX_ACTIVE", 0) or 1
    print(f"{k:32s} bank_conflict/idx_active={m.get('SQ_LDS_BANK_CONFLICT',0)/li:6.3f} "
          f"addr_conflict/idx_active={m.get('SQ_LDS_ADDR_CONFLICT',0)/li:6.3f} "
          f"wait_any/wave={m.get('SQ_WAIT_ANY',0)/wc:6.3f} wait_inst_lds/wave={m.get('SQ_WAIT_INST_LDS',0)/wc:6.3f} "
          f"active_lds/wave={m.get('SQ_ACTIVE_INST_LDS',0)/wc:6.3f} lds_insts={m.get('SQ_INSTS_LDS',0):.3g}")
PY
