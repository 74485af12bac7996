#!/bin/bash
# Kernel trace of the fit workload (bench.py --workload fit): per-kernel time and the GPU-busy
# share of the MCMC phase.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fit -o run --output-format csv -- python3 $R/bench.py --workload fit > $R/gpurun_out/prof_fit.log 2>&1 || exit 1
python3 - "$R" <<'PY'
import csv, sys, collections
R = sys.argv[1]
rows = list(csv.DictReader(open(f"{R}/gpurun_out/prof_fit/run_kernel_trace.csv")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t0, t1 = ev[0][0], ev[-1][1]
busy, cur_s, cur_e = 0, None, None
for s, e, _ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"kernels {len(ev)}, span {(t1-t0)/1e6:.1f} ms, busy {busy/1e6:.1f} ms ({100*busy/(t1-t0):.0f}%)")
import re
def key(n):
    n = re.sub(r"^void ", "", n.replace("(anonymous namespace)::", ""))
    return n.split("(")[0][:60]
agg = collections.defaultdict(lambda: [0, 0])
for s, e, n in ev:
    k = key(n)
    agg[k][0] += 1; agg[k][1] += e - s
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:15]:
    print(f"{k:60s} {c:7d} {t/1e6:9.1f} ms  {t/c/1e3:8.1f} us")
# one Metropolis group in the middle of the run: kernels between consecutive pp_kernel starts
pp = [i for i, (_, _, n) in enumerate(ev) if "pp_kernel" in n]
if len(pp) > 10:
    a, b = pp[len(pp) // 2], pp[len(pp) // 2 + 1]
    base, prev_e = ev[a][0], None
    print(f"one group ({(ev[b][0] - ev[a][0]) / 1e3:.1f} us pp_kernel start to start):")
    for s, e, n in ev[a:b + 1]:
        gap = (s - prev_e) / 1e3 if prev_e is not None else 0.0
        print(f"  +{(s - base) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:6.1f}  {key(n)}")
        prev_e = e
PY
