#!/bin/bash
# GPU box job: per-kernel PMC means for an arbitrary program, one --pmc pass per counter group
# plus one kernel-trace pass for durations.
#   tools/pmc_probe.sh TAG "COUNTERS;COUNTERS;..." python3 prog.py args...
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; GROUPS_=$2; shift 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_kt -o run --output-format csv -- "$@" > $R/gpurun_out/${TAG}_kt.log 2>&1 || exit 1
IFS=';' read -ra GS <<< "$GROUPS_"
i=0
for g in "${GS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g -d $R/gpurun_out/${TAG}_p$i -o run --output-format csv -- "$@" > $R/gpurun_out/${TAG}_p$i.log 2>&1 || exit 1
  i=$((i+1))
done
python3 - "$R" "$TAG" $i <<'PY'
import csv, glob, sys, collections
R, TAG, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
def key(s):
    return s.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:36]
kt = glob.glob(f"{R}/gpurun_out/{TAG}_kt/**/*kernel_trace.csv", recursive=True)[0]
dur = collections.defaultdict(list)
for r in csv.DictReader(open(kt)):
    dur[key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for i in range(n):
    f = glob.glob(f"{R}/gpurun_out/{TAG}_p{i}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        agg[key(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    d = dur[k]
    print(f"{k:36s} n={len(d):4d} dur_mean={sum(d)/len(d)/1e3:9.2f} us")
    for c, v in sorted(agg[k].items()):
        print(f"    {c:28s} mean {sum(v)/len(v):16.1f}")
PY
