"""Per-step timeline of the last potrf in a rocprofv3 kernel trace: for each block step k the
panel and update kernel durations and the idle gap before each launch (us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "chol_diag" in r["Kernel_Name"]]
seq = [r for r in rows[idx[-1]:] if "chol_" in r["Kernel_Name"]]
t0 = int(seq[0]["Start_Timestamp"])
tot, gaps = {}, 0.0
prev_end = None
line = []
step = 0
for r in seq:
    n = r["Kernel_Name"].split("::")[1].split("(")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    tot[n] = tot.get(n, 0) + (e - s) / 1e3
    gap = 0.0 if prev_end is None else max(0, s - prev_end) / 1e3
    gaps += gap
    prev_end = e
    line.append(f"{n.split('_')[1]} {(e - s) / 1e3:5.1f} (+{gap:4.1f})")
    if "update" in n or r is seq[-1]:
        print(f"k={step:2d} t={(s - t0) / 1e3:7.1f}  " + "  ".join(line))
        line = []
        step += 1
print("per-kernel totals (us):", {k: round(v, 1) for k, v in tot.items()})
print(f"launch gaps (us): {gaps:.1f}")
print("potrf span (us):", (int(seq[-1]["End_Timestamp"]) - t0) / 1e3)
