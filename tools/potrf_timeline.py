"""Print the per-step kernel timeline of the last potrf in a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "chol_diag" in r["Kernel_Name"]]
seq = [r for r in rows[idx[-1]:] if "chol_" in r["Kernel_Name"]]
t0 = int(seq[0]["Start_Timestamp"])
tot = {}
for r in seq:
    n = r["Kernel_Name"].split("::")[1].split("(")[0]
    tot[n] = tot.get(n, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
step = 0
for r in seq:
    n = r["Kernel_Name"].split("::")[1].split("(")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if step % 8 == 0 or "diag" in n:
        print(f"{n:20s} start {(s - t0) / 1e3:9.1f}  dur {(e - s) / 1e3:7.1f}  grid {r['Grid_Size_X']}")
    if "update" in n:
        step += 1
print("per-kernel totals (us):", {k: round(v, 1) for k, v in tot.items()})
print("potrf span (us):", (int(seq[-1]["End_Timestamp"]) - t0) / 1e3)
