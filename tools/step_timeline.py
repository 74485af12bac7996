"""Timeline of the last gp_fit_predict step in a rocprofv3 kernel trace (bench.py C3 run):
kernel time per name, the step's span, and the idle time between consecutive kernels once
the TRMM phase has started (the prediction stream's launch gaps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts with the factorisation's schedule kernel (enqueued ahead of the Gram since
# round 5), or with the Gram in older traces
mark = "pp_schedule_kernel" if any("pp_schedule_kernel" in r["Kernel_Name"] for r in rows) \
    else "ardse_kernel"
starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
seq = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows[starts[-1]:]


def name(r):
    n = r["Kernel_Name"]
    n = n.split("::")[1] if "::" in n else n
    return n.split("(")[0].split("<")[0]


t0 = int(seq[0]["Start_Timestamp"])
tot, cnt = {}, {}
for r in seq:
    n = name(r)
    tot[n] = tot.get(n, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[n] = cnt.get(n, 0) + 1
end = max(int(r["End_Timestamp"]) for r in seq)
print(f"step span {(end - t0) / 1e3:.1f} us")
for n in sorted(tot, key=lambda k: -tot[k]):
    print(f"  {n:28s} {cnt[n]:5d} launches {tot[n]:9.1f} us")
tr = [r for r in seq if name(r) in ("trmm_pair_kernel", "finalize_kernel", "trmv_kernel",
                                    "trmv_part_kernel", "trmv_sum_kernel")]
first_trmv = min(int(r["Start_Timestamp"]) for r in tr)
last_fact = max(int(r["End_Timestamp"]) for r in seq if name(r).startswith(("chol_", "pp_")))
last_cross = max(int(r["End_Timestamp"]) for r in seq if name(r).startswith("cross_"))
print(f"  factorisation ends {(last_fact - t0) / 1e3:.1f} us, cross-covariance ends "
      f"{(last_cross - t0) / 1e3:.1f} us, prediction starts {(first_trmv - t0) / 1e3:.1f} us")
gap = 0
for a, b in zip(tr, tr[1:]):
    gap += max(0, int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
print(f"  prediction phase: {len(tr)} kernels, idle between them {gap / 1e3:.1f} us")
# the step period (Gram to Gram) and what runs between the last prediction kernel of one step
# and the Gram of the next
if len(starts) > 2:
    per = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
           for a, b in zip(starts, starts[1:])]
    print(f"  step period (step start to step start) us: min {min(per):.1f} median "
          f"{sorted(per)[len(per) // 2]:.1f} max {max(per):.1f} over {len(per)}")
    last_pred = max(int(r["End_Timestamp"]) for r in tr)
    nxt = rows[starts[-1]]
    print(f"  last prediction kernel end -> next step start: "
          f"{(int(nxt['Start_Timestamp']) - last_pred) / 1e3:.1f} us; between them:")
    for r in rows:
        s0 = int(r["Start_Timestamp"])
        if last_pred - 50000 <= s0 <= int(nxt["Start_Timestamp"]) and name(r) not in (
                "trmm_pair_kernel", "finalize_kernel"):
            print(f"    {name(r):28s} start {(s0 - last_pred) / 1e3:8.1f} us  dur "
                  f"{(int(r['End_Timestamp']) - s0) / 1e3:7.1f} us")
