"""Per-kernel statistics from a rocprofv3 SQLite output (``*_results.db``): name, calls, total,
average (rocprofv3 --kernel-trace without --output-format csv writes only the database).
    python tools/rocdb_stats.py RUN_results.db [--csv OUT.csv] [--timeline OUT.txt]"""
import argparse
import csv
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--timeline", help="write every dispatch (start_us, dur_us, name)")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    kt = next((t for t in tabs if t.startswith("rocpd_kernel_dispatch")), None)
    if kt is None:
        kt = next(t for t in tabs if "kernel" in t.lower() and "dispatch" in t.lower())
    cols = [r[1] for r in con.execute(f"pragma table_info({kt})")]
    st = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol") or t == "rocpd_info_kernel_symbol")
    scols = [r[1] for r in con.execute(f"pragma table_info({st})")]
    namecol = "display_name" if "display_name" in scols else ("kernel_name" if "kernel_name" in scols else "name")
    q = (f"select s.{namecol}, k.start, k.end from {kt} k join {st} s on k.kernel_id = s.id "
         "order by k.start")
    rows = list(con.execute(q))
    agg = {}
    for name, s, e in rows:
        d = (e - s) / 1e3
        c = agg.setdefault(name, [0, 0.0, 0.0])
        c[0] += 1
        c[1] += d
        c[2] = max(c[2], d)
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for _, v in out)
    w = csv.writer(open(a.csv, "w") if a.csv else sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MaxUs", "Percentage"])
    for name, (n, t, mx) in out:
        w.writerow([name[:120], n, f"{t:.1f}", f"{t / n:.2f}", f"{mx:.2f}", f"{100 * t / tot:.2f}"])
    if a.timeline:
        t0 = rows[0][1] if rows else 0
        with open(a.timeline, "w") as f:
            for name, s, e in rows:
                f.write(f"{(s - t0) / 1e3:12.1f} {(e - s) / 1e3:10.1f} {name[:90]}\n")


if __name__ == "__main__":
    main()
