"""Per-kernel duration summary of a rocprofv3 kernel trace: the rocpd SQLite database (ROCm 7 default output)
or a CSV kernel_stats file.  python tools/kt_summary.py DB_OR_CSV [--csv OUT]"""
import csv
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    disp = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    sym = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    names = {r[0]: r[1] for r in cur.execute(f"select id, kernel_name from {sym}")}
    d = defaultdict(list)
    for kid, s, e in cur.execute(f"select kernel_id, start, end from {disp}"):
        d[names.get(kid, str(kid))].append(e - s)
    return d


def main():
    d = from_db(sys.argv[1])
    rows = []
    for k, v in d.items():
        v = sorted(v)
        rows.append((sum(v), k, len(v), sum(v) / len(v), v[0], v[-1]))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    out = []
    for t, k, n, avg, mn, mx in rows:
        out.append({"Name": k, "Calls": n, "TotalDurationNs": t, "AverageNs": round(avg, 1), "Percentage": round(100 * t / tot, 2),
                    "MinNs": mn, "MaxNs": mx})
        print(f"{k[:70]:70s} {n:5d} avg {avg/1e6:8.4f} ms  min {mn/1e6:8.4f}  max {mx/1e6:8.4f}  {100*t/tot:5.1f}%")
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
