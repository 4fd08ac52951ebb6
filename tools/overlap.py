"""Per-kernel durations from a rocprofv3 kernel-trace CSV, split by whether another queue's kernel overlapped the
launch: python tools/overlap.py <kernel_trace.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pats = sys.argv[2:]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows]
    ks.sort()
    stats = defaultdict(lambda: [[], []])
    for i, (s, e, q, n) in enumerate(ks):
        short = n.split("(")[0][-48:]
        if pats and not any(p in n for p in pats):
            continue
        ov = any(s2 < e and e2 > s and q2 != q for (s2, e2, q2, _) in ks[max(0, i - 200):i + 200] if (s2, e2) != (s, e))
        stats[short][1 if ov else 0].append((e - s) / 1000.0)
    for k, (a, b) in sorted(stats.items(), key=lambda kv: -sum(kv[1][0]) - sum(kv[1][1])):
        f = lambda v: f"{len(v):5d} x {sum(v) / len(v):8.2f} us" if v else f"{0:5d}" + " " * 14
        print(f"{k:50s} alone {f(a)}   overlapped {f(b)}")


if __name__ == "__main__":
    main()
