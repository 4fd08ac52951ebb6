"""Summarize rocprofv3 counter_collection CSVs (last dispatch of the kernel): python tools/pmc_summary.py FILES..."""
import collections
import csv
import sys

for f in sys.argv[1:]:
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        d[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    last = max(d)
    print(f, "dispatches", len(d))
    for k, v in sorted(d[last].items()):
        print(f"   {k:28s} {v:.4g}")
