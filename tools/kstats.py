"""Print a rocprofv3 --stats kernel_stats.csv as a compact table (tools/kstats.py FILE [N])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f'{r["Name"][:64]:64s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1000:9.2f}us '
          f'{float(r["TotalDurationNs"]) / 1e6:8.3f}ms')
