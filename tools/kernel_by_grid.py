"""Launches of one kernel in a rocprofv3 kernel trace, grouped by grid size: count, mean and median duration.
The bench's roofline kernel is detect's 4097-image launch; kernel_stats.csv averages every detect launch of the run
(the sequence leg's 40-image launches too), so the roofline's HIP-event time is compared with this breakdown.

    python tools/kernel_by_grid.py OUT/trace_kernel_trace.csv [detect_kernel]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "detect_kernel"
    by = defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if name not in k.split("(")[0]:
            continue
        grid = (int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) * int(r.get("Grid_Size_Y") or 1) *
                int(r.get("Grid_Size_Z") or 1))
        by[(k.split("(")[0].replace("void ", ""), grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for (k, grid), d in sorted(by.items(), key=lambda x: -len(x[1]) * statistics.mean(x[1])):
        print(f"  {k} grid {grid}: {len(d)} launches, mean {statistics.mean(d):.4f} ms, "
              f"median {statistics.median(d):.4f} ms")


if __name__ == "__main__":
    main()
