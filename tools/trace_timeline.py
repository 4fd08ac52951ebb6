"""Print a rocprofv3 kernel trace as a per-step timeline (start / end relative to the first kernel, in us), to see
which kernels overlap (e.g. the pose LM on the side stream beside the next step's image kernels).

    python tools/trace_timeline.py gpurun_out/prof/bench_kernel_trace.csv [--last 20]
"""
import csv
import sys


def short(name):
    n = name.split("(")[0]
    for k in ("detect", "topk", "brief", "match_finalize", "match", "track_build", "pose_lm", "map_", "copyBuffer",
              "fillBuffer", "elementwise"):
        if k in n:
            return k
    return n[-24:]


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 40
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{short(r['Kernel_Name']):>16} q{r['Queue_Id']} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
