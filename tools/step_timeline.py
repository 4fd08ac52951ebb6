"""Per-stream timeline of the bench's timed steps from a rocprofv3 kernel trace ('step timeline').

    rocprofv3 --kernel-trace --output-format csv -d OUT -o trace -- python bench.py --steps 5 ... ;
    python tools/step_timeline.py OUT/trace_kernel_trace.csv [--step N]

A step is delimited by consecutive launches of detect_kernel (the first kernel of the main stream's chain). Prints,
for the chosen step, every kernel with its queue, start / end relative to the step's detect start, and the busy time
per queue; then, over all whole steps, the mean step length and each queue's mean busy time inside a step."""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2, help="which step to print (python index over whole steps)")
    ap.add_argument("--anchor", default="detect_kernel")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                 r["Kernel_Name"].split("(")[0].split("::")[-1].replace("void ", "")) for r in rows)
    anchors = [k for k in ks if k[3].startswith(args.anchor)]
    qmain = anchors[0][2]
    anchors = [k for k in anchors if k[2] == qmain]
    steps = list(zip(anchors, anchors[1:]))
    if not steps:
        print("fewer than two anchor launches")
        return
    a, b = steps[args.step]
    t0, t1 = a[0], b[0]
    print(f"step {args.step}: {(t1 - t0) / 1000:.1f} us (detect to next detect on queue {qmain})")
    busy = defaultdict(float)
    for s, e, q, n in ks:
        if e <= t0 or s >= t1:
            continue
        ov = (min(e, t1) - max(s, t0)) / 1000
        busy[q] += ov
        print(f"  q{q:>2} {(s - t0) / 1000:9.1f} .. {(e - t0) / 1000:9.1f}  {(e - s) / 1000:8.1f} us  {n}")
    print("busy per queue inside the step (us):", {q: round(v, 1) for q, v in sorted(busy.items())})
    lens, tot = [], defaultdict(float)
    for a, b in steps:
        t0, t1 = a[0], b[0]
        lens.append((t1 - t0) / 1000)
        for s, e, q, n in ks:
            if e > t0 and s < t1:
                tot[q] += (min(e, t1) - max(s, t0)) / 1000
    m = len(steps)
    print(f"over {m} steps: mean {sum(lens) / m:.1f} us;", "mean busy per queue:",
          {q: round(v / m, 1) for q, v in sorted(tot.items())})


if __name__ == "__main__":
    main()
