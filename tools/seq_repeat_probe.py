#!/usr/bin/env python3
"""Why one sequence-leg repeat in four runs ~45% slower (tools/bench_sequence.py, profiles/r06/c4): the same timed
loop as bench_sequence.measure over N repeats, with the frontends (their yv_batch / yv_ba / window allocations)
either made right before each repeat (as the bench does) or all made before the first repeat. If the slow repeats
follow the allocation, not the position in time, the cause is where the buffers land.

    python tools/seq_repeat_probe.py [--frames 1000] [--repeats 9] [--mode new|precreate] [--gap-ms 0]
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--repeats", type=int, default=9)
    ap.add_argument("--mode", default="new", choices=("new", "precreate", "fixedstream", "torchnew"))
    ap.add_argument("--stress", type=int, default=0, help="torch streams made (and kept) before the frontends")
    ap.add_argument("--priority", type=int, default=0, help="the BA stream's priority (-1 high)")
    ap.add_argument("--gap-ms", type=float, default=0.0)
    a = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    from ya_vo_amd.sequence import SequenceFrontend
    from ya_vo_amd.synth import synth_sequence
    n, chunk = a.frames, 20
    fr = synth_sequence(1234, n, stereo=True)
    ctx = yv.Context(0)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    d = torch.from_numpy(fr.reshape(2 * n, *fr.shape[2:])).to("cuda:0")

    keep = [torch.cuda.Stream(device="cuda:0") for _ in range(a.stress)]
    fixed = torch.cuda.Stream(device="cuda:0", priority=a.priority) if a.mode == "fixedstream" else None

    def make():
        # new / precreate: the frontend's default BA stream (the context's side stream); torchnew: a fresh torch stream
        # per frontend (the round-5 default)
        s = torch.cuda.Stream(device="cuda:0", priority=a.priority) if a.mode == "torchnew" else fixed
        return SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT, expected_frames=n, ba_priority=a.priority,
                                ba_stream=s)

    def timed(fe):
        sec = {}
        gc.collect()
        gc.disable()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for c in range(n // chunk):
            fe.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk], sec)
        fe.flush(sec)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        gc.enable()
        return dt, sec

    fe = make()
    timed(fe)
    fe.close()
    pre = [make() for _ in range(a.repeats)] if a.mode == "precreate" else None
    out = []
    for r in range(a.repeats):
        fe = pre[r] if pre else make()
        dt, sec = timed(fe)
        out.append({"seconds": round(dt, 4), "ba": round(sec.get("ba", 0.0), 4)})
        if not pre:
            fe.close()
        if a.gap_ms > 0:
            time.sleep(a.gap_ms / 1e3)
    if pre:
        for fe in pre:
            fe.close()
    print(json.dumps({"mode": a.mode, "gap_ms": a.gap_ms, "priority": a.priority, "stress": a.stress,
                      "repeats": out}))
    del keep
    ctx.close()


if __name__ == "__main__":
    main()
