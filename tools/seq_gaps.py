#!/usr/bin/env python3
"""Where a configs[2] chunk's time goes without a profiler attached (rocprofv3's per-dispatch signals throttle the
host's run-ahead and move the picture): HIP events recorded on the BA stream and the context stream around each host
call of SequenceFrontend's device-window loop, plus host clocks, printed per chunk.

    python tools/seq_gaps.py [--frames 200] [--chunk 20] [--out gpurun_out/seq_gaps.json]

Per chunk c (GPU clock, ms relative to the chunk's issue):
  fe_start / fe_end    the context stream reaching this chunk's front end / its end (events before / after issue)
  ba_prev_end          the previous window's solve done on the BA stream
  ba_start / ba_end    the BA stream reaching this chunk's begin (enqueue time: the stream is idle then) / done
and the host seconds of each call (issue, end, place_record, begin)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--chunk", type=int, default=20)
    ap.add_argument("--reserve", type=int, default=1)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    from ya_vo_amd.sequence import SequenceFrontend
    from ya_vo_amd.synth import synth_sequence

    n, chunk = a.frames, a.chunk
    fr = synth_sequence(1234, n, stereo=True)
    H, W = fr.shape[2:]
    offsets = np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8)
    ctx = yv.Context(0)
    ctx.set_brief_offsets(offsets)
    d = torch.from_numpy(fr.reshape(2 * n, H, W)).to("cuda:0")
    T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
    cs = torch.cuda.ExternalStream(ctx.stream)

    def run(record):
        fe = SequenceFrontend(ctx, chunk, scene.K_KITTI, T_RIGHT, H=H, W=W,
                              expected_frames=n if a.reserve else 0)
        ev, host = [], []
        torch.cuda.synchronize()
        t00 = time.perf_counter()
        for c in range(n // chunk):
            e = {k: torch.cuda.Event(enable_timing=True) for k in
                 ("fe_start", "fe_end", "ba_prev_end", "ba_start", "ba_end")}
            h = {}
            t0 = time.perf_counter()
            e["fe_start"].record(cs)
            first = fe.next_frame
            fe.batch.run(d[2 * c * chunk:2 * (c + 1) * chunk].data_ptr(), 2 * chunk, fe.W, fe.H * fe.W,
                         fe.match_thr, carry_from=2 * (chunk - 1))
            fe.batch.track_map(fe.d_prior.data_ptr(), fe.d_poses.data_ptr(), first, 1, fe.d_block.data_ptr(), chunk)
            e["fe_end"].record(cs)
            t1 = time.perf_counter()
            if fe._ba_pending:
                fe._local_ba_device_end()
            e["ba_prev_end"].record(fe.ba_stream)
            t2 = time.perf_counter()
            ctx.map_place(fe.d_block.data_ptr(), 1, fe.bb, fe.d_base.data_ptr(), fe.d_anchors.data_ptr())
            v = fe.batch.view()
            fe.win.add_block(fe.d_block.data_ptr(), first, chunk, v.edge_uv, v.edge_query, v.matches, fe.max_kp)
            fe.next_frame = first + chunk
            t3 = time.perf_counter()
            e["ba_start"].record(fe.ba_stream)
            fe._local_ba_device_begin()
            e["ba_end"].record(fe.ba_stream)
            t4 = time.perf_counter()
            h = {"issue": t1 - t0, "end": t2 - t1, "place_record": t3 - t2, "begin": t4 - t3}
            ev.append(e)
            host.append(h)
        fe.flush()
        torch.cuda.synchronize()
        total = time.perf_counter() - t00
        fe.close()
        return total, ev, host

    run(False)
    total, ev, host = run(True)
    ref = ev[0]["fe_start"]
    rows = []
    for c, (e, h) in enumerate(zip(ev, host)):
        r = {k: round(ref.elapsed_time(x), 3) for k, x in e.items()}
        r.update({"host_" + k: round(1e3 * v, 3) for k, v in h.items()})
        rows.append(r)
    print(f"total {1e3 * total:.2f} ms for {n} frames = {n / total:.0f} frames/s")
    print("chunk  fe_start  fe_end  ba_prev_end  ba_start  ba_end | host issue end place begin (ms)")
    for c, r in enumerate(rows):
        print(f"{c:5d} {r['fe_start']:9.3f} {r['fe_end']:7.3f} {r['ba_prev_end']:11.3f} {r['ba_start']:9.3f} "
              f"{r['ba_end']:7.3f} | {r['host_issue']:.3f} {r['host_end']:.3f} {r['host_place_record']:.3f} "
              f"{r['host_begin']:.3f}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"total_s": total, "frames": n, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
