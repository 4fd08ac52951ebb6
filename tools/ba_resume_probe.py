#!/usr/bin/env python3
"""How often the device LM of the configs[2] window solves suspends and is resumed from the host
(yv_ba_debug_resumes), per BA iteration budget: python tools/ba_resume_probe.py [--frames 60] [--chunk 20]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--chunk", type=int, default=20)
    ap.add_argument("--seed", type=int, default=71)
    a = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    from ya_vo_amd.sequence import SequenceFrontend
    from ya_vo_amd.synth import synth_sequence
    T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
    fr = synth_sequence(a.seed, a.frames, stereo=True)
    ctx = yv.Context(0)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8))
    d = torch.from_numpy(fr.reshape(2 * a.frames, *fr.shape[2:])).to("cuda:0")
    for iters in (10, 20, 40):
        fe = SequenceFrontend(ctx, a.chunk, scene.K_KITTI, T_RIGHT, ba_iters=iters)
        for c in range(a.frames // a.chunk):
            fe.process_chunk(d[2 * c * a.chunk:2 * (c + 1) * a.chunk])
        fe.flush()
        print(f"frames {a.frames} chunk {a.chunk} ba_iters {iters}: resumes {fe.ba.resumes()}, "
              f"iterations run {[x[1] for x in fe.ba_log]}", flush=True)
        fe.close()


if __name__ == "__main__":
    main()
