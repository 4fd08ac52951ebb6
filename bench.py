#!/usr/bin/env python3
"""Benchmark of the YA_VO front-end hot path on MI355X (BASELINE.json configs[1]).

A step = one pass of the hot path over one resident batch of B synthetic 1241x376 stereo frames per GPU:
for every frame, FAST-12 + Harris + top-2000 and blur + BRIEF on the left and right images, Hamming
matching L_{k-1} -> L_k (the reference's temporal matchFeatures, src/LoopHandler.cc:189,534) and L_k -> R_k
(stereo), removeOutliers(20) on both match lists, then PnP: the kept stereo matches are triangulated
(LoopHandler::triangulation) and the pose-only LM (LoopHandler::optimizePoseOnly) solves every frame's pose
from the kept temporal matches, and the chunk's shared-map block (keyframe poses + LM-inlier landmarks,
include/yavo/yavo_map.h) is written after the LM.  `value` = stereo frames per second over all GPUs
(max-over-ranks wall time).  One process per GPU; ONE sequence shards across ranks (weak scaling): rank r owns
frames [1 + rB, 1 + (r+1)B) and detects / describes its predecessor frame rB in the same run (the 1-frame halo,
ya_vo_amd.sharding.FrameShard), so no image stage communicates.  The only
collective is the shared map's: every step the ranks all-gather their map blocks (RCCL over xGMI) on a
communication stream and place them in world coordinates, overlapped with the next step's image kernels.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

H, W = 376, 1241
MAX_KP = 2000
T_RIGHT = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)  # stereo right camera, KITTI baseline 0.54 m
METRIC = "frames/sec (detect+describe+match+PnP) on 1241×376 KITTI stereo; RMSE vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP4_MFMA_PEAK_TOPS = 10000.0  # dense FP4 MFMA peak (MI355X_MICROARCH.md; no sparsity): the matcher runs on
# v_mfma_scale_f32_16x16x128_f8f6f4 with FP4 operands (max_kp <= 2048)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-op/s
# FP64 vector peak (AMD MI355X spec, 78.6 TFLOP/s: 16 FP64 FMA lanes per SIMD per clock, so one wave64 FP64
# instruction issues in 4 cycles); the MI355X guide does not list FP64
FP64_PEAK_TFLOPS = 256 * 4 * 16 * 2 * 2.4e9 / 1e12
SIMD_CYCLES_PER_S = 256 * 4 * 2.4e9


def kernel_source_digest() -> str:
    """sha256 over the product's kernel and ABI sources (ya_vo_amd/csrc, include/yavo): the stamp tying
    profiles/pmc_traffic.json's counters to the code they were measured on."""
    import hashlib
    h = hashlib.sha256()
    files = []
    for d, exts in ((os.path.join(ROOT, "ya_vo_amd", "csrc"), (".hip", ".h")), (os.path.join(ROOT, "include", "yavo"), (".h",))):
        files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=2048,
                    help="stereo frames per step per GPU (2048: eight pose-LM problems per CU, four rounds; r03 measured "
                         "214k / 219k / 221k frames/s at 1024 / 1536 / 2048 on one box, profiles/r03/c51)")
    ap.add_argument("--cpu-baseline", choices=["both", "literal", "efficient", "none"], default="both")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads of the CPU baseline (0: the usable cores, affinity capped by OMP_NUM_THREADS)")
    ap.add_argument("--literal-frames", type=int, default=20, help="frames of the ref-literal CPU sample")
    ap.add_argument("--no-timing", action="store_true", help="do not record per-stage HIP events")
    ap.add_argument("--stage-steps", type=int, default=5,
                    help="steps of the separate per-stage pass after the timed region (events around every stage)")
    ap.add_argument("--no-overlap", action="store_true", help="run the pose LM in order on the main stream")
    ap.add_argument("--overlap-mode", type=int, default=1, choices=[1, 2, 3, 4],
                    help="pose LM beside the next step: 1 after the edge build, 2 / 3 / 4 after the next detect / "
                         "describe / top-K")
    ap.add_argument("--tracker", choices=["match", "lk"], default="match",
                    help="PnP correspondences: BRIEF temporal matches (default) or calcOpticalFlowPyrLK of frame "
                         "k-1's stereo map points (the reference's trackLastFrame)")
    ap.add_argument("--e2e-steps", type=int, default=20,
                    help="steps of the end-to-end leg (every step's frames uploaded from pinned host memory, "
                         "overlapped with the previous step's kernels); 0 skips it")
    ap.add_argument("--png-steps", type=int, default=6,
                    help="steps of the PNG-input end-to-end leg (rank 0, N=1): the step's frames written once as a "
                         "KITTI stereo sequence of PNG files, every step decoded on the host threads (cv::imread's "
                         "part, yv_seq_upload) into pinned staging and copied to HBM, overlapped with the previous "
                         "step's kernels; 0 skips it")
    ap.add_argument("--png-threads", type=int, default=0, help="decode threads of the PNG leg (0: the usable cores)")
    ap.add_argument("--loop-handler-frames", type=int, default=200,
                    help="frames of the drop-in C++ LoopHandler leg (rank 0, N=1; tools/bench_loop_handler.py); 0 "
                         "skips it")
    ap.add_argument("--collective-world1", action="store_true",
                    help="at N=1, still run the shared-map exchange through a 1-rank process group (RCCL)")
    ap.add_argument("--sequence-frames", type=int, default=1000,
                    help="frames of the configs[2] leg's timed runs (rank 0, N=1; median of 5): the full front end "
                         "with the local BA window (tools/bench_sequence.py); after them the first 200 frames are "
                         "compared with the CPU oracle loop; 0 skips it")
    ap.add_argument("--sequence-cpu", type=int, default=1,
                    help="1: run tests/sequence_chain.py (the same loop over the CPU oracle) for the sequence leg's "
                         "trajectory check; 0: skip it")
    ap.add_argument("--kf-every", type=int, default=4,
                    help="shared map: frames with global index %% kf_every == 0 are keyframes (their LM inliers "
                         "become landmarks); 0 disables the map and its all-gather")
    return ap.parse_args()


def stage_bytes(counts, n_img):
    """Algorithmic HBM bytes per launch of each stage over n_img images (DESIGN.md 'Algorithmic bytes')."""
    img = H * W
    cand = float(np.sum(counts["cand"][:n_img]))
    det = float(np.sum(counts["det"][:n_img]))
    kp = float(np.sum(counts["kp"][:n_img]))
    nq = float(np.sum(counts["match"]))
    nf = float(np.sum(counts["filt"]))
    return {
        # image read once, blurred image written once, candidate keys (8 B) appended
        "detect": 2 * n_img * img + 8 * cand,
        # candidate keys read once; (row, col) + response + kp_src written
        "topk": 8 * cand + 12 * det + 16 * kp,
        # blurred image read once; 48-B KeyPoint + 32-B descriptor written per keypoint
        "brief": n_img * img + 80 * kp,
        # query + train descriptors read, 4-B match key written per query
        "match": 2 * 32 * nq + 4 * nq,
        # keys + query records read, 100-B Matches written (all + filtered) + 8-B {dist, j} per query
        "finalize": (4 + 48) * nq + 100 * (nq + nf) + 8 * nq,
        # per temporal query: 2 x {dist, j}; per edge: 3 keypoint (x, y) reads, X + uv + query index written
        "track_edges": 16 * counts["tq"] + (24 + 44) * counts["edges"],
        # per edge: X + uv read, outlier flag written (the LM iterates on these; it is latency bound)
        "track_pose": 41 * counts["edges"],
    }


def stage_valu_ops(counts, n_img):
    """Algorithmic lane-operations of the VALU-bound stages, SURVEY.md 8(d)'s per-unit figures."""
    kq = counts["match"].astype(np.float64)
    kt = counts["train"].astype(np.float64)
    # detect: FAST P * (16 abs-diff-compare + run scan) = 36 M lane-ops per image + the 9x9
    # separable blur, 9 + 9 MACs per pixel
    # matcher (VALU formulation): Kq * Kt * (8 xor + 8 bcnt-accumulate + 2 min) = 18 per pair
    return {"detect": n_img * (36.0e6 + 18.0 * H * W), "match": float(np.sum(kq * kt)) * 18.0}


def write_png_sequence(base, left, right, threads):
    """KITTI layout: base/image_0/%06d.png (left), image_1 (right) and a calib.txt."""
    from concurrent.futures import ThreadPoolExecutor
    for side in ("image_0", "image_1"):
        os.makedirs(os.path.join(base, side), exist_ok=True)
    jobs = [(os.path.join(base, side, f"{k:06d}.png"), imgs[k]) for side, imgs in (("image_0", left), ("image_1", right))
            for k in range(len(imgs))]

    from ya_vo_amd.io import png_write_gray

    def write(j):
        png_write_gray(j[0], j[1])  # Sub rows, deflate level 1 + Z_RLE as cv::imwrite; ctypes releases the GIL
    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(write, jobs))
    with open(os.path.join(base, "calib.txt"), "w") as f:
        for i in range(2):
            f.write(f"P{i}: 7.188560e+02 0 6.071928e+02 {-386.1448 * i:.6e} 0 7.188560e+02 1.852157e+02 0 0 0 1 0\n")


def png_end_to_end(ctx, shard, images, halo_right, B, steps, threads, gpu_decode=True):
    """PNG-input end-to-end rate: the shard's frames as a KITTI stereo PNG sequence (sequence frame 0 =
    the halo frame, 1..B = the shard).  gpu_decode: every step the files are read by `threads` host threads straight
    into pinned staging, copied up compressed and decoded by the inflate / unfilter kernels on the context stream
    (yv_seq_upload_gpu); otherwise decoded on the host threads into pinned staging and copied up (yv_seq_upload).
    Either way the host prepares step i + 1 while the GPU runs step i.  Timed: every read, decode, copy and step."""
    import shutil
    import tempfile
    import torch
    from ya_vo_amd.io import PngDecoder, Sequence
    tmp = tempfile.mkdtemp(prefix="yavo_png_")
    try:
        t0 = time.perf_counter()
        left = [images[2 * B]] + [images[2 * k] for k in range(B)]
        right = [halo_right] + [images[2 * k + 1] for k in range(B)]
        write_png_sequence(tmp, left, right, threads)
        write_s = time.perf_counter() - t0
        png_bytes = sum(os.path.getsize(os.path.join(tmp, d, f)) for d in ("image_0", "image_1")
                        for f in os.listdir(os.path.join(tmp, d)))
        seq = Sequence(tmp, stereo=True)
        dev = torch.device("cuda", ctx.device)
        img = H * W
        bufs = [torch.empty((2 * B + 2) * img, dtype=torch.uint8, device=dev) for _ in range(2)]
        dec = PngDecoder(ctx, 2 * B + 2, H, W) if gpu_decode else None

        def upload(k):
            if dec is not None:  # one decode: frames 1..B -> images 0 .. 2B-1, the halo frame 0 -> 2B, 2B + 1
                dec.upload_frames(seq, list(range(1, B + 1)) + [0], bufs[k].data_ptr(), img, threads)
                return
            seq.upload(ctx, 1, B, bufs[k].data_ptr(), img, threads)              # frames -> images 0 .. 2B-1
            seq.upload(ctx, 0, 1, bufs[k].data_ptr() + 2 * B * img, img, threads)  # halo frame -> 2B (+ its right)

        for i in range(4 if dec is not None else 1):  # warm-up: the decoder's four staging slots get allocated
            upload(i % 2)
            shard.step(bufs[i % 2].data_ptr())
        shard.drain()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(steps):
            upload(i % 2)  # the context stream orders it after step i - 2's kernels, the last readers of the buffer
            shard.step(bufs[i % 2].data_ptr())
        shard.drain()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        res = {"frames_per_s": round(B * steps / el, 2), "ms_per_step": round(1e3 * el / steps, 3), "steps": steps,
               "host_threads": threads, "png_bytes_per_stereo_frame": round(png_bytes / (B + 1)),
               "png_write_s": round(write_s, 2)}
        if dec is not None:
            codes, bad = dec.status()
            # the decoded images are the step's frames: the pipeline's inputs came through the PNG files intact
            res["decode_errors"] = int(bad)
            res["images_bit_identical"] = bool(np.array_equal(
                bufs[(steps - 1) % 2][:2 * B * img].cpu().numpy(), images[:2 * B].reshape(-1)))
            # the decode alone (read + inflate + unfilter), GPU idle otherwise
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            dec.upload_sequence(seq, 1, B, bufs[0].data_ptr(), img, threads)
            dec.status()
            res["decode_only_frames_per_s"] = round(B / (time.perf_counter() - t2), 2)
            res["how"] = ("KITTI stereo PNG sequence written as cv::imwrite does (Sub rows, deflate level 1, Z_RLE) -> "
                          "yv_seq_upload_gpu (host threads read the files into pinned staging, the IDAT streams go up "
                          "compressed, inflate + unfilter kernels on the context stream) -> the step's kernels; the "
                          "host reads step i+1 while the GPU runs step i; timed region = every read + copy + decode + "
                          "step")
            dec.close()
        else:
            t2 = time.perf_counter()
            seq.read(1, B, threads)
            res["decode_only_frames_per_s"] = round(B / (time.perf_counter() - t2), 2)
            res["how"] = ("the same files -> yv_seq_upload (host decode threads -> pinned staging -> async HBM copy on "
                          "the context stream) -> the step's kernels")
        seq.close()
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def loop_handler_leg(frames):
    """The drop-in C++ LoopHandler (ya_vo_amd/bin/yavo_loop_handler) on a synthetic mono PNG sequence, serial and
    pipelined (tools/bench_loop_handler.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_loop_handler
    r = bench_loop_handler.measure(frames, readers=min(16, cpu_threads_available()))
    return {"serial_frames_per_s": r["serial"]["frames_per_s"], "pipelined_frames_per_s": r["pipelined"]["frames_per_s"],
            "trajectories_identical": r["trajectories_identical"], "serial": r["serial"], "pipelined": r["pipelined"],
            "pipelined_modes": r["pipelined_modes"], "what": r["what"]}


def cpu_threads_available() -> int:
    """Host cores this process may use: its affinity mask, capped by OMP_NUM_THREADS (the GPU box sets it to the
    CPU share of one GPU, 16; os.cpu_count() there reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def cpu_baseline(kind, threads, offsets, images, B, gpu_poses, edges, literal_frames=20):
    """Oracle (CPU restatement of the reference) on the GPU box's host cores, on bounded samples of the SAME frames
    the GPU processed.  images: the shard layout (L_k, R_k interleaved, then the halo frame's left image at 2B).

    literal:   the reference's costs (per-pixel ring rebuild, three whole-image products per corner, bit-loop
               popcount), one thread per frame; `literal_frames` frames run concurrently on `threads` cores and the
               median frame time is reported (value = 1 / median).
    efficient: the same outputs (local Harris sums, precomputed ring), `threads` threads over frames.
    Both report per-stage milliseconds per frame (FAST+Harris, blur+BRIEF, match+removeOutliers, triangulation,
    pose LM; the timers of src/FastDetector.cc:289,336-349 and src/LoopHandler.cc:471-482 split the same way).
    pose_check: the GPU's relative poses against the CPU chain (bit-identity in the kernel's edge-sum order on the
    sample frames) and, over EVERY frame of the step, the pose LM on the GPU's edges in the reference's sequential
    sum order (sum_mode 0): the metric's "RMSE vs CPU ref"."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind
    from track_chain import track_pose
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    orc = oracle_bind.Oracle()

    def prev_image(k):
        return images[2 * B] if k == 0 else images[2 * (k - 1)]

    def left_kp(img):
        return orc.brief(img, orc.fast(img, MAX_KP)[0], offsets)

    def one_frame(k, prev_left_kp, mode):
        """Frame k (track k): detect+describe L_k, R_k; temporal + stereo matches; triangulation; pose LM.  The
        F-RANSAC of (re)initialisation is timed on the frame's kept temporal matches too, outside the frame time."""
        timers, init_timers = {}, {}
        t_start = time.perf_counter()
        kps = []
        for img in images[2 * k:2 * k + 2]:
            t0 = time.perf_counter()
            rc, _, _ = orc.fast(img, MAX_KP, mode=mode)
            t1 = time.perf_counter()
            kps.append(orc.brief(img, rc, offsets))
            t2 = time.perf_counter()
            timers["fast_harris"] = timers.get("fast_harris", 0.0) + t1 - t0
            timers["blur_brief"] = timers.get("blur_brief", 0.0) + t2 - t1
        T = track_pose(orc, prev_left_kp, kps[0], kps[1], scene.K_KITTI, T_RIGHT, timers=timers,
                       init_timers=init_timers, n_tracks=B)[3]  # the batch's LM order for B tracks
        timers.update({"f_ransac_init": init_timers.get("f_ransac", 0.0)})
        return T, time.perf_counter() - t_start - timers["f_ransac_init"], timers

    def stage_table(results):
        # f_ransac_init: getFRANSAC (400 hypotheses) on the frame's kept temporal matches, the reference's
        # (re)initialisation stage (src/LoopHandler.cc:225,567); not part of the per-frame time
        keys = ("fast_harris", "blur_brief", "match", "triangulate", "pose_lm", "f_ransac_init")
        return {key: round(1e3 * float(np.mean([r[2].get(key, 0.0) for r in results])), 3) for key in keys}

    res, cpu_poses = {}, {}
    if kind in ("both", "literal"):
        n = min(literal_frames, B)
        prevs = [left_kp(prev_image(k)) for k in range(n)]  # frame k-1's keypoints, as the reference carries them
        t0 = time.perf_counter()
        with ThreadPoolExecutor(min(threads, n)) as ex:  # ctypes releases the GIL inside the oracle
            out = list(ex.map(lambda k: one_frame(k, prevs[k], 0), range(n)))
        wall = time.perf_counter() - t0
        per = np.array([r[1] for r in out])
        for k, r in enumerate(out):
            cpu_poses[k] = r[0]
        # the same chain for frames 0 and 1 again, one after the other on one thread with nothing else running: the
        # single-core rate without the concurrent sample's shared-memory-bandwidth contention
        iso = [one_frame(k, prevs[k], 0)[1] for k in range(min(2, n))]
        iso_s = float(np.mean(iso))
        res["literal"] = {"value": 1.0 / iso_s, "unit": "frames/s", "cores": 1, "kind": "port",
                          "sample": f"frames 0..{len(iso) - 1} of the benchmarked shard (detect+describe L,R; match "
                                    "L_{k-1}->L_k, L_k->R_k; removeOutliers; triangulation; pose LM) with the "
                                    "reference's costs: per-pixel ring rebuild, three whole-image products per corner "
                                    "(src/FastDetector.cc:249-251), bit-loop popcount; one thread, the frames run one "
                                    "after the other with nothing else on the host, value = 1 / mean frame time",
                          "isolated_frame_s": [round(x, 4) for x in iso],
                          "concurrent_sample": f"frames 0..{n - 1}, one thread per frame, {n} frames run concurrently "
                                               f"on {min(threads, n)} cores",
                          "median_frame_s": round(float(np.median(per)), 4),
                          "min_frame_s": round(float(per.min()), 4), "max_frame_s": round(float(per.max()), 4),
                          "frames": n, "wall_s": round(wall, 3), "stages_ms_per_frame": stage_table(out)}
    if kind in ("both", "efficient"):
        n = min(2 * threads, B)
        prevs = [left_kp(prev_image(k)) for k in range(n)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            out = list(ex.map(lambda k: one_frame(k, prevs[k], 1), range(n)))
        dt = time.perf_counter() - t0
        for k, r in enumerate(out):
            cpu_poses[k] = r[0]
        res["efficient"] = {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
                            "sample": f"frames 0..{n - 1} of the benchmarked shard, same outputs with local Harris "
                                      f"sums and a precomputed ring, {threads} threads over frames",
                            "seconds": round(dt, 3), "stages_ms_per_frame": stage_table(out)}
    # the full chain also on a block in the middle of the step and on its last 16 frames (images up to 4096: the
    # device buffers' offsets there are far past 2^31 bytes), efficient mode (same outputs)
    extra = sorted((set(range(max(B // 2 - 8, 0), min(B // 2 + 8, B))) | set(range(max(B - 16, 0), B))) - set(cpu_poses))
    if extra:
        prevs_x = {k: left_kp(prev_image(k)) for k in extra}
        with ThreadPoolExecutor(threads) as ex:
            out_x = list(ex.map(lambda k: one_frame(k, prevs_x[k], 1), extra))
        for k, r in zip(extra, out_x):
            cpu_poses[k] = r[0]
    ks = sorted(cpu_poses)
    same = bool(np.array_equal(np.array([gpu_poses[k] for k in ks]), np.array([cpu_poses[k] for k in ks])))
    runs, start = [], None
    for i, k in enumerate(ks):
        if start is None:
            start = k
        if i + 1 == len(ks) or ks[i + 1] != k + 1:
            runs.append(f"{start}..{k}")
            start = None
    # every frame of the step: the oracle's pose LM on the GPU's own edges, in the kernel's order (must reproduce the
    # GPU pose bit for bit) and in the reference's sequential order (the metric's RMSE)
    ec, eX, euv = edges
    prior = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)

    def both_orders(k):
        X, uv = eX[k, :ec[k]], euv[k, :ec[k]]
        return (orc.pose_lm(X, uv, scene.K_KITTI, prior, yv.track_lm_sum_mode(len(ec)))[0],
                orc.pose_lm(X, uv, scene.K_KITTI, prior, 0)[0])

    with ThreadPoolExecutor(threads) as ex:
        lm = list(ex.map(both_orders, range(len(ec))))
    gpu_order = np.array([x[0] for x in lm])
    seq_order = np.array([x[1] for x in lm])
    d = gpu_poses - seq_order
    # the same LMs with the host C library's pow / sin / cos (as g2o / Sophus call them) instead of the restated
    # functions the kernels share: how many of the step's poses the substitution moves, and by how much
    orc.set_libm_flavour(1)
    try:
        with ThreadPoolExecutor(threads) as ex:
            libm = np.array(list(ex.map(
                lambda k: orc.pose_lm(eX[k, :ec[k]], euv[k, :ec[k]], scene.K_KITTI, prior, yv.track_lm_sum_mode(len(ec)))[0],
                range(len(ec)))))
    finally:
        orc.set_libm_flavour(0)
    dl = gpu_poses - libm
    res["pose_check"] = {
        "frames": len(ec),
        "pose_rmse_vs_cpu_ref": float(np.sqrt(np.mean(np.sum(d[:, 4:] ** 2, axis=1)))),
        "max_abs_diff_vs_cpu_ref": float(np.abs(d).max()),
        "cpu_ref": "oracle pose LM (optimizePoseOnly) in the reference's sequential edge order (sum_mode 0) on the "
                   "GPU's edges, every frame of the step",
        "bit_identical_gpu_order_all_frames": bool(np.array_equal(gpu_poses, gpu_order)),
        "host_libm_flavour": {"poses_differing": int(np.sum(~np.all(dl == 0, axis=1))),
                              "max_abs_diff": float(np.abs(dl).max()),
                              "what": "oracle pose LM on the GPU's edges, kernel sum order, with glibc's pow / sin / "
                                      "cos (the reference's g2o / Sophus calls) instead of the restated ones"},
        "chain_frames": len(ks),
        "chain_frame_ranges": runs,
        "chain_bit_identical": same,
        "chain": "full CPU chain (detect .. pose LM) vs the GPU, kernel sum order: the cpu_baseline sample frames, a "
                 "16-frame block in the middle of the step and its last 16 frames"}
    return res


def launch_plan(n_gpus, environ, device_count, backend):
    """Rank environments for `bench.py --gpus N` started without a launcher (no WORLD_SIZE in the environment): one
    fresh child process per GPU, each told its RANK / LOCAL_RANK / WORLD_SIZE and the rendezvous on 127.0.0.1.
    Returns None when this process is itself the only rank (N = 1 or a launcher already set WORLD_SIZE).  Raises
    ValueError when the request cannot be honoured: RCCL ("nccl") needs one visible device per rank; the gloo rehearsal
    may place several ranks on one device (device = local rank modulo the visible devices)."""
    if n_gpus < 1:
        raise ValueError(f"--gpus must be >= 1 (got {n_gpus})")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n_gpus and n_gpus != 1:
            raise ValueError(f"--gpus {n_gpus} but the launcher set WORLD_SIZE={ws}")
        return None
    if n_gpus == 1:
        return None
    if backend == "nccl" and device_count < n_gpus:
        raise ValueError(f"--gpus {n_gpus} needs {n_gpus} visible GPUs for RCCL, {device_count} visible")
    if device_count < 1:
        raise ValueError("no visible GPU")
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    plans = []
    for r in range(n_gpus):
        env = dict(environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n_gpus), "LOCAL_WORLD_SIZE": str(n_gpus),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes on this host)
        plans.append(env)
    return plans


def spawn_ranks(plans, argv, script=None):
    """Run one child per rank environment (this script again, same arguments), rank 0's stdout passed through (it prints
    the JSON line), the other ranks' stdout sent to stderr.  Waits for all; if any rank fails the others are stopped
    (by their own PIDs) and its exit code is returned."""
    import subprocess
    procs = []
    for env in plans:
        out = None if env["RANK"] == "0" else sys.stderr
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env, stdout=out))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    backend = os.environ.get("YAVO_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` without torchrun: one fresh process per GPU, started before this process touches the GPU
        # (counting devices does not initialise the runtime on this image)
        import torch
        try:
            plans = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), backend)
        except ValueError as e:
            print(f"bench.py: {e}", file=sys.stderr)
            sys.exit(2)
        sys.exit(spawn_ranks(plans, sys.argv[1:]))
    elif "WORLD_SIZE" in os.environ:
        try:
            launch_plan(args.gpus, os.environ, 0, backend)
        except ValueError as e:
            print(f"bench.py: {e}", file=sys.stderr)
            sys.exit(2)
    import torch
    import torch.distributed as dist
    import ya_vo_amd as yv
    from ya_vo_amd import map as ymap
    from ya_vo_amd import scene
    from ya_vo_amd.sharding import FrameShard, shard_images
    from ya_vo_amd.synth import synth_stereo_batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL ("nccl"); YAVO_BENCH_BACKEND=gloo rehearses the multi-rank logic with
    # several ranks sharing fewer GPUs (device = local rank modulo the visible devices)
    dev_index = local_rank % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(dev_index)
        dist.init_process_group(backend)
    elif args.collective_world1:
        # a 1-rank group: the shared-map exchange then runs the N > 1 path (the RCCL all-gather on its stream)
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(port))
        torch.cuda.set_device(dev_index)
        dist.init_process_group(backend, rank=0, world_size=1)
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)

    offsets = np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"), np.int8)
    ctx = yv.Context(dev_index)
    ctx.set_brief_offsets(offsets)
    B = args.frames
    # one sequence (one synthetic field) sharded over the ranks: rank r owns frames
    # [1 + r B, 1 + (r + 1) B) and recomputes its predecessor frame r B (the 1-frame halo) in the same run, so its
    # first temporal pair is the sequence's own L_{rB} -> L_{rB+1}; frame 0 is the sequence's first (no predecessor)
    first = 1 + rank * B
    fr = synth_stereo_batch(1234, B + 1, start=first - 1)  # [2(B+1), H, W]: the halo frame, then the shard
    images = shard_images(fr[2:], fr[0], fr[1] if args.tracker == "lk" else None)
    halo_right = fr[1].copy()
    del fr
    n_img = images.shape[0]
    d_frames = torch.from_numpy(images).to(dev)
    use_map = args.kf_every > 0 and args.tracker == "match"
    max_kf = max(ymap.max_keyframes(B, 1 + r * B, args.kf_every) for r in range(world)) if use_map else 0
    shard = FrameShard(ctx, B, first, scene.K_KITTI, T_RIGHT, halo=True, world=world, rank=rank, backend=backend,
                       kf_every=args.kf_every if use_map else 0, max_kf=max_kf,
                       overlap_mode=0 if args.no_overlap else args.overlap_mode, tracker=args.tracker)
    batch = shard.batch
    NT = shard.n_tracks
    pairs, tracks = shard.pairs, shard.tracks

    def step():
        shard.step(d_frames.data_ptr())

    for _ in range(args.warmup):
        step()
    shard.drain()
    if not args.no_timing:
        # inside the timed region only the dominant kernel (detect) is bracketed by events; the per-stage table
        # comes from a separate pass after it (--stage-steps), so nine events per step do not tax `value`
        batch.enable_timing(2)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    shard.drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # PCIe-inclusive rate: the same step's frames uploaded from pinned host memory, timed alone;
    # reported beside `value` (which has the inputs resident in HBM), never as it
    h_frames = torch.from_numpy(images).pin_memory()
    d_up = torch.empty_like(d_frames)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        d_up.copy_(h_frames, non_blocking=True)
    torch.cuda.synchronize()
    h2d_ms = (time.perf_counter() - t1) / 3 * 1e3
    del d_up, h_frames

    # end-to-end rate: every step's frames go host -> HBM from pinned memory into one of two device
    # buffers on a copy stream while the previous step's kernels run.  The upload of step i + 1 waits only for the
    # run of step i - 1 (the last reader of that buffer: detect reads the raw images) and step i waits for its
    # upload, so the copy engine and the kernels overlap; the timed region holds every upload.  Reported beside
    # `value` (inputs resident), never as it.
    e2e = None
    if args.e2e_steps > 0:
        h_frames = torch.from_numpy(images).pin_memory()
        bufs = [d_frames, torch.empty_like(d_frames)]
        copy_stream = torch.cuda.Stream(device=dev)
        ctx_stream = torch.cuda.ExternalStream(ctx.stream, device=dev)
        up_ev = [torch.cuda.Event() for _ in range(2)]
        run_ev = [torch.cuda.Event() for _ in range(2)]

        def upload(i):
            k = i % 2
            with torch.cuda.stream(copy_stream):
                if i >= 2:
                    copy_stream.wait_event(run_ev[k])
                bufs[k].copy_(h_frames, non_blocking=True)
                up_ev[k].record(copy_stream)

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        upload(0)
        for i in range(args.e2e_steps):
            if i + 1 < args.e2e_steps:
                upload(i + 1)
            ctx_stream.wait_event(up_ev[i % 2])
            shard.step(bufs[i % 2].data_ptr())
            run_ev[i % 2].record(ctx_stream)
        shard.drain()
        torch.cuda.synchronize()
        e2e_s = time.perf_counter() - t2
        if world > 1:
            dist.barrier()
            t = torch.tensor([e2e_s], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e2e_s = float(t.item())
        e2e = {"frames_per_s": round(B * world * args.e2e_steps / e2e_s, 2),
               "ms_per_step": round(1e3 * e2e_s / args.e2e_steps, 4), "steps": args.e2e_steps,
               "h2d_bytes_per_step_per_gpu": int(images.nbytes),
               "h2d_GBps_per_gpu": round(images.nbytes * args.e2e_steps / e2e_s / 1e9, 2),
               "how": "pinned host frames -> two device buffers on a copy stream, step i+1's upload overlapped with "
                      "step i's kernels; timed region = all uploads + all steps"}
        del h_frames, bufs

    png_e2e = None
    if args.png_steps > 0 and world == 1 and args.tracker == "match":
        thr = args.png_threads or cpu_threads_available()
        try:
            png_e2e = png_end_to_end(ctx, shard, images, halo_right, B, args.png_steps, thr, gpu_decode=True)
        except Exception as e:  # reported, never fatal to the headline
            png_e2e = {"error": repr(e)[:300]}
        try:
            png_e2e["host_decode"] = png_end_to_end(ctx, shard, images, halo_right, B, args.png_steps, thr,
                                                    gpu_decode=False)
        except Exception as e:
            png_e2e["host_decode"] = {"error": repr(e)[:300]}
    seq = None
    if args.sequence_frames > 0 and world > 1 and args.tracker == "match":
        # configs[2]'s front end frame-sharded over the ranks (every rank; SequenceShard)
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import bench_sequence
            seq = bench_sequence.measure_sharded(ctx, rank, world, args.sequence_frames, 20, repeats=5)
        except Exception as e:  # reported, never fatal to the headline
            seq = {"error": repr(e)[:300]}
    if args.sequence_frames > 0 and world == 1 and rank == 0 and args.tracker == "match":
        # BASELINE configs[2]: the full front end + local BA over the first 200 frames (tools/bench_sequence.py)
        try:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import bench_sequence
            seq = bench_sequence.measure(args.sequence_frames, 20, repeats=5, cpu=bool(args.sequence_cpu),
                                         cpu_threads=min(16, cpu_threads_available()), ctx=ctx, check_frames=200)
            seq.pop("_trajectory", None)
        except Exception as e:  # reported, never fatal to the headline
            seq = {"error": repr(e)[:300]}
    lh = None
    if args.loop_handler_frames > 0 and world == 1 and rank == 0:
        try:
            lh = loop_handler_leg(args.loop_handler_frames)
        except Exception as e:
            lh = {"error": repr(e)[:300]}

    v = batch.view()
    counts = {
        "cand": ctx.download(v.cand_count, np.uint32, n_img + 1).astype(np.int64),
        "det": ctx.download(v.det_count, np.int32, n_img + 1).astype(np.int64),
        "kp": ctx.download(v.kp_count, np.int32, n_img + 1).astype(np.int64),
        "match": ctx.download(v.match_count, np.int32, len(pairs)).astype(np.int64),
        "filt": ctx.download(v.filt_count, np.int32, len(pairs)).astype(np.int64),
    }
    counts["train"] = np.array([counts["kp"][t] for _, t in pairs], np.int64)
    ec = ctx.download(v.edge_count, np.int32, NT)
    counts["edges"] = float(np.sum(ec))
    counts["tq"] = float(np.sum([counts["match"][tp] for _, tp in tracks])) if args.tracker == "match" else 0.0
    inliers = ctx.download(v.track_inliers, np.int32, NT)
    gpu_poses = shard.poses()
    edges = None
    if rank == 0 and world == 1 and args.cpu_baseline != "none" and args.tracker == "match":
        eX = ctx.download(v.edge_X, np.float64, NT * MAX_KP * 3).reshape(NT, MAX_KP, 3)
        euv = ctx.download(v.edge_uv, np.float64, NT * MAX_KP * 2).reshape(NT, MAX_KP, 2)
        edges = (ec, eX, euv)

    stages = {}
    roofline = None
    per_stage = None
    coll_stats = None
    if not args.no_timing:
        ms_t, nruns_t = batch.stage_times()
        detect_timed_ms = float(ms_t[0]) / max(nruns_t, 1)
        batch.enable_timing(True)
        shard.set_collective_timing(True)
        for _ in range(args.stage_steps):
            step()
        shard.drain()
        coll_stats = shard.collective_stats()
        shard.set_collective_timing(False)
        ms, nruns = batch.stage_times()
        per_launch_ms = {name: float(ms[i]) / max(nruns, 1) for i, name in enumerate(yv.STAGE_NAMES)}
        per_launch_ms["detect"] = detect_timed_ms
        stages = {k: round(x, 4) for k, x in per_launch_ms.items()}
        nbytes = stage_bytes(counts, n_img)
        # the dominant kernel is the longest on the critical path: with overlap the pose LM runs beside the
        # next batch on the side stream and the edge build beside the next detect on its own stream;
        # neither is on it
        crit = {k: t for k, t in per_launch_ms.items() if args.no_overlap or k not in ("track_pose", "track_edges")}
        dom = max(crit, key=crit.get)
        dur_s = per_launch_ms[dom] / 1e3
        achieved = nbytes[dom] / dur_s / 1e9
        traffic = None
        fp64 = {}
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        traffic_stamp = None
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
                # counters taken on this step size AND on this code (the kernel sources' digest), else null
                traffic_stamp = {"commit": pmc.get("commit"), "source_sha256": pmc.get("source_sha256"),
                                 "matches_code": pmc.get("source_sha256") == kernel_source_digest()}
                if pmc.get("frames_per_step") == B and traffic_stamp["matches_code"]:
                    traffic = pmc.get("per_launch_bytes", {}).get(dom)
                    fp64 = pmc.get("fp64_per_launch", {})
            except (OSError, ValueError):
                traffic = None
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "traffic_stamp": traffic_stamp,
                    "algorithmic_bytes_per_launch": int(nbytes[dom]), "launch_ms": round(per_launch_ms[dom], 4)}
        # every stage against the bound that limits it: VALU lane-ops for detect, FP4 MFMA ops
        # for the matcher (2 * Kq * Kt * 256 per pair, FP4 MFMA), HBM bytes for the rest
        ops = stage_valu_ops(counts, n_img)
        per_stage = {}
        for st, t_ms in per_launch_ms.items():
            if t_ms <= 0:
                continue
            if st == "detect":
                a = ops["detect"] / (t_ms / 1e3) / 1e12
                per_stage[st] = {"bound": "valu", "achieved": round(a, 3), "peak": round(VALU_PEAK_TOPS, 1),
                                 "unit": "T lane-op/s", "frac": round(a / VALU_PEAK_TOPS, 4)}
            elif st == "match":
                mops = float(np.sum(counts["match"].astype(np.float64) * counts["train"])) * 256 * 2
                a = mops / (t_ms / 1e3) / 1e12
                per_stage[st] = {"bound": "mfma_fp4", "achieved": round(a, 1), "peak": FP4_MFMA_PEAK_TOPS,
                                 "unit": "T op/s", "frac": round(a / FP4_MFMA_PEAK_TOPS, 4)}
            elif st in ("track_pose", "track_edges"):
                # FP64 VALU: the launch's FP64 wave-instructions from the PMC pass (tools/pmc_traffic.sh,
                # profiles/pmc_traffic.json) over this run's per-launch time.  SQ_INSTS_VALU_FLOPS_FP64 counts per
                # wave-instruction (ADD + MUL + 2 FMA), so lane-FLOPs = 64 x it, an upper bound (the LM's lane-0 LDLT
                # runs one lane); issue_frac = FP64 wave-instructions x 4 cycles / SIMD-cycles of the launch
                f = fp64.get(st)
                if f:
                    a = 64.0 * f["flops"] / (t_ms / 1e3) / 1e12
                    per_stage[st] = {"bound": "fp64_valu", "achieved": round(a, 3), "peak": round(FP64_PEAK_TFLOPS, 1),
                                     "unit": "TFLOP/s", "frac": round(a / FP64_PEAK_TFLOPS, 4),
                                     "issue_frac": round(4 * f["wave_instructions"] / (SIMD_CYCLES_PER_S * t_ms / 1e3), 4),
                                     "fp64_wave_flops_per_launch": f["flops"],
                                     "fp64_wave_instructions_per_launch": f["wave_instructions"],
                                     "note": ("serial LM per problem, beside the next step's image kernels (DESIGN.md "
                                              "4.2, 4.4)" if st == "track_pose" else
                                              "one 4 x 4 Jacobi SVD triangulation per stereo edge, beside the next "
                                              "step's detect (DESIGN.md 4.3, 7.1)") +
                                             "; achieved = 64 lanes x PMC FP64 wave-FLOPs / launch time"}
                else:
                    per_stage[st] = {"bound": "latency" if st == "track_pose" else "fp64_valu",
                                     "note": "FP64 counters not taken at this code (profiles/pmc_traffic.json)",
                                     "ms": round(t_ms, 4)}
            else:
                a = nbytes[st] / (t_ms / 1e3) / 1e9
                per_stage[st] = {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(a / HBM_PEAK_GBS, 5)}
        if dom in ops:
            tops = ops[dom] / dur_s / 1e12
            roofline["valu"] = {"achieved": round(tops, 3), "peak": round(VALU_PEAK_TOPS, 1), "unit": "T lane-op/s",
                                "frac": round(tops / VALU_PEAK_TOPS, 4)}

    frames_total = B * world * args.steps
    value = frames_total / elapsed
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "configs[1] + PnP: FAST+BRIEF+Hamming match, 1241x376 synthetic stereo, 2000 "
                               "kp/image, stereo triangulation + pose-only LM per frame",
                   "H": H, "W": W, "max_kp": MAX_KP, "frames_per_step_per_gpu": B, "images_per_frame": 2,
                   "match_pairs_per_frame": 2,
                   "frames": f"one synthetic sequence (field seed 1234); rank r owns frames [1 + r*B, 1 + (r+1)*B) "
                             f"and detects / describes its predecessor frame r*B in the same run (1-frame halo, "
                             f"image {n_img - 1}), so every temporal pair L_(k-1) -> L_k is the sequence's own",
                   "halo_images_per_step_per_gpu": n_img - 2 * B,
                   "devices_used": min(world, max(torch.cuda.device_count(), 1)),
                   "parallelism": f"frame-sharded x{world}" + (f", {'RCCL' if backend == 'nccl' else backend} "
                                                                 "all-gather of shared-map blocks"
                                                                 if use_map and world > 1 else ""),
                   "mean_candidates_per_image": round(float(np.mean(counts["cand"][:n_img])), 1),
                   "mean_keypoints_per_image": round(float(np.mean(counts["kp"][:n_img])), 1),
                   "mean_filtered_matches_per_pair": round(float(np.mean(counts["filt"])), 1),
                   "tracker": args.tracker, "pnp_frames_per_step": NT,
                   "mean_pnp_edges_per_frame": round(counts["edges"] / max(NT, 1), 1),
                   "mean_pnp_inliers_per_frame": round(float(np.mean(inliers)), 1)},
        "stages_ms_per_launch": stages,
        "stage_timing": None if args.no_timing else
        f"detect: HIP events over the timed region ({args.steps} steps); the other stages: a separate "
        f"{args.stage_steps}-step pass after it with events around every stage",
        "stage_rooflines": per_stage if not args.no_timing else None,
        "h2d_upload_ms_per_step": round(h2d_ms, 4),
        "pcie_inclusive_frames_per_s": round(frames_total / (elapsed + args.steps * h2d_ms / 1e3), 2),
        "end_to_end": e2e,
        "png_end_to_end": png_e2e,
        "loop_handler": lh,
        "sequence": seq,
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if use_map:
        # the last placed map (rank 0's copy of every rank's block): its keyframes and landmarks per step
        raw = shard.placed_map()
        bb = shard.bb
        n_kf = n_lm = 0
        for r in range(world):
            h, kfs, lms = ymap.parse_block(raw[r])
            n_kf += int(h["n_kf"])
            n_lm += sum(len(x) for x in lms)
        out["shared_map"] = {"kf_every": args.kf_every, "block_bytes": bb, "keyframes_per_step": n_kf,
                             "landmarks_per_step": n_lm, "allgather_bytes_per_rank_per_step": bb * world,
                             "world_size_seen": dist.get_world_size() if dist.is_initialized() else 1,
                             "collective_timing": coll_stats,
                             "collective": ("none (1 rank)" if world == 1 and not shard.collective else
                                            "all_gather_into_tensor (RCCL, 1-rank group)" if world == 1 else
                                            "all_gather_into_tensor (RCCL)" if backend == "nccl" else
                                            f"all_gather ({backend} rehearsal)")}
    if rank == 0 and world == 1 and args.cpu_baseline != "none" and args.tracker == "match":
        threads = args.cpu_threads or cpu_threads_available()
        cb = cpu_baseline(args.cpu_baseline, threads, offsets.reshape(256, 4), images, B, gpu_poses, edges,
                          args.literal_frames)
        main_cb = cb.get("literal") or cb.get("efficient")
        out["cpu_baseline"] = main_cb
        if "efficient" in cb and main_cb is not cb["efficient"]:
            out["cpu_baseline_efficient"] = cb["efficient"]
        out["cpu_baseline_host_cpus"] = os.cpu_count()
        out["cpu_baseline_usable_cpus"] = cpu_threads_available()
        out["pose_check"] = cb["pose_check"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    shard.close()
    ctx.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
