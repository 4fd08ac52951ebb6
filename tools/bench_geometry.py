"""Throughput of the geometry rows on their own next to the oracle on the host, at the
bench's shapes: 256 match lists / pose problems of ~1900 entries (one per stereo frame of a bench step).

    python tools/bench_geometry.py [--lists 256] [--n 1900] [--iters 400]

Prints one JSON object (committed as profiles/r01_geometry.json).  GPU times: HIP events around the batched
launches, inputs resident in HBM.  CPU: the oracle (the reference's algorithms restated), single thread, on a
bounded sample."""
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
    ap.add_argument("--lists", type=int, default=256)
    ap.add_argument("--n", type=int, default=1900)
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import ya_vo_amd as yv
    from ya_vo_amd import MATCH_DTYPE, scene
    import oracle_bind

    orc = oracle_bind.Oracle()
    ctx = yv.Context(0)
    dev = "cuda:0"
    L, n, iters = args.lists, args.n, args.iters
    out = {"lists": L, "entries_per_list": n, "ransac_iterations": iters}

    # ---- F-RANSAC: L lists of n matches (two-view synthetic, 10% gross mismatches), iters hypotheses each
    lists = np.zeros((L, n), MATCH_DTYPE)
    samples = np.zeros((L, iters, 8), np.int32)
    for l in range(L):
        _, _, _, ua, ub = scene.two_view_matches(n, seed=100 + l)
        m = lists[l]
        m["pt1"]["x"], m["pt1"]["y"] = np.round(ua[:, 0]), np.round(ua[:, 1])
        m["pt2"]["x"], m["pt2"]["y"] = np.round(ub[:, 0]), np.round(ub[:, 1])
        rng = np.random.default_rng(l)
        bad = rng.choice(n, n // 10, replace=False)
        m["pt2"]["x"][bad] = rng.integers(0, 376, len(bad))
        samples[l] = rng.integers(0, n, (iters, 8))
    d_m = torch.from_numpy(lists.view(np.uint8).reshape(-1)).to(dev)
    d_cnt = torch.full((L,), n, dtype=torch.int32, device=dev)
    d_s = torch.from_numpy(samples.reshape(-1)).to(dev)
    d_F = torch.zeros(L * 9, dtype=torch.float64, device=dev)
    d_inl = torch.zeros(L, dtype=torch.int32, device=dev)
    d_found = torch.zeros(L, dtype=torch.int32, device=dev)
    # one explicit stream for the library launches, the copies and the events (the null stream would let the
    # library fall back to its own non-blocking context stream, unordered with torch's work)
    ts = torch.cuda.Stream()
    torch.cuda.set_stream(ts)
    stream = ts.cuda_stream
    assert stream != 0

    def ransac():
        assert ctx.lib.yv_f_ransac_batch(ctx.handle, d_m.data_ptr(), n, d_cnt.data_ptr(), L, d_s.data_ptr(),
                                         iters * 8, iters, 0.1, d_F.data_ptr(), d_inl.data_ptr(),
                                         d_found.data_ptr(), stream) == 0

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    ms = timed(ransac)
    t0 = time.perf_counter()
    ok, F, inl = orc.f_ransac(lists[0], samples[0], 0.1)
    cpu = time.perf_counter() - t0
    gpu_F = d_F[:9].cpu().numpy().reshape(3, 3)
    out["f_ransac"] = {"gpu_ms_per_launch": round(ms, 4), "gpu_lists_per_s": round(L / ms * 1e3, 1),
                       "gpu_hypotheses_per_s": round(L * iters / ms * 1e3, 1),
                       "cpu_oracle_lists_per_s": round(1 / cpu, 3), "cpu_threads": 1,
                       "list0_bit_identical": bool(np.array_equal(gpu_F, F) and int(d_inl[0]) == inl)}

    # ---- pose LM / GN: L problems of n edges (0.5 px noise, 10% gross outliers)
    probs = [scene.random_scene(n, seed=200 + i, noise_px=0.5, outlier_frac=0.1) for i in range(L)]
    priors = np.stack([scene.perturb(p[2], np.random.default_rng(i)) for i, p in enumerate(probs)])
    offs = (np.arange(L + 1) * n).astype(np.int32)
    d_off = torch.from_numpy(offs).to(dev)
    d_X = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[0] for p in probs]))).to(dev)
    d_uv = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[1] for p in probs]))).to(dev)
    d_K = torch.from_numpy(np.tile(scene.K_KITTI.reshape(1, 9), (L, 1))).to(dev)
    d_prior = torch.from_numpy(priors).to(dev)
    d_P = torch.empty_like(d_prior)
    d_out = torch.zeros(L * n, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(L, dtype=torch.int32, device=dev)

    def lm():
        d_P.copy_(d_prior)
        assert ctx.lib.yv_pose_lm_batch(ctx.handle, L, d_off.data_ptr(), d_X.data_ptr(), d_uv.data_ptr(),
                                        d_K.data_ptr(), d_P.data_ptr(), d_out.data_ptr(), d_res.data_ptr(),
                                        stream) == 0

    def gn():
        d_P.copy_(d_prior)
        assert ctx.lib.yv_pose_gn_batch(ctx.handle, L, d_off.data_ptr(), d_X.data_ptr(), d_uv.data_ptr(),
                                        d_K.data_ptr(), d_P.data_ptr(), d_res.data_ptr(), stream) == 0

    for name, fn, cpu_fn in (("pose_lm", lm, lambda: orc.pose_lm(probs[0][0], probs[0][1], scene.K_KITTI, priors[0], yv.lm_sum_mode(1))),
                             ("pose_gn", gn, lambda: orc.pose_gn(probs[0][0], probs[0][1], scene.K_KITTI, priors[0], 1))):
        ms = timed(fn)
        torch.cuda.synchronize()
        P0 = d_P[0].cpu().numpy()
        t0 = time.perf_counter()
        ref = cpu_fn()
        cpu = time.perf_counter() - t0
        out[name] = {"gpu_ms_per_launch": round(ms, 4), "gpu_problems_per_s": round(L / ms * 1e3, 1),
                     "cpu_oracle_problems_per_s": round(1 / cpu, 2), "cpu_threads": 1,
                     "problem0_bit_identical": bool(np.array_equal(P0, ref[0]))}

    # ---- triangulation of n matches through the host-pointer entry point (includes the PCIe copies) and
    # the oracle
    Ta, Tb, _, ua, ub = scene.two_view_matches(n, seed=7)
    m = lists[0]
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ctx.triangulate(Ta, Tb, scene.K_KITTI, m)
    host_ms = (time.perf_counter() - t0) / args.reps * 1e3
    t0 = time.perf_counter()
    orc.triangulate_matches(Ta, Tb, scene.K_KITTI, m)
    cpu = time.perf_counter() - t0
    out["triangulate"] = {"host_api_ms_per_list": round(host_ms, 4), "cpu_oracle_ms_per_list": round(cpu * 1e3, 3),
                          "note": "batched device-resident triangulation runs inside track_build_kernel "
                                  "(bench.py stage track_edges)"}
    # ---- pyramidal LK: L frame pairs (synthetic 1241x376, frame k+1 = frame k shifted), 2000 points each --
    from ya_vo_amd.synth import synth_stereo_batch
    H, W = 376, 1241
    LP = max(L // 2, 1)
    imgs = synth_stereo_batch(77, LP + 1)[::2]  # left images of consecutive frames
    imgs = np.ascontiguousarray(imgs[: LP + 1])
    n_img = len(imgs)
    n_pairs = n_img - 1
    npts = 2000
    rng = np.random.default_rng(3)
    pts = np.stack([rng.uniform(20, W - 21, (n_pairs, npts)), rng.uniform(20, H - 21, (n_pairs, npts))], -1)
    pts = pts.astype(np.float32)
    d_img = torch.from_numpy(imgs).to(dev)
    d_pairs = torch.from_numpy(np.stack([np.arange(n_pairs), np.arange(1, n_pairs + 1)], 1).astype(np.int32)).to(dev)
    d_cnt = torch.full((n_pairs,), npts, dtype=torch.int32, device=dev)
    d_pts = torch.from_numpy(pts).to(dev)
    d_next = torch.zeros_like(d_pts)
    d_st = torch.zeros((n_pairs, npts), dtype=torch.uint8, device=dev)
    d_err = torch.zeros((n_pairs, npts), dtype=torch.float32, device=dev)
    lk = yv.Lk(ctx, n_img, H, W)

    def lk_build():
        lk.build(d_img.data_ptr(), n_img, W, H * W, stream)

    def lk_track():
        lk.track(d_pairs.data_ptr(), n_pairs, d_pts.data_ptr(), d_cnt.data_ptr(), npts, d_next.data_ptr(),
                 d_st.data_ptr(), d_err.data_ptr(), stream=stream)

    ms_b = timed(lk_build)
    ms_t = timed(lk_track)
    torch.cuda.synchronize()
    g = d_next[0].cpu().numpy()
    t0 = time.perf_counter()
    o, os_, oe, _ = orc.lk(imgs[0], imgs[1], pts[0], sum_mode=1)
    cpu = time.perf_counter() - t0
    out["lk"] = {"pairs": n_pairs, "points_per_pair": npts, "gpu_pyramid_ms": round(ms_b, 4),
                 "gpu_track_ms": round(ms_t, 4),
                 "gpu_points_per_s": round(n_pairs * npts / ((ms_b * n_img / n_img + ms_t) / 1e3), 1),
                 "cpu_oracle_points_per_s": round(npts / cpu, 1), "cpu_threads": 1,
                 "pair0_bit_identical": bool(np.array_equal(g, o)),
                 "pair0_tracked": int(os_.sum())}
    lk.close()
    # ---- findEssentialMat (RANSAC) + recoverPose: L lists of n correspondences, 20% gross mismatches --------
    from epipolar_scene import K_KITTI, two_view_scene
    ne = n
    e1 = np.zeros((L, ne, 2), np.float32)
    e2 = np.zeros((L, ne, 2), np.float32)
    for l in range(L):
        a, b, _, _ = two_view_scene(ne, outlier_frac=0.2, seed=500 + l, angle=0.02 + 0.0001 * l)
        e1[l], e2[l] = a, b
    d_e1, d_e2 = torch.from_numpy(e1).to(dev), torch.from_numpy(e2).to(dev)
    d_ecnt = torch.full((L,), ne, dtype=torch.int32, device=dev)
    d_E = torch.zeros((L, 9), dtype=torch.float64, device=dev)
    d_ef = torch.zeros(L, dtype=torch.int32, device=dev)
    d_es = torch.zeros((L, 3), dtype=torch.int32, device=dev)
    d_R = torch.zeros((L, 9), dtype=torch.float64, device=dev)
    d_t = torch.zeros((L, 3), dtype=torch.float64, device=dev)
    es = yv.Essential(ctx, L, ne)

    def ess_find():
        es.find(d_e1.data_ptr(), d_e2.data_ptr(), d_ecnt.data_ptr(), L, ne, d_E.data_ptr(), d_ef.data_ptr(),
                d_stats=d_es.data_ptr(), stream=stream)

    def ess_recover():
        es.recover(d_E.data_ptr(), d_e1.data_ptr(), d_e2.data_ptr(), d_ecnt.data_ptr(), L, ne, K_KITTI,
                   d_R.data_ptr(), d_t.data_ptr(), stream=stream)

    ms_f = timed(ess_find)
    ms_r = timed(ess_recover)
    torch.cuda.synchronize()
    gE = d_E[0].cpu().numpy().reshape(3, 3)
    st = d_es.cpu().numpy()
    t0 = time.perf_counter()
    ok0, oE, _, _ = orc.find_essential(e1[0], e2[0])
    og, oR, ot, _ = orc.recover_pose(oE, e1[0], e2[0], K_KITTI)
    cpu = time.perf_counter() - t0
    out["essential"] = {"pairs": L, "points_per_pair": ne, "outlier_frac": 0.2,
                        "gpu_find_ms": round(ms_f, 4), "gpu_recover_ms": round(ms_r, 4),
                        "gpu_pairs_per_s": round(L / ((ms_f + ms_r) / 1e3), 1),
                        "mean_ransac_iterations": round(float(st[:, 0].mean()), 2),
                        "cpu_oracle_pairs_per_s": round(1 / cpu, 2), "cpu_threads": 1,
                        "pair0_bit_identical": bool(ok0 and np.array_equal(gE, oE) and
                                                    np.array_equal(d_R[0].cpu().numpy().reshape(3, 3), oR))}
    es.close()

    # ---- sliding-window BA (BASELINE config 5): 20 keyframes, 10k landmarks x 5 observations, 10 LM iterations
    w = scene.ba_window(n_poses=20, n_landmarks=10000, obs=5, noise_px=1.0, seed=0)
    P, NL, NE = len(w["poses0"]), len(w["X0"]), len(w["ep"])
    ba = yv.BundleAdjuster(ctx, P, NL, NE)
    ba.set_problem(P, 1, NL, w["ep"], w["el"], w["meas"], K_KITTI)
    ba.solve(w["poses0"], w["X0"], 10)  # warm
    ts_ = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        T, X, log, it = ba.solve(w["poses0"], w["X0"], 10)
        ts_.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    oT, oX, oit, olog = orc.ba_lm(w["poses0"], 1, w["X0"], w["ep"], w["el"], w["meas"], K_KITTI, 10)
    cpu = time.perf_counter() - t0
    ms = 1e3 * float(np.median(ts_))
    out["bundle_adjustment"] = {"poses": P, "fixed": 1, "landmarks": NL, "edges": NE, "lm_iterations": it,
                                "gpu_ms_per_solve": round(ms, 3), "gpu_ms_per_iteration": round(ms / max(it, 1), 3),
                                "gpu_solves_per_s": round(1e3 / ms, 2), "includes": "host estimate in/out + LM control",
                                "cpu_oracle_ms_per_solve": round(1e3 * cpu, 1), "cpu_threads": 1,
                                "chi2": [float(log[0]), float(log[-1])],
                                "bit_identical": bool(it == oit and np.array_equal(T, oT) and np.array_equal(X, oX)
                                                      and np.array_equal(log, olog))}
    ba.close()
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
