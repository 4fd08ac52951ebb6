"""GPU parity of the geometry rows (F-RANSAC, triangulation, world2Camera, pose-only LM, GN) against the
oracle.  The kernels evaluate every expression in the oracle's order with contraction off and sum edges in
the oracle's tree order (sum_mode 1), so results are compared bit for bit; against the reference's
sequential edge order (sum_mode 0) they agree within the stated tolerance (poses 1e-9 absolute)."""
import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd import MATCH_DTYPE, scene

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-9  # |pose_gpu - pose_reference_order| (quaternion + translation), stated in DESIGN.md
LM_ORDER = yv.lm_sum_mode(1)  # yv_pose_lm's edge-sum order (oracle sum_mode 4 / 5 / 6 / 7, yv_pose_lm_sum_mode)
GN_ORDER = 1     # the GN kernel's: 256-thread tree


def _match_array(ua, ub):
    m = np.zeros(len(ua), MATCH_DTYPE)
    m["pt1"]["x"] = np.round(ua[:, 0])
    m["pt1"]["y"] = np.round(ua[:, 1])
    m["pt2"]["x"] = np.round(ub[:, 0])
    m["pt2"]["y"] = np.round(ub[:, 1])
    return m


@pytest.mark.parametrize("n,iters,seed", [(200, 400, 2), (8, 50, 3), (1970, 400, 4), (50, 1, 5)])
def test_f_ransac_matches_oracle(ctx, oracle, n, iters, seed):
    Ta, Tb, X, ua, ub = scene.two_view_matches(n, seed=seed)
    m = _match_array(ua, ub)
    rng = np.random.default_rng(seed)
    if seed == 4:  # add gross mismatches
        bad = rng.choice(n, n // 5, replace=False)
        m["pt2"]["x"][bad] = rng.integers(0, 376, len(bad))
    samples = rng.integers(0, n, (iters, 8)).astype(np.int32)
    found, F, inl = ctx.f_ransac(m, samples, 0.1)
    ofound, oF, oinl = oracle.f_ransac(m, samples, 0.1)
    assert found == ofound and inl == oinl
    np.testing.assert_array_equal(F, oF)


def test_f_ransac_too_few(ctx):
    m = np.zeros(7, MATCH_DTYPE)
    found, F, inl = ctx.f_ransac(m, np.zeros((4, 8), np.int32), 0.1)
    assert not found


def test_triangulate_matches_oracle(ctx, oracle):
    Ta, Tb, X, ua, ub = scene.two_view_matches(1500, seed=6)
    m = _match_array(ua, ub)
    Tb2 = scene.perturb(Tb, np.random.default_rng(1), rot=0.003, trans=0.01)
    for pa, pb in ((Ta, Tb), (Tb2, Ta)):
        n, Xw, ok = ctx.triangulate(pa, pb, scene.K_KITTI, m)
        on, oX, ook = oracle.triangulate_matches(pa, pb, scene.K_KITTI, m)
        assert n == on
        np.testing.assert_array_equal(ok, ook)
        np.testing.assert_array_equal(Xw, oX)


def test_world2camera_matches_oracle(ctx, oracle):
    X, uv, T, _ = scene.random_scene(777, seed=7)
    np.testing.assert_array_equal(ctx.world2camera(X, T, scene.K_KITTI), oracle.world2camera(X, T, scene.K_KITTI))


@pytest.mark.parametrize("n,noise,outl,seed", [(300, 0.0, 0.0, 9), (1500, 0.5, 0.1, 10), (2000, 1.0, 0.3, 11),
                                               (7, 0.3, 0.0, 12), (0, 0.0, 0.0, 13)])
def test_pose_lm_matches_oracle(ctx, oracle, n, noise, outl, seed):
    X, uv, T_true, _ = scene.random_scene(max(n, 1), seed=seed, noise_px=noise, outlier_frac=outl)
    X, uv = X[:n], uv[:n]
    prior = scene.perturb(T_true, np.random.default_rng(seed))
    T, out, inl = ctx.pose_lm(X, uv, scene.K_KITTI, prior)
    oT, oout, oinl = oracle.pose_lm(X, uv, scene.K_KITTI, prior, LM_ORDER)
    assert inl == oinl
    np.testing.assert_array_equal(out, oout)
    np.testing.assert_array_equal(T, oT)
    rT, rout, rinl = oracle.pose_lm(X, uv, scene.K_KITTI, prior, 0)
    assert rinl == inl
    np.testing.assert_allclose(T, rT, rtol=0, atol=POSE_TOL)


@pytest.mark.parametrize("noise,outl,perturb", [(0.0, 0.0, False), (0.2, 0.0, False), (0.2, 0.0, True),
                                                (0.5, 0.05, False), (2.2, 0.0, True)])
def test_pose_lm_round_replay_matches_oracle(ctx, oracle, noise, outl, perturb):
    """The kernel skips a round that replays the last executed one (same active set and, across the Huber drop, no
    Huber weight applied); the oracle runs all four rounds.  Cases: exact prior (no Huber, no outliers: rounds 1-3
    replayed), perturbed prior (Huber active early: round 3 runs), noise near the chi2 threshold (levels flip between
    rounds: no replay)."""
    X, uv, T_true, _ = scene.random_scene(1200, seed=31, noise_px=noise, outlier_frac=outl)
    prior = scene.perturb(T_true, np.random.default_rng(31)) if perturb else T_true
    T, out, inl = ctx.pose_lm(X, uv, scene.K_KITTI, prior)
    oT, oout, oinl = oracle.pose_lm(X, uv, scene.K_KITTI, prior, LM_ORDER)
    assert inl == oinl
    np.testing.assert_array_equal(out, oout)
    np.testing.assert_array_equal(T, oT)


@pytest.mark.parametrize("n,seed", [(100, 12), (2000, 14)])
def test_pose_gn_matches_oracle(ctx, oracle, n, seed):
    X, uv, T_true, _ = scene.random_scene(n, seed=seed, noise_px=0.3)
    prior = scene.perturb(T_true, np.random.default_rng(seed), rot=0.01, trans=0.05)
    T, it = ctx.pose_gn(X, uv, scene.K_KITTI, prior)
    oT, oit = oracle.pose_gn(X, uv, scene.K_KITTI, prior, GN_ORDER)
    assert it == oit
    np.testing.assert_array_equal(T, oT)
    rT, rit = oracle.pose_gn(X, uv, scene.K_KITTI, prior, 0)
    np.testing.assert_allclose(T, rT, rtol=0, atol=POSE_TOL)


def test_pose_lm_batch(ctx, oracle):
    """Several pose problems in one launch (the batched frontend form)."""
    import torch
    probs = [scene.random_scene(n, seed=20 + i, noise_px=0.5, outlier_frac=0.1) for i, n in enumerate((50, 900, 1600))]
    priors = [scene.perturb(p[2], np.random.default_rng(i)) for i, p in enumerate(probs)]
    offs = np.cumsum([0] + [len(p[0]) for p in probs]).astype(np.int32)
    # random_scene's X is a transposed view; np.concatenate keeps its Fortran order and torch keeps strides,
    # so force the row-major [n][3] / [n][2] layouts the ABI documents
    Xall = np.ascontiguousarray(np.concatenate([p[0] for p in probs]))
    uvall = np.ascontiguousarray(np.concatenate([p[1] for p in probs]))
    dev = "cuda:0"
    d_off = torch.from_numpy(offs).to(dev)
    d_X = torch.from_numpy(Xall).to(dev)
    d_uv = torch.from_numpy(uvall).to(dev)
    d_K = torch.from_numpy(np.tile(scene.K_KITTI.reshape(1, 9), (len(probs), 1))).to(dev)
    d_P = torch.from_numpy(np.stack(priors)).to(dev)
    d_out = torch.zeros(len(Xall), dtype=torch.uint8, device=dev)
    d_inl = torch.zeros(len(probs), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    st = ctx.lib.yv_pose_lm_batch(ctx.handle, len(probs), d_off.data_ptr(), d_X.data_ptr(), d_uv.data_ptr(),
                                  d_K.data_ptr(), d_P.data_ptr(), d_out.data_ptr(), d_inl.data_ptr(), None)
    assert st == 0
    ctx.sync()
    P = d_P.cpu().numpy()
    out = d_out.cpu().numpy().astype(bool)
    inl = d_inl.cpu().numpy()
    for i, p in enumerate(probs):
        oT, oout, oinl = oracle.pose_lm(p[0], p[1], scene.K_KITTI, priors[i], yv.lm_sum_mode(len(probs)))
        assert inl[i] == oinl
        np.testing.assert_array_equal(P[i], oT)
        np.testing.assert_array_equal(out[offs[i]:offs[i + 1]], oout)


def _non_finite_scene(n, seed):
    """A scene whose prior puts some points exactly in the camera plane (pc_z = 0: u / 0 = inf, 0 / 0 = NaN errors),
    so the LM's passes meet non-finite operands (the literal J^T Omega J form, lm_pass)."""
    rng = np.random.default_rng(seed)
    T = scene.pose([0.0, 0.0, 0.0, 1.0], [0.25, -0.5, -5.0])  # identity rotation: pc = X + t exactly
    z = rng.uniform(9.0, 40.0, n)
    X = np.stack([rng.uniform(-0.6, 0.6, n) * z, rng.uniform(-0.25, 0.25, n) * z, z], 1)
    X[:3, 2] = 5.0                                  # pc_z = 0 under the prior
    X[3] = [-0.25, 0.5, 5.0]                        # pc = 0: 0 / 0
    uv = scene.project(T, X) + rng.normal(scale=0.4, size=(n, 2))
    uv[:4] = [[600.0, 180.0], [10.0, 20.0], [1200.0, 300.0], [607.0, 185.0]]
    return np.ascontiguousarray(X), np.ascontiguousarray(uv), T


def test_pose_lm_non_finite_matches_oracle(ctx, oracle):
    X, uv, prior = _non_finite_scene(800, 5)
    T, out, inl = ctx.pose_lm(X, uv, scene.K_KITTI, prior)
    oT, oout, oinl = oracle.pose_lm(X, uv, scene.K_KITTI, prior, LM_ORDER)
    assert inl == oinl
    np.testing.assert_array_equal(out, oout)
    np.testing.assert_array_equal(T, oT)


def test_pose_lm_batch_non_finite_matches_oracle(ctx, oracle):
    """300 problems (the 256-thread kernel), every 3rd with non-finite operands."""
    import torch
    count = 300
    probs, priors = [], []
    for i in range(count):
        if i % 3 == 0:
            X, uv, prior = _non_finite_scene(600 + i, 100 + i)
        else:
            X, uv, T_true, _ = scene.random_scene(600 + i, seed=100 + i, noise_px=0.4)
            prior = scene.perturb(T_true, np.random.default_rng(i))
        probs.append((X, uv))
        priors.append(prior)
    offs = np.cumsum([0] + [len(p[0]) for p in probs]).astype(np.int32)
    dev = "cuda:0"
    d_off = torch.from_numpy(offs).to(dev)
    d_X = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[0] for p in probs]))).to(dev)
    d_uv = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[1] for p in probs]))).to(dev)
    d_K = torch.from_numpy(np.tile(scene.K_KITTI.reshape(1, 9), (count, 1))).to(dev)
    d_P = torch.from_numpy(np.stack(priors)).to(dev)
    d_out = torch.zeros(int(offs[-1]), dtype=torch.uint8, device=dev)
    d_inl = torch.zeros(count, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    assert ctx.lib.yv_pose_lm_batch(ctx.handle, count, d_off.data_ptr(), d_X.data_ptr(), d_uv.data_ptr(),
                                    d_K.data_ptr(), d_P.data_ptr(), d_out.data_ptr(), d_inl.data_ptr(), None) == 0
    ctx.sync()
    P = d_P.cpu().numpy()
    inl = d_inl.cpu().numpy()
    out = d_out.cpu().numpy().astype(bool)
    mode = yv.lm_sum_mode(count)
    for i in range(count):
        oT, oout, oinl = oracle.pose_lm(probs[i][0], probs[i][1], scene.K_KITTI, priors[i], mode)
        assert inl[i] == oinl, i
        np.testing.assert_array_equal(P[i], oT, err_msg=str(i))
        np.testing.assert_array_equal(out[offs[i]:offs[i + 1]], oout, err_msg=str(i))


@pytest.mark.parametrize("count", [256, 512])
def test_pose_lm_batch_many_repeatable(ctx, oracle, count):
    """256 / 512 bench-sized problems (the 512- and the 256-thread kernel), launched three times: every launch
    bit-identical to the oracle.  Many concurrent 4-wave workgroups expose cross-wave races in the kernel's round control (the
    Huber-flag read of the replay decision raced with the next round's reset before it was read ahead of the
    barrier: 3 of 512 bench poses moved by up to 2.6e-4 between steps)."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(77)
    probs, priors = [], []
    mode = yv.lm_sum_mode(count)
    for i in range(count):
        n = int(rng.integers(1700, 2000))
        noise = float(rng.choice([0.2, 0.5, 0.9, 1.3]))
        p = scene.random_scene(n, seed=1000 + i, noise_px=noise, outlier_frac=float(rng.choice([0.0, 0.02, 0.1])))
        probs.append(p)
        priors.append(p[2] if i % 3 == 0 else scene.perturb(p[2], np.random.default_rng(i)))
    offs = np.cumsum([0] + [len(p[0]) for p in probs]).astype(np.int32)
    Xall = np.ascontiguousarray(np.concatenate([p[0] for p in probs]))
    uvall = np.ascontiguousarray(np.concatenate([p[1] for p in probs]))
    dev = "cuda:0"
    d_off = torch.from_numpy(offs).to(dev)
    d_X = torch.from_numpy(Xall).to(dev)
    d_uv = torch.from_numpy(uvall).to(dev)
    d_K = torch.from_numpy(np.tile(scene.K_KITTI.reshape(1, 9), (len(probs), 1))).to(dev)
    with ThreadPoolExecutor(8) as ex:
        ref = list(ex.map(lambda i: oracle.pose_lm(probs[i][0], probs[i][1], scene.K_KITTI, priors[i], mode),
                          range(len(probs))))
    oP = np.stack([r[0] for r in ref])
    oinl = np.array([r[2] for r in ref])
    for _ in range(3):
        d_P = torch.from_numpy(np.stack(priors)).to(dev)
        d_out = torch.zeros(len(Xall), dtype=torch.uint8, device=dev)
        d_inl = torch.zeros(len(probs), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        assert ctx.lib.yv_pose_lm_batch(ctx.handle, len(probs), d_off.data_ptr(), d_X.data_ptr(), d_uv.data_ptr(),
                                        d_K.data_ptr(), d_P.data_ptr(), d_out.data_ptr(), d_inl.data_ptr(),
                                        None) == 0
        ctx.sync()
        P = d_P.cpu().numpy()
        bad = np.nonzero(np.any(P != oP, axis=1))[0]
        assert len(bad) == 0, f"problems {bad[:10].tolist()} differ from the oracle"
        np.testing.assert_array_equal(d_inl.cpu().numpy(), oinl)


def test_pose_gn_batch(ctx, oracle):
    import torch
    probs = [scene.random_scene(n, seed=30 + i, noise_px=0.3) for i, n in enumerate((40, 700, 2000, 0))]
    priors = [scene.perturb(p[2], np.random.default_rng(i), rot=0.01, trans=0.05) for i, p in enumerate(probs)]
    offs = np.cumsum([0] + [len(p[0]) for p in probs]).astype(np.int32)
    dev = "cuda:0"
    d_off = torch.from_numpy(offs).to(dev)
    d_X = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[0] for p in probs]))).to(dev)
    d_uv = torch.from_numpy(np.ascontiguousarray(np.concatenate([p[1] for p in probs]))).to(dev)
    d_K = torch.from_numpy(np.tile(scene.K_KITTI.reshape(1, 9), (len(probs), 1))).to(dev)
    d_P = torch.from_numpy(np.stack(priors)).to(dev)
    d_it = torch.full((len(probs),), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    assert ctx.lib.yv_pose_gn_batch(ctx.handle, len(probs), d_off.data_ptr(), d_X.data_ptr(), d_uv.data_ptr(),
                                    d_K.data_ptr(), d_P.data_ptr(), d_it.data_ptr(), None) == 0
    ctx.sync()
    P, it = d_P.cpu().numpy(), d_it.cpu().numpy()
    for i, p in enumerate(probs):
        oT, oit = oracle.pose_gn(p[0], p[1], scene.K_KITTI, priors[i], GN_ORDER)
        assert it[i] == oit
        np.testing.assert_array_equal(P[i], oT)


def test_f_ransac_batch(ctx, oracle):
    """Several match lists (padded to a common stride) in one launch, incl. a list too short to fit."""
    import torch
    sizes, iters, stride = (300, 5, 1200, 60), 128, 1200
    lists = np.zeros((len(sizes), stride), MATCH_DTYPE)
    samples = np.zeros((len(sizes), iters, 8), np.int32)
    for l, n in enumerate(sizes):
        _, _, _, ua, ub = scene.two_view_matches(n, seed=40 + l)
        lists[l, :n] = _match_array(ua, ub)
        samples[l] = np.random.default_rng(l).integers(0, n, (iters, 8))
    dev = "cuda:0"
    d_m = torch.from_numpy(lists.view(np.uint8).reshape(-1)).to(dev)
    d_cnt = torch.tensor(sizes, dtype=torch.int32, device=dev)
    d_s = torch.from_numpy(samples.reshape(-1)).to(dev)
    d_F = torch.zeros(len(sizes) * 9, dtype=torch.float64, device=dev)
    d_inl = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
    d_found = torch.full((len(sizes),), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    assert ctx.lib.yv_f_ransac_batch(ctx.handle, d_m.data_ptr(), stride, d_cnt.data_ptr(), len(sizes), d_s.data_ptr(),
                                     iters * 8, iters, 0.1, d_F.data_ptr(), d_inl.data_ptr(), d_found.data_ptr(),
                                     None) == 0
    ctx.sync()
    F, inl, found = d_F.cpu().numpy().reshape(-1, 3, 3), d_inl.cpu().numpy(), d_found.cpu().numpy()
    for l, n in enumerate(sizes):
        ofound, oF, oinl = oracle.f_ransac(lists[l, :n], samples[l], 0.1)
        assert bool(found[l]) == ofound
        if ofound:
            assert inl[l] == oinl
            np.testing.assert_array_equal(F[l], oF)
