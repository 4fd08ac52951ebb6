"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the committed golden fixtures.

Bar: bit-exact for everything here -- FAST candidate counts, top-K order and Harris responses (float, but
computed operation-for-operation like the oracle with contraction off), BRIEF bits, match indices /
distances and the filtered lists.
"""
import os

import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd.synth import synth_frame

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _crops():
    return np.load(os.path.join(GOLDEN, "kitti_crops.npz"))


def _images():
    c = _crops()
    rng = np.random.default_rng(7)
    return {
        "synth_kitti_1234": synth_frame(1234, 0, 0),
        "synth_kitti_77_f5": synth_frame(77, 5, 15),
        "crop_epilines": c["epilines"],
        "crop_epilinesOpencv": c["epilinesOpencv"],
        "uniform_noise": rng.integers(0, 256, (376, 1241)).astype(np.uint8),  # ~17k candidates
        "flat": np.full((64, 80), 128, np.uint8),                            # no candidates
        "tiny_9x9": rng.integers(0, 256, (9, 9)).astype(np.uint8),
        "odd_shape": synth_frame(5, 3, 7, 131, 203),
        "checker": (np.indices((96, 160)).sum(0) % 2 * 255).astype(np.uint8),
    }


@pytest.mark.parametrize("name", list(_images().keys()))
def test_detect_matches_oracle(ctx, oracle, name):
    img = _images()[name]
    rc, resp, nc = ctx.detect(img, 2000)
    orc, oresp, onc = oracle.fast(img, 2000)
    assert nc == onc
    np.testing.assert_array_equal(rc, orc)
    np.testing.assert_array_equal(resp.view(np.uint32), oresp.view(np.uint32))


@pytest.mark.parametrize("name", ["synth_kitti_1234", "crop_epilines", "crop_epilinesOpencv", "uniform_noise",
                                  "odd_shape", "checker"])
def test_detect_eigen_flavour_matches_oracle(ctx, oracle, name):
    """HAVE_EIGEN's cv::eigen (Eigen 3.4 SelfAdjointEigenSolver<MatrixXf>, yv_set_harris_eigen(1)): candidate set,
    responses and the top-2000 order bit-identical to the oracle's restatement."""
    img = _images()[name]
    ctx.set_harris_eigen(1)
    oracle.set_harris_eigen(1)
    try:
        rc, resp, nc = ctx.detect(img, 2000)
        orc, oresp, onc = oracle.fast(img, 2000)
    finally:
        ctx.set_harris_eigen(0)
        oracle.set_harris_eigen(0)
    assert nc == onc
    np.testing.assert_array_equal(rc, orc)
    np.testing.assert_array_equal(resp.view(np.uint32), oresp.view(np.uint32))


def test_batch_eigen_flavour_matches_oracle(ctx, oracle):
    """The fused batch detect kernel with the HAVE_EIGEN flavour: keypoints of every image equal the oracle's."""
    import torch
    frames = [synth_frame(9, 2 * k, 5 * k) for k in range(3)]
    offsets = np.fromfile(os.path.join(GOLDEN, "brief_offsets_mt19937_42.bin"), np.int8).reshape(256, 4)
    H, W = frames[0].shape
    d = torch.from_numpy(np.stack(frames)).to("cuda:0")
    b = yv.Batch(ctx, 3, H, W, 2000, 0)
    ctx.set_harris_eigen(1)
    oracle.set_harris_eigen(1)
    try:
        b.run(d.data_ptr(), 3, W, H * W, 20)
        ctx.sync()
        v = b.view()
        kpc = ctx.download(v.kp_count, np.int32, 3)
        for i, img in enumerate(frames):
            orc, _, _ = oracle.fast(img, 2000)
            kps = ctx.download(v.keypoints + i * 2000 * 48, yv.KEYPOINT_DTYPE, kpc[i])
            np.testing.assert_array_equal(kps, oracle.brief(img, orc, offsets))
    finally:
        ctx.set_harris_eigen(0)
        oracle.set_harris_eigen(0)
        b.close()


@pytest.mark.parametrize("max_kp", [0, 1, 7, 100, 1999, 2000])
def test_detect_cut_sizes(ctx, oracle, max_kp):
    img = synth_frame(1234, 0, 0)
    rc, resp, nc = ctx.detect(img, max_kp)
    orc, oresp, onc = oracle.fast(img, max_kp)
    assert nc == onc and len(rc) == min(max_kp, onc)
    np.testing.assert_array_equal(rc, orc)
    np.testing.assert_array_equal(resp, oresp)


def test_detect_large_cut(ctx, oracle):
    img = np.random.default_rng(3).integers(0, 256, (376, 1241)).astype(np.uint8)
    ctx.set_fast_params(40, 4096)
    try:
        rc, resp, nc = ctx.detect(img, 4096)
    finally:
        ctx.set_fast_params(40, 2000)
    orc, oresp, onc = oracle.fast(img, 4096)
    np.testing.assert_array_equal(rc, orc)
    np.testing.assert_array_equal(resp, oresp)


def test_detect_golden(ctx):
    g = np.load(os.path.join(GOLDEN, "fast_golden.npz"))
    c = _crops()
    for name, img in (("crop_epilines", c["epilines"]), ("synth_1234_f1", synth_frame(1234, 1, 3))):
        rc, resp, nc = ctx.detect(img, 2000)
        assert nc == int(g[name + "__ncand"][0])
        np.testing.assert_array_equal(rc, g[name + "__rc"])
        np.testing.assert_array_equal(resp, g[name + "__resp"])


@pytest.mark.parametrize("name", ["synth_kitti_1234", "crop_epilines", "uniform_noise", "odd_shape"])
def test_describe_matches_oracle(ctx, oracle, offsets, name):
    img = _images()[name]
    orc, _, _ = oracle.fast(img, 2000)
    k = ctx.describe(img, orc)
    ok = oracle.brief(img, orc, offsets)
    np.testing.assert_array_equal(k, ok)


def test_describe_boundary_and_out_of_buffer(ctx, oracle, offsets):
    img = synth_frame(9, 0, 0, 60, 90)
    H, W = img.shape
    # row H-8 / col W-8 pass checkBoundry and read past the row end / buffer end (reference: UB -> 0)
    rc = np.array([[8, 8], [H - 8, W - 8], [30, 45], [7, 20], [20, W - 7], [H - 8, 40], [52, W - 8],
                   [H - 9, W - 9], [8, W - 8]], np.int32)
    np.testing.assert_array_equal(ctx.describe(img, rc), oracle.brief(img, rc, offsets))
    assert len(ctx.describe(img, np.zeros((0, 2), np.int32))) == 0


@pytest.mark.parametrize("W", [1321, 1700])
def test_describe_wide_image(ctx, oracle, offsets, W):
    """Rows wider than 1320 px: the band has more 16-B words than four per thread, so its first 4 x 1024 words come
    by LDS-DMA and the rest through registers (brief_kernel), each with its own column-W patch."""
    img = synth_frame(3, 0, 0, 120, W)
    orc, _, _ = oracle.fast(img, 2000)
    assert len(orc) > 100
    np.testing.assert_array_equal(ctx.describe(img, orc), oracle.brief(img, orc, offsets))


def test_describe_after_new_offsets(ctx, oracle, offsets):
    """The batch forms the tests' LDS offsets once per offsets table: a new table (yv_set_brief_offsets) between two
    calls on the same workspace must take effect, and restoring the first one must too."""
    img = _images()["synth_kitti_1234"]
    orc, _, _ = oracle.fast(img, 2000)
    other = np.random.default_rng(5).integers(-8, 9, offsets.shape).astype(np.int8)
    try:
        np.testing.assert_array_equal(ctx.describe(img, orc), oracle.brief(img, orc, offsets))
        ctx.set_brief_offsets(other)
        np.testing.assert_array_equal(ctx.describe(img, orc), oracle.brief(img, orc, other))
    finally:
        ctx.set_brief_offsets(offsets)
    np.testing.assert_array_equal(ctx.describe(img, orc), oracle.brief(img, orc, offsets))


def test_describe_golden(ctx):
    b = np.load(os.path.join(GOLDEN, "brief_golden.npz"))
    g = np.load(os.path.join(GOLDEN, "fast_golden.npz"))
    img = synth_frame(1234, 0, 0)
    np.testing.assert_array_equal(ctx.describe(img, g["synth_1234_f0__rc"]), b["synth_1234_f0"])


def _rand_kp(n, rng, pool=None):
    k = np.zeros(n, yv.KEYPOINT_DTYPE)
    k["x"] = rng.integers(0, 376, n)
    k["y"] = rng.integers(0, 1241, n)
    k["id"] = rng.permutation(n)
    if pool is None:
        k["featVec"] = rng.integers(0, 256, (n, 32))
    else:
        k["featVec"] = pool[rng.integers(0, len(pool), n)]
    return k


# train lists <= 2048 run the FP4 MFMA matcher (the key's 11-bit train index: 2048 is its last size), longer ones the
# int8 +-1 form; the pool of 37 descriptors makes most minima ties
@pytest.mark.parametrize("nq,nt", [(1970, 1970), (1, 1), (7, 4096), (4096, 33), (513, 511), (5, 0), (2048, 2048),
                                   (65, 2049)])
def test_match_matches_oracle(ctx, oracle, nq, nt):
    rng = np.random.default_rng(nq * 131 + nt)
    pool = rng.integers(0, 256, (37, 32)).astype(np.uint8)  # few distinct descriptors: many exact ties
    q = _rand_kp(nq, rng, pool if nq % 2 else None)
    t = _rand_kp(nt, rng, pool)
    m = ctx.match_features(q, t)
    np.testing.assert_array_equal(m, oracle.match(q, t))


def test_match_and_filter_golden(ctx):
    g = np.load(os.path.join(GOLDEN, "match_golden.npz"))
    b = np.load(os.path.join(GOLDEN, "brief_golden.npz"))
    m = ctx.match_features(b["synth_1234_f0"], b["synth_1234_f1"])
    np.testing.assert_array_equal(m, g["matches"])
    np.testing.assert_array_equal(ctx.filter_matches(m, 20), g["filtered"])


@pytest.mark.parametrize("thr", [0, 20, 64, 300])
def test_filter_matches_oracle(ctx, oracle, thr):
    rng = np.random.default_rng(thr)
    m = np.zeros(3000, yv.MATCH_DTYPE)
    m["distance"] = rng.integers(0, 120, 3000)
    m["pt1"]["id"] = np.arange(3000)
    m["pt2"]["x"] = rng.integers(0, 376, 3000)
    np.testing.assert_array_equal(ctx.filter_matches(m, thr), oracle.remove_outliers(m, thr))
    m["distance"] = 2**31 - 1
    assert len(ctx.filter_matches(m, thr)) == len(oracle.remove_outliers(m, thr)) == 0


def _device_frames(ctx, frames):
    """Copy a [N, H, W] uint8 stack to device memory owned by torch (kept alive by the caller)."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(frames)).to("cuda:0")
    torch.cuda.synchronize()
    return t


@pytest.mark.parametrize("k9", [[2, 9, 25, 44, 96, 44, 25, 9, 2], [0, 0, 0, 28, 200, 28, 0, 0, 0]])
def test_batch_blur_custom_taps(ctx, oracle, k9):
    """The detect kernel's fused blur with other tap sets (yv_set_blur_kernel): taps <= 127 take the int8
    matrix-core horizontal pass (its accumulator bias is 128 x the taps' sum), a tap above 127 the v_dot4 form; both
    byte-equal to the oracle's blur with the same taps, a border image shape included."""
    import torch  # noqa: F401
    default = np.array(yv.DEFAULT_BLUR_KERNEL, np.uint16)
    for H, W in ((376, 1241), (77, 150)):
        frames = np.stack([synth_frame(5 + i, i, 2 * i, H, W) for i in range(2)])
        b = yv.Batch(ctx, 2, H, W, 2000, 0)
        try:
            ctx.set_blur_kernel(np.array(k9, np.uint16))
            d = _device_frames(ctx, frames)
            b.run(d.data_ptr(), 2, W, H * W, 20)
            ctx.sync()
            v = b.view()
            bp = v.blur_pitch
            for i in range(2):
                blur = ctx.download(v.blurred + i * H * bp, np.uint8, H * bp).reshape(H, bp)[:, :W]
                np.testing.assert_array_equal(blur, oracle.blur(frames[i], np.array(k9, np.uint16)))
        finally:
            ctx.set_blur_kernel(default)
            b.close()


def test_batch_pipeline_matches_oracle(ctx, oracle, offsets):
    """Stereo sequence through the device pipeline: images [L0, R0, L1, R1, ...], pairs temporal
    (L_{k-1} -> L_k, as buildInitMap / reinitialize) and stereo (L_k -> R_k); two runs chained through the
    carry slot.  Every output equals the oracle."""
    import torch  # noqa: F401
    H, W, n_frames = 376, 1241, 3
    seq = [(synth_frame(31, k, 3 * k), synth_frame(31, k, 3 * k + 8)) for k in range(2 * n_frames)]
    b = yv.Batch(ctx, 2 * n_frames, H, W, 2000, 2 * n_frames)
    carry = 2 * n_frames
    pairs = []
    for k in range(n_frames):
        pairs.append((carry if k == 0 else 2 * (k - 1), 2 * k))  # temporal
        pairs.append((2 * k, 2 * k + 1))                          # stereo
    b.set_pairs(pairs)
    ref_kp = {}
    for run in range(2):
        frames = np.stack([im for k in range(run * n_frames, (run + 1) * n_frames) for im in seq[k]])
        d = _device_frames(ctx, frames)
        b.run(d.data_ptr(), len(frames), W, H * W, 20, carry_from=2 * (n_frames - 1))
        ctx.sync()
        v = b.view()
        kpc = ctx.download(v.kp_count, np.int32, b.max_images + 1)
        detc = ctx.download(v.det_count, np.int32, b.max_images + 1)
        candc = ctx.download(v.cand_count, np.uint32, b.max_images + 1)
        for i, img in enumerate(frames):
            orc, oresp, onc = oracle.fast(img, 2000)
            assert candc[i] == onc and detc[i] == len(orc)
            rc = ctx.download(v.det_rc + i * 2000 * 8, np.int32, 2 * detc[i]).reshape(-1, 2)
            np.testing.assert_array_equal(rc, orc)
            kps = ctx.download(v.keypoints + i * 2000 * 48, yv.KEYPOINT_DTYPE, kpc[i])
            ok = oracle.brief(img, orc, offsets)
            np.testing.assert_array_equal(kps, ok)
            bp = v.blur_pitch  # 128-B aligned row pitch >= W + 1 (the padding columns are not part of the image)
            assert bp % 128 == 0 and bp > W
            blur = ctx.download(v.blurred + i * H * bp, np.uint8, H * bp).reshape(H, bp)[:, :W]
            np.testing.assert_array_equal(blur, oracle.blur(img))
            ref_kp[(run, i)] = ok
        mc = ctx.download(v.match_count, np.int32, len(pairs))
        fc = ctx.download(v.filt_count, np.int32, len(pairs))
        for p, (qi, ti) in enumerate(pairs):
            if qi == carry:
                if run == 0:
                    assert mc[p] == 0  # empty carry slot on the first run: nothing to match
                    continue
                qk = ref_kp[(run - 1, 2 * (n_frames - 1))]
            else:
                qk = ref_kp[(run, qi)]
            tk = ref_kp[(run, ti)]
            om = oracle.match(qk, tk)
            of = oracle.remove_outliers(om, 20)
            assert mc[p] == len(om) and fc[p] == len(of)
            m = ctx.download(v.matches + p * 2000 * 100, yv.MATCH_DTYPE, mc[p])
            f = ctx.download(v.filtered + p * 2000 * 100, yv.MATCH_DTYPE, fc[p])
            np.testing.assert_array_equal(m, om)
            np.testing.assert_array_equal(f, of)
    b.close()


def test_large_batch_tail_matches_oracle(ctx, oracle, offsets):
    """A 642-image batch (321 stereo frames, the bench's layout and pairs): the candidate-key buffer offsets pass
    2^31 bytes at image 592 (453,744 keys x 8 B per image), so the images on both sides of that boundary and the last
    ones are compared with the oracle: candidate counts, FAST + Harris + top-2000 rows / columns, the blurred image,
    BRIEF keypoints, and the temporal + stereo Matches / removeOutliers of the pairs between them
    (src/FastDetector.cc:277-369, src/BriefDescriptor.cc:86-231)."""
    from ya_vo_amd.synth import synth_stereo_batch
    H, W, n_frames, thr = 376, 1241, 321, 20
    frames = synth_stereo_batch(4242, n_frames)
    n_img = len(frames)
    assert (n_img - 1) * (H - 8) * (W - 8) * 8 > 2 ** 31
    pairs = []
    for k in range(n_frames):
        if k > 0:
            pairs.append((2 * (k - 1), 2 * k))  # temporal L_{k-1} -> L_k
        pairs.append((2 * k, 2 * k + 1))        # stereo L_k -> R_k
    b = yv.Batch(ctx, n_img, H, W, 2000, len(pairs))
    b.set_pairs(pairs)
    d = _device_frames(ctx, frames)
    b.run(d.data_ptr(), n_img, W, H * W, thr, carry_from=-1)
    ctx.sync()
    v = b.view()
    kpc = ctx.download(v.kp_count, np.int32, b.max_images + 1)
    detc = ctx.download(v.det_count, np.int32, b.max_images + 1)
    candc = ctx.download(v.cand_count, np.uint32, b.max_images + 1)
    check = [0, 1, 590, 591, 592, 593, 594, 595, n_img - 4, n_img - 3, n_img - 2, n_img - 1]
    ref = {}
    bp = v.blur_pitch
    for i in check:
        img = frames[i]
        orc, _, onc = oracle.fast(img, 2000)
        assert candc[i] == onc and detc[i] == len(orc), i
        rc = ctx.download(v.det_rc + i * 2000 * 8, np.int32, 2 * detc[i]).reshape(-1, 2)
        np.testing.assert_array_equal(rc, orc)
        blur = ctx.download(v.blurred + i * H * bp, np.uint8, H * bp).reshape(H, bp)[:, :W]
        np.testing.assert_array_equal(blur, oracle.blur(img))
        kps = ctx.download(v.keypoints + i * 2000 * 48, yv.KEYPOINT_DTYPE, kpc[i])
        ref[i] = oracle.brief(img, orc, offsets)
        np.testing.assert_array_equal(kps, ref[i])
    mc = ctx.download(v.match_count, np.int32, len(pairs))
    fc = ctx.download(v.filt_count, np.int32, len(pairs))
    compared = 0
    for p, (qi, ti) in enumerate(pairs):
        if qi not in ref or ti not in ref:
            continue
        om = oracle.match(ref[qi], ref[ti])
        of = oracle.remove_outliers(om, thr)
        assert mc[p] == len(om) and fc[p] == len(of)
        np.testing.assert_array_equal(ctx.download(v.matches + p * 2000 * 100, yv.MATCH_DTYPE, mc[p]), om)
        np.testing.assert_array_equal(ctx.download(v.filtered + p * 2000 * 100, yv.MATCH_DTYPE, fc[p]), of)
        compared += 1
    assert compared >= 8
    b.close()
    del d


def test_batch_is_deterministic_and_timed(ctx):
    H, W = 376, 1241
    frames = np.stack([synth_frame(2, k, 3 * k) for k in range(4)])
    d = _device_frames(ctx, frames)
    b = yv.Batch(ctx, 4, H, W, 2000, 3)
    b.set_pairs([(0, 1), (1, 2), (2, 3)])
    b.enable_timing(True)
    outs = []
    for _ in range(3):
        b.run(d.data_ptr(), 4, W, H * W, 20)
        ctx.sync()
        v = b.view()
        outs.append(ctx.download(v.matches, yv.MATCH_DTYPE, 3 * 2000))
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[0], outs[2])
    ms, n = b.stage_times()
    assert n == 3 and np.all(ms[:5] > 0) and np.all(ms[5:] == 0)  # no tracks set: stages 5-6 idle
    b.enable_timing(2)  # detect-only events (bench.py's timed region): same results, only ms[0]
    b.run(d.data_ptr(), 4, W, H * W, 20)
    ctx.sync()
    np.testing.assert_array_equal(ctx.download(b.view().matches, yv.MATCH_DTYPE, 3 * 2000), outs[0])
    ms, n = b.stage_times()
    assert n == 1 and ms[0] > 0 and np.all(ms[1:] == 0)
    b.close()


def test_cpp_frontend_demo_matches_oracle(oracle, offsets, tmp_path):
    """The C++ host side (ya_vo_amd/frontend: FastDetector / Brief over the C ABI, LoopHandler-shaped
    driver) produces the oracle's keypoints and matches for a short synthetic sequence."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "ya_vo_amd", "bin", "yavo_frontend_demo")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(root, "ya_vo_amd", "frontend")], check=True)
    H, W, n = 376, 1241, 3
    frames = np.stack([synth_frame(555, k, 3 * k) for k in range(n)])
    raw = tmp_path / "frames.raw"
    with open(raw, "wb") as f:
        f.write(np.array([n, H, W], np.int32).tobytes())
        f.write(frames.tobytes())
    out = tmp_path / "out.bin"
    off = os.path.join(GOLDEN, "brief_offsets_mt19937_42.bin")
    env = dict(os.environ)
    r = subprocess.run([exe, str(raw), off, str(out)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    buf = open(out, "rb").read()
    pos = 0

    def take(dtype, count):
        nonlocal pos
        a = np.frombuffer(buf, dtype, count, pos)
        pos += a.nbytes
        return a

    prev = None
    for k in range(n):
        nk = int(take(np.int32, 1)[0])
        kps = take(yv.KEYPOINT_DTYPE, nk)
        orc, _, _ = oracle.fast(frames[k], 2000)
        ok = oracle.brief(frames[k], orc, offsets)
        np.testing.assert_array_equal(kps, ok)
        if prev is not None:
            nm = int(take(np.int32, 1)[0])
            m = take(yv.MATCH_DTYPE, nm)
            nf = int(take(np.int32, 1)[0])
            f = take(yv.MATCH_DTYPE, nf)
            om = oracle.match(prev, ok)
            np.testing.assert_array_equal(m, om)
            np.testing.assert_array_equal(f, oracle.remove_outliers(om, 20))
        prev = ok
    assert pos == len(buf)
