"""GPU parity of cv::findEssentialMat (RANSAC) + cv::recoverPose with the CPU oracle
(oracle/yavo_oracle_essential.c): E, the inlier mask, found flag, RANSAC statistics, R, t and the cheirality count,
bit for bit, through the host drop-ins (yv_find_essential / yv_recover_pose) and the batched workspace."""
import numpy as np
import pytest

import ya_vo_amd as yv
from epipolar_scene import K_KITTI, two_view_scene

pytestmark = pytest.mark.gpu
FOCAL, PP = 718.856, (607.1928, 185.2157)


@pytest.mark.parametrize("n,outl,seed", [(600, 0.0, 0), (600, 0.3, 1), (2000, 0.2, 2), (40, 0.4, 3), (6, 0.0, 4),
                                         (5, 0.0, 5)])
def test_find_essential_host_matches_oracle(ctx, oracle, n, outl, seed):
    p1, p2, _, _ = two_view_scene(n, outlier_frac=outl, seed=seed)
    ok, E, mask = ctx.find_essential(p1, p2, FOCAL, PP)
    ook, oE, omask, _ = oracle.find_essential(p1.astype(np.float32), p2.astype(np.float32), FOCAL, PP)
    assert ok == ook
    np.testing.assert_array_equal(E, oE if ook else np.zeros((3, 3)))
    np.testing.assert_array_equal(mask, omask)
    good, R, t = ctx.recover_pose(E, p1, p2, K_KITTI)
    og, oR, ot, _ = oracle.recover_pose(E, p1.astype(np.float32), p2.astype(np.float32), K_KITTI)
    assert good == og
    np.testing.assert_array_equal(R, oR)
    np.testing.assert_array_equal(t, ot)


def test_find_essential_host_small(ctx):
    p1, p2, _, _ = two_view_scene(4, seed=7)
    ok, E, mask = ctx.find_essential(p1, p2, FOCAL, PP)
    assert not ok and not E.any() and not mask.any()


@pytest.mark.parametrize("capacity", [8, 9])
def test_essential_batch_matches_oracle(ctx, oracle, capacity):
    """Lists of different lengths (incl. n < 5, n == 5 and pure noise) in one batched call.  A workspace of <= 8 lists
    runs the five-point solver's latency form (one iteration per 16-lane row, 1024-iteration rounds, subsets drawn in
    parallel from the RNG table: the 64-point list re-draws often, the noise list needs all 1000 iterations), a larger
    one the throughput form (one iteration per lane, 64-iteration rounds, sequential draws): both give the oracle's
    results."""
    import torch
    cases = [(2000, 0.2, 10), (0, 0.0, 11), (4, 0.0, 12), (5, 0.0, 13), (300, 0.5, 14), (150, 1.0, 15), (64, 0.1, 16),
             (1000, 0.0, 17)]
    P, stride = len(cases), 2048
    pts1 = np.zeros((P, stride, 2), np.float32)
    pts2 = np.zeros((P, stride, 2), np.float32)
    counts = np.zeros(P, np.int32)
    for p, (n, outl, seed) in enumerate(cases):
        if n:
            a, b, _, _ = two_view_scene(n, outlier_frac=outl, seed=seed)
            pts1[p, :n], pts2[p, :n] = a, b
        counts[p] = n
    dev = "cuda:0"
    d1, d2 = torch.from_numpy(pts1).to(dev), torch.from_numpy(pts2).to(dev)
    dc = torch.from_numpy(counts).to(dev)
    dE = torch.zeros((P, 9), dtype=torch.float64, device=dev)
    dmask = torch.zeros((P, stride), dtype=torch.uint8, device=dev)
    dfound = torch.zeros(P, dtype=torch.int32, device=dev)
    dstats = torch.zeros((P, 3), dtype=torch.int32, device=dev)
    dR = torch.zeros((P, 9), dtype=torch.float64, device=dev)
    dt = torch.zeros((P, 3), dtype=torch.float64, device=dev)
    dgood = torch.zeros(P, dtype=torch.int32, device=dev)
    es = yv.Essential(ctx, max(P, capacity), stride)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        es.find(d1.data_ptr(), d2.data_ptr(), dc.data_ptr(), P, stride, dE.data_ptr(), dfound.data_ptr(),
                dmask.data_ptr(), dstats.data_ptr(), FOCAL, PP, stream=stream.cuda_stream)
        es.recover(dE.data_ptr(), d1.data_ptr(), d2.data_ptr(), dc.data_ptr(), P, stride, K_KITTI, dR.data_ptr(),
                   dt.data_ptr(), dgood.data_ptr(), stream=stream.cuda_stream)
    stream.synchronize()
    es.close()
    E, found, mask, stats = dE.cpu().numpy(), dfound.cpu().numpy(), dmask.cpu().numpy(), dstats.cpu().numpy()
    R, t, good = dR.cpu().numpy(), dt.cpu().numpy(), dgood.cpu().numpy()
    for p, (n, _, _) in enumerate(cases):
        ook, oE, omask, ost = oracle.find_essential(pts1[p, :n], pts2[p, :n], FOCAL, PP)
        assert bool(found[p]) == ook, p
        if not ook:
            assert not E[p].any() and not mask[p, :n].any()
            continue
        np.testing.assert_array_equal(E[p].reshape(3, 3), oE)
        np.testing.assert_array_equal(mask[p, :n].astype(bool), omask)
        assert tuple(stats[p]) == (ost["iters"], ost["models"], ost["best"]), p
        og, oR, ot, _ = oracle.recover_pose(oE, pts1[p, :n], pts2[p, :n], K_KITTI)
        assert good[p] == og
        np.testing.assert_array_equal(R[p].reshape(3, 3), oR)
        np.testing.assert_array_equal(t[p], ot)
