"""Synthetic two-view scenes for the findEssentialMat / recoverPose tests (KITTI intrinsics)."""
import numpy as np

K_KITTI = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]])


def two_view_scene(n, outlier_frac=0.0, seed=0, noise=0.0, angle=0.05, t=(0.2, 0.01, 1.0), rounded=True):
    """points1 in camera 1, points2 = R X + t in camera 2, projected with the KITTI K -> (p1, p2, R, t_unit)."""
    r = np.random.default_rng(seed)
    X = np.c_[r.uniform(-10, 10, n), r.uniform(-3, 3, n), r.uniform(5, 40, n)]
    c, s = np.cos(angle), np.sin(angle)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    t = np.asarray(t, np.float64)
    X2 = X @ R.T + t

    def proj(P):
        return (P / P[:, 2:3]) @ K_KITTI.T

    p1, p2 = proj(X)[:, :2], proj(X2)[:, :2]
    if noise:
        p1 = p1 + r.normal(0, noise, p1.shape)
        p2 = p2 + r.normal(0, noise, p2.shape)
    if rounded:
        p1, p2 = np.round(p1), np.round(p2)
    k = int(outlier_frac * n)
    if k:
        p2[:k] += r.uniform(-60, 60, (k, 2))
    return p1, p2, R, t / np.linalg.norm(t)


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
