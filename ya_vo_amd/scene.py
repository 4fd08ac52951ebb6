"""Synthetic geometry for the PnP / triangulation / F-RANSAC rows: known
poses, 3D points and their projections, so every solver can be checked against ground truth.

Poses use Sophus::SE3d::data() order {qx, qy, qz, qw, tx, ty, tz} (T_cw, world -> camera).  Projections
follow the reference's edge (include/Optimizer.hpp:75-103): uv = (K (R X + t))[:2] / z.  K defaults to
KITTI seq 00's P0 (tests/calib.txt).
"""
from __future__ import annotations

import numpy as np

K_KITTI = np.array([[718.856, 0.0, 607.1928], [0.0, 718.856, 185.2157], [0.0, 0.0, 1.0]])


def quat_from_axis_angle(axis, angle) -> np.ndarray:
    axis = np.asarray(axis, np.float64)
    axis = axis / np.linalg.norm(axis)
    s = np.sin(angle / 2)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, np.cos(angle / 2)])


def quat_to_R(q) -> np.ndarray:
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def pose(q, t) -> np.ndarray:
    return np.concatenate([np.asarray(q, np.float64), np.asarray(t, np.float64)])


def transform(T, X) -> np.ndarray:
    return (quat_to_R(T[:4]) @ np.asarray(X, np.float64).T).T + T[4:]


def project(T, X, K=K_KITTI) -> np.ndarray:
    pc = transform(T, X)
    u = (K @ pc.T).T
    return u[:, :2] / u[:, 2:3]


def random_scene(n: int, seed: int = 0, noise_px: float = 0.0, outlier_frac: float = 0.0, K=K_KITTI):
    """n world points 4..40 m in front of a camera at T_true; returns (X [n,3], uv [n,2], T_true, outlier mask)."""
    rng = np.random.default_rng(seed)
    T_true = pose(quat_from_axis_angle(rng.normal(size=3), rng.uniform(0.02, 0.2)), rng.normal(scale=0.5, size=3))
    # points in camera coordinates, mapped back to the world
    z = rng.uniform(4.0, 40.0, n)
    xs = rng.uniform(-0.6, 0.6, n) * z
    ys = rng.uniform(-0.25, 0.25, n) * z
    pc = np.stack([xs, ys, z], 1)
    R = quat_to_R(T_true[:4])
    X = np.ascontiguousarray((R.T @ (pc - T_true[4:]).T).T)
    uv = project(T_true, X, K)
    if noise_px > 0:
        uv = uv + rng.normal(scale=noise_px, size=uv.shape)
    out = np.zeros(n, bool)
    if outlier_frac > 0:
        k = int(round(outlier_frac * n))
        idx = rng.choice(n, k, replace=False)
        uv[idx] += rng.uniform(20, 80, size=(k, 2)) * rng.choice([-1, 1], size=(k, 2))
        out[idx] = True
    return X, uv, T_true, out


def perturb(T, rng, rot=0.02, trans=0.1) -> np.ndarray:
    dq = quat_from_axis_angle(rng.normal(size=3), rot)
    x1, y1, z1, w1 = dq
    x2, y2, z2, w2 = T[:4]
    q = np.array([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2,
                  w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2])
    return pose(q / np.linalg.norm(q), T[4:] + rng.normal(scale=trans, size=3))


def two_view_matches(n: int, seed: int = 0, K=K_KITTI):
    """Two camera poses and n exact correspondences as MATCH_DTYPE-like fields: pixel (row, col) per
    the reference's convention (x = row, y = col), integer-rounded as KeyPoint stores them, plus the
    3D points.  Used for F-RANSAC and triangulation."""
    rng = np.random.default_rng(seed)
    Ta = pose([0, 0, 0, 1], [0, 0, 0])
    Tb = pose(quat_from_axis_angle([0.1, 1.0, 0.05], 0.05), [0.05, -0.02, -1.0])
    z = rng.uniform(5.0, 30.0, n)
    pc = np.stack([rng.uniform(-0.5, 0.5, n) * z, rng.uniform(-0.2, 0.2, n) * z, z], 1)
    X = pc  # Ta = identity
    ua = project(Ta, X, K)
    ub = project(Tb, X, K)
    return Ta, Tb, X, ua, ub


def ba_window(n_poses: int = 20, n_landmarks: int = 10000, obs: int = 5, noise_px: float = 1.0, seed: int = 0,
              K=K_KITTI, init_rot: float = 0.005, init_trans: float = 0.05, init_point: float = 0.1):
    """Sliding-window BA problem: n_poses keyframes moving ~1 m forward per frame with a
    slow yaw, n_landmarks points each observed by `obs` consecutive keyframes (pixel noise N(0, noise_px)), edges in
    landmark order.  Returns dict(poses_true, X_true, poses0, X0 (perturbed initial estimates, the first pose
    exact), ep, el, meas)."""
    rng = np.random.default_rng(seed)
    poses = []
    for k in range(n_poses):
        # camera k at world position c_k, looking along +z with yaw 0.01 k: T_cw = [R | -R c]
        q = quat_from_axis_angle([0.0, 1.0, 0.0], 0.01 * k)
        c = np.array([0.05 * np.sin(0.3 * k), 0.02 * k, 1.0 * k])
        R = quat_to_R(q)
        poses.append(pose(q, -R @ c))
    poses = np.array(poses)
    anchors = rng.integers(0, max(n_poses - obs + 1, 1), n_landmarks)
    X = np.zeros((n_landmarks, 3))
    for i, a in enumerate(anchors):
        z = rng.uniform(8.0, 40.0)
        pc = np.array([rng.uniform(-0.5, 0.5) * z, rng.uniform(-0.2, 0.2) * z, z])
        T = poses[a]
        X[i] = quat_to_R(T[:4]).T @ (pc - T[4:])
    ep, el, meas = [], [], []
    for i, a in enumerate(anchors):
        for k in range(a, min(a + obs, n_poses)):
            uv = project(poses[k], X[i:i + 1], K)[0] + rng.normal(scale=noise_px, size=2)
            ep.append(k)
            el.append(i)
            meas.append(uv)
    poses0 = poses.copy()
    for k in range(1, n_poses):
        poses0[k] = perturb(poses[k], rng, rot=init_rot, trans=init_trans)
    X0 = X + rng.normal(scale=init_point, size=X.shape)
    return dict(poses_true=poses, X_true=X, poses0=poses0, X0=X0, ep=np.array(ep, np.int32),
                el=np.array(el, np.int32), meas=np.array(meas, np.float64))
