"""The reference's LoopHandler loop (src/LoopHandler.cc) over the CPU oracle -- test infrastructure: the checker for
ya_vo_amd/frontend/loop_handler.cpp (the C++ LoopHandler over the C ABI).  Same state machine, same bookkeeping,
same primitives in the GPU kernels' sum orders (LK: sum_mode 1, pose LM: lm_sum_mode()), so the two trajectories
must agree bit for bit.

    INIT      buildInitMap (:532-652): matchFeatures -> removeOutliers(20) -> getFRANSAC (F unused) ->
              findEssentialMat(curr, prev) -> recoverPose -> pose = SE3(R, t)^-1 -> triangulate2View(first view)
    TRACKING  track (:132-165): pose guess = relativeMotion * last.pose -> trackLastFrame (world2Camera filter +
              pyramidal LK, :306-449) -> optimizePoseOnly (:730-861); fewer than 2 tracked or 100 inliers ->
              reinitialize (:168-296) + insertKeyFrame
"""
import math

import numpy as np

from ya_vo_amd import MATCH_DTYPE, lm_sum_mode

INT_MIN = -2147483648
FOCAL, PP = 718.8560, (607.1928, 185.2157)
IDENTITY = np.array([0, 0, 0, 1, 0, 0, 0], np.float64)
EVENT_FIELDS = ("frame", "kind", "keypoints", "matches_kept", "essential_found", "tracked", "inliers",
                "new_landmarks", "f_inliers")
FIRST, INIT_MAP, TRACKED, REINIT = 0, 1, 2, 3


def trunc_int(v):
    """cv::Point2i(double, double)'s conversion: truncation toward zero; out of int range / NaN -> INT_MIN (x86-64)."""
    v = float(v)
    if not (-2147483649.0 < v < 2147483648.0):
        return INT_MIN
    return int(math.trunc(v))


class Frame:
    def __init__(self, fid, img):
        self.id, self.img, self.pose = fid, img, IDENTITY.copy()
        self.kps = None
        self.features = []  # [kp_x (row), kp_y (col), map point index or None]


class LoopChain:
    def __init__(self, orc, K, offsets):
        self.orc, self.K, self.offsets = orc, np.asarray(K, np.float64).reshape(3, 3), offsets
        self.status = "INIT"
        self.last = self.curr = None
        self.rel = IDENTITY.copy()
        self.mps = []  # map point positions (index = ptID - 1)
        self.keyframes = set()
        self.poses, self.events = [], []
        self._ev = None
        self.rng = orc.mt19937(0)  # getFRANSAC's engine (loop_handler.hpp ransac_rng_{0})

    # ---- primitives ----
    def features(self, img):
        rc, _, _ = self.orc.fast(img, 2000)
        return self.orc.brief(img, rc, self.offsets)

    def matches(self):
        m = self.orc.match(self.last.kps, self.curr.kps)
        return self.orc.remove_outliers(m, 20) if len(m) else np.zeros(0, MATCH_DTYPE)

    def f_ransac(self, filt):
        """getFRANSAC(filterMatches, F, 400, 0.1) (src/3DHandler.cc:145-195; F unused, :222, :562): the inlier count
        of the best of 400 eight-point hypotheses, or 0 when fewer than 8 matches (no draws then)."""
        n = len(filt)
        if n < 8:
            return 0
        smp = self.rng.uniform_ints(0, n - 1, 8 * 400)
        ok, _, mi = self.orc.f_ransac(filt, smp, 0.1)
        return mi if ok else 0

    def essential_pose(self, filt):
        prev = np.stack([filt["pt1"]["x"], filt["pt1"]["y"]], 1).astype(np.float32).astype(np.float64)
        curr = np.stack([filt["pt2"]["x"], filt["pt2"]["y"]], 1).astype(np.float32).astype(np.float64)
        ok, E, _, _ = self.orc.find_essential(curr, prev, FOCAL, PP, 0.999, 1.0)
        self._ev["essential_found"] = int(ok)
        _, R, t, _ = self.orc.recover_pose(E, curr, prev, self.K)
        return self.orc.se3_from_Rt(R, t)

    def triangulate2view(self, filt, first_view):
        if len(filt) == 0:
            return 0
        _, X, ok = self.orc.triangulate_matches(self.last.pose, self.curr.pose, self.K, filt)
        n = 0
        for i in range(len(filt)):
            if not ok[i]:
                continue
            self.mps.append(X[i].copy())
            mp = len(self.mps) - 1
            if first_view:
                self.curr.features[i][2] = mp
                self.last.features[i][2] = mp
            else:
                self.curr.features.append([int(filt[i]["pt2"]["x"]), int(filt[i]["pt2"]["y"]), mp])
            n += 1
        return n

    # ---- the loop ----
    def build_init_map(self):
        filt = self.matches()
        self._ev["matches_kept"] = len(filt)
        for m in filt:
            self.last.features.append([int(m["pt1"]["x"]), int(m["pt1"]["y"]), None])
            self.curr.features.append([int(m["pt2"]["x"]), int(m["pt2"]["y"]), None])
        self._ev["f_inliers"] = self.f_ransac(filt)
        curr_pose = self.essential_pose(filt)
        self.curr.pose = self.orc.se3_inverse(curr_pose)
        self.keyframes.update((self.last.id, self.curr.id))
        self._ev["new_landmarks"] = self.triangulate2view(filt, True)
        self.rel = self.orc.se3_mul(self.curr.pose, self.orc.se3_inverse(self.last.pose))
        return True

    def track_last_frame(self):
        idx = [i for i, f in enumerate(self.last.features) if f[2] is not None]
        if not idx:
            return 0
        X = np.array([self.mps[self.last.features[i][2]] for i in idx])
        proj = self.orc.world2camera(X, self.curr.pose, self.K)
        prev_pts, keep = [], []
        for k, i in enumerate(idx):
            nx = trunc_int(proj[k, 1] / proj[k, 2])
            ny = trunc_int(proj[k, 0] / proj[k, 2])
            if not (nx < 0 or ny < 0):
                f = self.last.features[i]
                prev_pts.append((f[1], f[0]))  # Point2i(kp.y, kp.x)
                keep.append(i)
        if not keep:
            return 0
        nxt, st, _, _ = self.orc.lk(self.last.img, self.curr.img, np.array(prev_pts, np.float32), 11, 3, 30, 0.01,
                                    0.001, sum_mode=1)
        good = 0
        for k, i in enumerate(keep):
            if st[k] and self.last.features[i][2] is not None:
                self.curr.features.append([trunc_int(nxt[k, 1]), trunc_int(nxt[k, 0]), self.last.features[i][2]])
                good += 1
        return good

    def optimize_pose_only(self):
        fi = [i for i, f in enumerate(self.curr.features) if f[2] is not None]
        X = np.array([self.mps[self.curr.features[i][2]] for i in fi]).reshape(-1, 3)
        uv = np.array([(self.curr.features[i][0], self.curr.features[i][1]) for i in fi], np.float64).reshape(-1, 2)
        T, out, inl = self.orc.pose_lm(X, uv, self.K, self.curr.pose, lm_sum_mode(1))
        self.curr.pose = T
        for k, i in enumerate(fi):
            if out[k]:
                self.curr.features[i][2] = None
        return int(inl)

    def track(self):
        self.curr.pose = self.orc.se3_mul(self.rel, self.last.pose)
        good = self.track_last_frame()
        self._ev["tracked"] = good
        if good < 2:
            return False
        inl = self.optimize_pose_only()
        self._ev["inliers"] = inl
        if inl < 100:
            return False
        self.rel = self.orc.se3_mul(self.curr.pose, self.orc.se3_inverse(self.last.pose))
        return True

    def reinitialize(self):
        self.curr.features = []
        filt = self.matches()
        self._ev["matches_kept"] = len(filt)
        self._ev["f_inliers"] = self.f_ransac(filt)
        curr_pose = self.orc.se3_inverse(self.essential_pose(filt))
        self.curr.pose = self.orc.se3_mul(curr_pose, self.last.pose)
        self._ev["new_landmarks"] = self.triangulate2view(filt, False)
        self.rel = self.orc.se3_mul(self.curr.pose, self.orc.se3_inverse(self.last.pose))
        return True

    def add_frame(self, k, fid, img):
        self.curr = Frame(fid, img)
        self.curr.kps = self.features(img)
        self._ev = dict(frame=k, kind=FIRST, keypoints=len(self.curr.kps), matches_kept=0, essential_found=0,
                        tracked=0, inliers=-1, new_landmarks=0, f_inliers=0)
        if self.status == "INIT":
            if self.last is not None:
                if self.build_init_map():
                    self.status = "TRACKING"
                self._ev["kind"] = INIT_MAP
        elif self.status == "TRACKING":
            self._ev["kind"] = TRACKED
            if not self.track():
                self.reinitialize()
                self.keyframes.add(self.curr.id)
                self._ev["kind"] = REINIT
        self.last = self.curr
        self.poses.append(self.curr.pose.copy())
        self.events.append(self._ev)

    def run(self, frames):
        for k, img in enumerate(frames):
            self.add_frame(k, k + 1, img)
        return np.array(self.poses), self.events
