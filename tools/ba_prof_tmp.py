import ctypes, sys, os, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import ya_vo_amd as yv
from ya_vo_amd import scene
ctx = yv.Context(0)
ctx.lib.yv_ba_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]
w = scene.ba_window(n_poses=20, n_landmarks=10000, obs=5, noise_px=1.0, seed=0)
ba = yv.BundleAdjuster(ctx, 20, 10000, 50000)
ba.set_problem(20, 1, 10000, w["ep"], w["el"], w["meas"], scene.K_KITTI)
for it in (1, 1, 1):
    ba.solve(w["poses0"], w["X0"], it)
    a = np.zeros(16); assert ctx.lib.yv_ba_debug_read(ba.handle, 16, a.ctypes.data, 16) == 0
    print("cycles pivot, load, factor, solve | bar1, update, bar2:", a[4:11])
