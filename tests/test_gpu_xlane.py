"""The in-wave butterflies of ya_vo_amd/csrc/yavo_xlane.h (DPP and gfx950 permlane swaps), which the pose LM's
fixed-order reduce-scatter and the matcher's row maxima rely on, checked lane by lane (yv_debug_xlane)."""
import ctypes

import numpy as np
import pytest

import ya_vo_amd as yv

pytestmark = pytest.mark.gpu


def test_xlane_butterflies(ctx):
    import torch
    lib = yv.load_library()
    lib.yv_debug_xlane.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.yv_debug_xlane.restype = ctypes.c_int
    out = torch.full((8, 64), -1, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    assert lib.yv_debug_xlane(ctypes.c_void_p(out.data_ptr()), None) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    lane = np.arange(64)
    for row, off in enumerate((1, 2, 4, 8)):
        np.testing.assert_array_equal(o[row], lane ^ off, err_msg=f"xor {off}")
    # half exchanges: every lane ends with {its own kept value, its partner's matching value} (lo = lane for the
    # lane with bit OFF clear, hi = 100 + lane for the lane with it set)
    for r0, off in ((4, 16), (6, 32)):
        up = (lane & off) != 0
        own = np.where(up, 100 + lane, lane)
        partner = np.where(up, 100 + (lane ^ off), lane ^ off)
        got = np.sort(o[r0:r0 + 2].T, axis=1)
        want = np.sort(np.stack([own, partner], 1), axis=1)
        np.testing.assert_array_equal(got, want, err_msg=f"swap {off}")
