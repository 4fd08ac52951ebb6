"""yavo_fp64.h's division, reciprocal and square root without the no-op range handling against the compiler's
operators, bit for bit, on random operands across the whole double range (both paths) and on the guard boundaries
(yv_debug_fp64)."""
import ctypes

import numpy as np
import pytest

import ya_vo_amd as yv

pytestmark = pytest.mark.gpu


def _operands(rng, n):
    """|x| = m * 2^e with e spread over the guard range and beyond, random signs; plus boundary exponents and specials."""
    def draw(k, lo, hi):
        return rng.uniform(1, 2, k) * np.exp2(rng.integers(lo, hi, k).astype(np.float64)) * rng.choice([-1.0, 1.0], k)
    a = np.concatenate([draw(n, -320, 321), draw(n // 4, -1074, 1024), draw(n // 4, -60, 60)])
    b = np.concatenate([draw(n, -320, 321), draw(n // 4, -1074, 1024), draw(n // 4, -60, 60)])
    edges = []
    for e in (-701, -700, -699, -301, -300, -299, 299, 300, 301, 302, 999, 1000, 1001):
        for m in (1.0, np.nextafter(1.0, 2.0), np.nextafter(2.0, 1.0), 1.5):
            edges.append(m * 2.0 ** e)
    edges = np.array(edges + [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308])
    ea, eb = np.meshgrid(np.concatenate([edges, -edges]), np.concatenate([edges, -edges]))
    return np.concatenate([a, ea.ravel()]), np.concatenate([b, eb.ravel()])


def _same(x, y):
    return (x.view(np.uint64) == y.view(np.uint64)) | (np.isnan(x) & np.isnan(y))


def test_fp64_forms_match_operators(ctx):
    import torch
    lib = yv.load_library()
    lib.yv_debug_fp64.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.yv_debug_fp64.restype = ctypes.c_int
    rng = np.random.default_rng(11)
    a, b = _operands(rng, 1 << 21)
    # an exact quotient family: a = b * k for small integers k (ties and exact results)
    k = rng.integers(1, 1 << 20, 1 << 16).astype(np.float64)
    bb = rng.uniform(1, 2, len(k)) * np.exp2(rng.integers(-250, 250, len(k)).astype(np.float64))
    a, b = np.concatenate([a, bb * k]), np.concatenate([b, bb])
    da = torch.from_numpy(a).to("cuda:0")
    db = torch.from_numpy(b).to("cuda:0")
    out = torch.zeros((len(a), 8), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    assert lib.yv_debug_fp64(ctypes.c_void_p(da.data_ptr()), ctypes.c_void_p(db.data_ptr()), len(a),
                             ctypes.c_void_p(out.data_ptr()), None) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    fast_div = (o[:, 7] % 2) == 1
    fast_sqrt = o[:, 7] >= 2
    assert fast_div.sum() > (1 << 20) and (~fast_div).sum() > 1000  # both paths exercised
    assert fast_sqrt.sum() > (1 << 20) and (~fast_sqrt).sum() > 1000
    for col, ref, what in ((0, 1, "div"), (2, 3, "rcp"), (4, 5, "sqrt"), (6, 1, "Rcp64.div")):
        bad = ~_same(o[:, col], o[:, ref])
        assert not bad.any(), f"{what}: {bad.sum()} differ, e.g. a={a[bad][:3]} b={b[bad][:3]}"
    # and the compiler's operators are IEEE: numpy agrees (no FTZ / approximate division in the build)
    with np.errstate(all="ignore"):
        assert _same(o[:, 1], a / b).all()
        assert _same(o[:, 3], 1.0 / b).all()
        assert _same(o[:, 5], np.sqrt(a)).all()
