#!/usr/bin/env python3
"""How much the FAST keypoint output depends on the two build-dependent choices SURVEY.md section 7 names
(hard parts 1 and 2), measured with the oracle on the reference's own images (full frames, read from
/root/reference/tests when present -- in the build container only) and on synthetic KITTI-shaped frames:

1. cv::eigen's flavour (src/FastDetector.cc:265): OpenCV's JacobiImpl_ (no Eigen) vs HAVE_EIGEN's
   SelfAdjointEigenSolver<MatrixXf>: responses whose bits differ, and whether the top-2000 cut (set / order)
   changes.
2. std::sort's unstable tie order (src/FastDetector.cc:343-345): libstdc++'s actual result vs the canonical order
   (response descending, row-major index ascending) both paths use: ties that straddle the 2000 cut, and whether the
   cut's set / order differ.

    python tools/eigen_flavour_report.py [--out profiles/r02/eigen_flavour.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
K = 2000


def images():
    out = {}
    ref = "/root/reference/tests"
    if os.path.isdir(ref):
        from PIL import Image
        for name in ("epilines.png", "epilinesOpencv.png"):
            p = os.path.join(ref, name)
            if os.path.exists(p):
                out["reference:" + name] = np.asarray(Image.open(p).convert("L"), np.uint8)
    from ya_vo_amd.synth import synth_frame
    for k in range(6):
        out[f"synth_1234_f{k}"] = synth_frame(1234, k, 3 * k)
    out["uniform_noise_s7"] = np.random.default_rng(7).integers(0, 256, (376, 1241)).astype(np.uint8)
    return out


def analyse(orc, img):
    H, W = img.shape
    res = {"shape": [H, W]}
    per = {}
    for fl in (0, 1):
        orc.set_harris_eigen(fl)
        rc, resp, nc, ci, cr = orc.fast(img, K, with_candidates=True)
        order = np.argsort(ci, kind="stable")  # scan order (row-major index)
        ci, cr = ci[order], cr[order]
        canon = rc[:, 0] * W + rc[:, 1]
        std = orc.std_sort_cut(ci, cr, W, K)
        # ties at the cut: candidates whose response equals the K-th one, inside and outside the cut
        if nc > K:
            kth = np.sort(cr)[::-1][K - 1]
            inside = int(np.sum(resp == kth))
            total = int(np.sum(cr == kth))
            straddle = total > inside
        else:
            inside = total = 0
            straddle = False
        per[fl] = dict(ci=ci, cr=cr, canon=canon, std=std)
        res[f"flavour{fl}"] = {
            "candidates": int(nc),
            "std_sort_vs_canonical": {
                "cut_set_differs": bool(set(std.tolist()) != set(canon.tolist())),
                "cut_positions_differ": int(np.sum(std != canon)),
                "tie_group_at_cut": total,
                "tie_group_inside_cut": inside,
                "tie_straddles_cut": bool(straddle),
            },
        }
    orc.set_harris_eigen(0)
    a, b = per[0], per[1]
    assert np.array_equal(a["ci"], b["ci"])  # the candidate set never depends on the flavour
    ra, rb = a["canon"], b["canon"]
    res["flavours"] = {
        "responses_bits_differ": int(np.sum(a["cr"].view(np.uint32) != b["cr"].view(np.uint32))),
        "max_rel_response_diff": float(np.max(np.abs(a["cr"].astype(np.float64) - b["cr"]) /
                                              np.maximum(np.abs(a["cr"].astype(np.float64)), 1e-30)))
        if len(a["cr"]) else 0.0,
        "cut_set_differs": bool(set(ra.tolist()) != set(rb.tolist())),
        "cut_set_symmetric_difference": int(len(set(ra.tolist()) ^ set(rb.tolist()))),
        "cut_positions_differ": int(np.sum(ra != rb)) if len(ra) == len(rb) else None,
        "first_differing_position": int(np.argmax(ra != rb)) if len(ra) == len(rb) and np.any(ra != rb) else None,
    }
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02", "eigen_flavour.json"))
    args = ap.parse_args()
    import oracle_bind
    orc = oracle_bind.Oracle()
    report = {"what": __doc__.split("\n\n")[0].strip(), "K": K, "images": {}}
    for name, img in images().items():
        report["images"][name] = r = analyse(orc, img)
        f = r["flavours"]
        print(f"{name:28s} cand {r['flavour0']['candidates']:6d}  resp bits differ {f['responses_bits_differ']:6d}  "
              f"cut set differs {f['cut_set_differs']!s:5s} (sym diff {f['cut_set_symmetric_difference']})  "
              f"positions differ {f['cut_positions_differ']}  std::sort vs canonical: "
              f"{r['flavour0']['std_sort_vs_canonical']['cut_positions_differ']} / "
              f"{r['flavour1']['std_sort_vs_canonical']['cut_positions_differ']} positions, straddle "
              f"{r['flavour0']['std_sort_vs_canonical']['tie_straddles_cut']} / "
              f"{r['flavour1']['std_sort_vs_canonical']['tie_straddles_cut']}")
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(report, fh, indent=1)


if __name__ == "__main__":
    main()
