"""Regenerates the committed golden fixtures under tests/golden/ (run in the build container).

Inputs
  * crops of the reference's KITTI-shaped test images (/root/reference/tests/epilines*.png, 1241x376 grey;
    KITTI is CC BY-NC-SA so only small crops are committed) -> kitti_crops.npz
  * synthetic frames from ya_vo_amd.synth (regenerated on the fly, nothing stored)
Outputs (all from the CPU oracle, oracle/build/liboracle.so)
  * fast_golden.npz   FastDetector::getFastFeatures: ncand, rc, resp per case
  * brief_golden.npz  Brief::computeBrief KeyPoint records per case (offsets = brief_offsets_mt19937_42.bin)
  * match_golden.npz  matchFeatures + removeOutliers(20) for synthetic frame 0 -> 1

Usage: python tests/golden/gen/make_golden.py [--crops]   (--crops re-extracts from /root/reference)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.dirname(HERE)
ROOT = os.path.dirname(os.path.dirname(GOLDEN))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from ya_vo_amd.synth import synth_frame  # noqa: E402
import oracle_bind  # noqa: E402

CROP_BOX = (128, 248, 400, 760)  # rows 128..247, cols 400..759


def extract_crops():
    from PIL import Image
    out = {}
    for name in ("epilines", "epilinesOpencv"):
        img = np.array(Image.open(f"/root/reference/tests/{name}.png"))
        r0, r1, c0, c1 = CROP_BOX
        out[name] = img[r0:r1, c0:c1].copy()
    np.savez_compressed(os.path.join(GOLDEN, "kitti_crops.npz"), **out)


def cases():
    crops = np.load(os.path.join(GOLDEN, "kitti_crops.npz"))
    yield "crop_epilines", crops["epilines"]
    yield "crop_epilinesOpencv", crops["epilinesOpencv"]
    yield "synth_1234_f0", synth_frame(1234, 0, 0)
    yield "synth_1234_f1", synth_frame(1234, 1, 3)


def main():
    if "--crops" in sys.argv or not os.path.exists(os.path.join(GOLDEN, "kitti_crops.npz")):
        extract_crops()
    orc = oracle_bind.Oracle()
    offsets = np.fromfile(os.path.join(GOLDEN, "brief_offsets_mt19937_42.bin"), np.int8).reshape(256, 4)
    fast, brief = {}, {}
    kps = {}
    for name, img in cases():
        rc, resp, nc = orc.fast(img, 2000)
        fast[name + "__rc"] = rc
        fast[name + "__resp"] = resp
        fast[name + "__ncand"] = np.array([nc])
        k = orc.brief(img, rc, offsets)
        brief[name] = k
        kps[name] = k
        print(f"{name}: {img.shape} candidates={nc} kept={len(rc)} described={len(k)}")
    np.savez_compressed(os.path.join(GOLDEN, "fast_golden.npz"), **fast)
    np.savez_compressed(os.path.join(GOLDEN, "brief_golden.npz"), **brief)
    m = orc.match(kps["synth_1234_f0"], kps["synth_1234_f1"])
    f = orc.remove_outliers(m, 20)
    np.savez_compressed(os.path.join(GOLDEN, "match_golden.npz"), matches=m, filtered=f)
    print(f"matches={len(m)} filtered={len(f)} min_dist={m['distance'].min()}")


if __name__ == "__main__":
    main()
