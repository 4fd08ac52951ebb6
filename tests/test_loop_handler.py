"""The C++ LoopHandler over the C ABI (ya_vo_amd/frontend/loop_handler.cpp, bin/yavo_loop_handler) against the
reference's LoopHandler behaviour (src/LoopHandler.cc) and the same loop over the CPU oracle (tests/loop_chain.py).

CPU: the reference's config plumbing (BASELINE configs[0]: config/KITTI_mock_test.json's keys basePath / sequence /
cameraType, `//` comments as jsoncpp accepts them) and its LoopHandlerTest cases (stereoStatus, getSeqNo,
getLeftImagesPath, getLeftTrainLength, getNextFrame dimensions, frame ids; tests/LoopHandlerTest.cc), plus the
oracle loop's state machine on a synthetic mono sequence.
GPU: the mono trajectory of the C++ LoopHandler is bit-identical to the oracle loop's, with the same per-frame
events (INIT, TRACKED, REINIT and their counts)."""
import json
import os
import subprocess

import numpy as np
import pytest

from ya_vo_amd.synth import synth_frame

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "ya_vo_amd", "bin", "yavo_loop_handler")
OFFSETS = os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin")
# KITTI sequence 00's calib.txt P0 / P1 (the reference's tests/calib.txt format)
CALIB = ("P0: 7.188560000000e+02 0.000000000000e+00 6.071928000000e+02 0.000000000000e+00 0.000000000000e+00 "
         "7.188560000000e+02 1.852157000000e+02 0.000000000000e+00 0.000000000000e+00 0.000000000000e+00 "
         "1.000000000000e+00 0.000000000000e+00\n"
         "P1: 7.188560000000e+02 0.000000000000e+00 6.071928000000e+02 -3.861448000000e+02 0.000000000000e+00 "
         "7.188560000000e+02 1.852157000000e+02 0.000000000000e+00 0.000000000000e+00 0.000000000000e+00 "
         "1.000000000000e+00 0.000000000000e+00\n")
K_SEQ00 = [718.856, 0.0, 607.1928, 0.0, 718.856, 185.2157, 0.0, 0.0, 1.0]


def offset(k, cut):
    """Frame k of the synthetic mono sequence: a crop of one noise field moving (1, 3) px per frame; from `cut` on
    the crop jumps to an unrelated region, so tracking fails there and the loop reinitialises."""
    return (k, 3 * k) if k < cut else (1000 + k, 500 + 3 * k)


def make_sequence(tmp_path, frames, seq="00", camera="mono", right=False, comment=True):
    from PIL import Image
    base = str(tmp_path / "dataset" / "sequences") + "/"
    for side in (("image_0", "image_1") if right else ("image_0",)):
        d = os.path.join(base, seq, side)
        os.makedirs(d, exist_ok=True)
        for k, img in enumerate(frames):
            Image.fromarray(img).save(os.path.join(d, f"{k:06d}.png"))
    with open(os.path.join(base, seq, "calib.txt"), "w") as f:
        f.write(CALIB)
    cfg = tmp_path / "KITTI_mock_test.json"
    cam = f'"cameraType" : "{camera}"' + (" //set to stereo if used" if comment else "")
    cfg.write_text('{\n    "basePath" : "%s", \n    "sequence" : "%s", \n    %s\n}\n' % (base, seq, cam))
    return str(cfg), base


def check_config(cfg):
    r = subprocess.run([BIN, cfg, "--check-config"], capture_output=True, text=True, timeout=60)
    return r.returncode, json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def small_frames():
    return [synth_frame(77, k, 3 * k, 120, 300) for k in range(4)]


def test_check_config_mono(tmp_path, small_frames):
    """LoopHandlerTest.cc: CopyConstructor / PathTrainTest / checkNextFrameDims / checkFrameIDs on a mono config."""
    cfg, base = make_sequence(tmp_path, small_frames)
    rc, out = check_config(cfg)
    assert rc == 0 and out["ok"]
    assert out["stereo"] is False
    assert out["sequence"] == "00"
    assert out["left_images_path"] == base + "00/image_0/"
    assert out["left_train_length"] == len(small_frames)
    np.testing.assert_allclose(out["K"], K_SEQ00, rtol=0, atol=1e-9)
    # getNextFrame: 1-based ids (Frame::createFrameID pre-increments, src/Frame.cc:43-47), the PNG's dimensions
    assert [f["id"] for f in out["frames"]] == [1, 2, 3]
    assert all((f["H"], f["W"]) == (120, 300) for f in out["frames"])


def test_check_config_stereo(tmp_path, small_frames):
    cfg, _ = make_sequence(tmp_path, small_frames, seq="07", camera="stereo", right=True, comment=False)
    rc, out = check_config(cfg)
    assert rc == 0 and out["stereo"] is True and out["sequence"] == "07"
    assert out["right_train_length"] == len(small_frames)


def test_check_config_errors(tmp_path, small_frames):
    # a stereo config without image_1, and an unreadable config: the constructor reports, nothing crashes
    cfg, _ = make_sequence(tmp_path, small_frames, camera="stereo", right=False)
    rc, out = check_config(cfg)
    assert rc == 1 and not out["ok"]
    bad = tmp_path / "bad.json"
    bad.write_text("{ \"basePath\" : ")
    rc, out = check_config(str(bad))
    assert rc == 1 and not out["ok"]


def test_oracle_loop_visits_every_state(oracle):
    """The oracle loop on the synthetic sequence reaches INIT, TRACKED and REINIT (so the GPU parity test below
    covers every branch of addFrame)."""
    from loop_chain import INIT_MAP, REINIT, TRACKED, LoopChain
    from ya_vo_amd import scene
    offsets = np.fromfile(OFFSETS, np.int8).reshape(256, 4)
    frames = [synth_frame(1234, *offset(k, 6), 376, 1241) for k in range(8)]
    P, ev = LoopChain(oracle, scene.K_KITTI, offsets).run(frames)
    kinds = [e["kind"] for e in ev]
    assert kinds[1] == INIT_MAP and TRACKED in kinds and REINIT in kinds
    assert np.all(np.isfinite(P))


@pytest.mark.gpu
def test_loop_handler_matches_oracle_loop(tmp_path, oracle):
    """BASELINE configs[0]-shaped run: the config file drives the C++ LoopHandler over a synthetic mono sequence on the
    GPU; its trajectory (T_cw per frame) equals the oracle loop's bit for bit, and so do the per-frame events."""
    from loop_chain import EVENT_FIELDS, LoopChain
    from ya_vo_amd import scene
    n = 10
    frames = [synth_frame(1234, *offset(k, 7), 376, 1241) for k in range(n)]
    cfg, _ = make_sequence(tmp_path, frames)
    pb, eb, pt = tmp_path / "poses.bin", tmp_path / "events.bin", tmp_path / "poses.txt"
    r = subprocess.run([BIN, cfg, "--poses-bin", str(pb), "--events", str(eb), "--poses", str(pt)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    gpu_poses = np.fromfile(pb, np.float64).reshape(-1, 7)
    gpu_events = np.fromfile(eb, np.int32).reshape(-1, len(EVENT_FIELDS))
    assert stats["frames"] == n and len(gpu_poses) == n

    offsets = np.fromfile(OFFSETS, np.int8).reshape(256, 4)
    P, ev = LoopChain(oracle, scene.K_KITTI, offsets).run(frames)
    ref_events = np.array([[e[f] for f in EVENT_FIELDS] for e in ev], np.int32)
    # getFRANSAC's F is unused by the reference (src/LoopHandler.cc:222, 562); its inlier count (the oracle loop
    # draws the same std::mt19937(0) samples) is compared with every other event field
    np.testing.assert_array_equal(gpu_events, ref_events)
    assert np.any(gpu_events[:, EVENT_FIELDS.index("f_inliers")] > 0)
    np.testing.assert_array_equal(gpu_poses, P)
    assert stats["init"] == 1 and stats["reinit"] >= 1 and stats["tracked"] >= 1
    # the KITTI-format trajectory (T_wc rows) is the same poses
    rows = np.loadtxt(pt).reshape(n, 3, 4)
    np.testing.assert_allclose(rows[:, :, 3], [oracle.se3_inverse(p)[4:] for p in P], rtol=0, atol=1e-6)


@pytest.mark.gpu
def test_loop_handler_pipelined_matches_oracle_loop(tmp_path, oracle):
    """The pipelined C++ LoopHandler (--pipeline 2: frame k + 1's read + detect + describe on a worker thread with its
    own GPU context while frame k is tracked; frame k + 1's LK on the side lane during frame k's pose LM) over 60
    synthetic mono frames with a reinitialisation at frame 40: the trajectory and per-frame events equal the oracle
    loop's bit for bit."""
    from loop_chain import EVENT_FIELDS, LoopChain
    from ya_vo_amd import scene
    n = 60
    frames = [synth_frame(4321, *offset(k, 40), 376, 1241) for k in range(n)]
    cfg, _ = make_sequence(tmp_path, frames)
    pb, eb = tmp_path / "poses.bin", tmp_path / "events.bin"
    r = subprocess.run([BIN, cfg, "--poses-bin", str(pb), "--events", str(eb), "--pipeline", "2"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    assert stats["frames"] == n and stats["pipeline"] == 2
    gpu_poses = np.fromfile(pb, np.float64).reshape(-1, 7)
    gpu_events = np.fromfile(eb, np.int32).reshape(-1, len(EVENT_FIELDS))
    offsets = np.fromfile(OFFSETS, np.int8).reshape(256, 4)
    P, ev = LoopChain(oracle, scene.K_KITTI, offsets).run(frames)
    ref_events = np.array([[e[f] for f in EVENT_FIELDS] for e in ev], np.int32)
    np.testing.assert_array_equal(gpu_events, ref_events)
    np.testing.assert_array_equal(gpu_poses, P)
    assert stats["init"] == 1 and stats["reinit"] >= 1 and stats["tracked"] >= 40
    assert stats["lk_ahead_frames"] >= 1  # the look-ahead LK's rows were used (and matched the oracle above)


@pytest.mark.gpu
def test_loop_handler_gpu_decode_matches_oracle_loop(tmp_path, oracle):
    """The pipelined C++ LoopHandler with the look-ahead decoded on the GPU (--gpu-decode 16: PNG inflate + unfilter,
    detect and describe of 16 frames per batch on the device, the next batch enqueued while this one is handed over)
    over 45 frames (three batches, the last one partial) with a reinitialisation: the trajectory and per-frame events
    equal the oracle loop's bit for bit."""
    from loop_chain import EVENT_FIELDS, LoopChain
    from ya_vo_amd import scene
    n = 45
    frames = [synth_frame(777, *offset(k, 30), 376, 1241) for k in range(n)]
    cfg, _ = make_sequence(tmp_path, frames)
    pb, eb = tmp_path / "poses.bin", tmp_path / "events.bin"
    r = subprocess.run([BIN, cfg, "--poses-bin", str(pb), "--events", str(eb), "--pipeline", "2", "--gpu-decode", "16",
                        "--readers", "4"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    assert stats["frames"] == n and stats["gpu_decode_batch"] == 16
    gpu_poses = np.fromfile(pb, np.float64).reshape(-1, 7)
    gpu_events = np.fromfile(eb, np.int32).reshape(-1, len(EVENT_FIELDS))
    offsets = np.fromfile(OFFSETS, np.int8).reshape(256, 4)
    P, ev = LoopChain(oracle, scene.K_KITTI, offsets).run(frames)
    ref_events = np.array([[e[f] for f in EVENT_FIELDS] for e in ev], np.int32)
    np.testing.assert_array_equal(gpu_events, ref_events)
    np.testing.assert_array_equal(gpu_poses, P)
    assert stats["reinit"] >= 1 and stats["tracked"] >= 20


@pytest.mark.gpu
def test_loop_handler_gpu_decode_truncated_png_ends_the_train(tmp_path, oracle):
    """A truncated PNG in the middle of a GPU-decoded batch (frame 20 of the 16-frame batch 16..31) fails alone, as
    cv::imread does per file: the frames before it are tracked, the loop ends cleanly (exit 0) at exactly that frame,
    and the trajectory is the oracle loop's over frames 0..19 -- the same end as the host-decoding pipeline."""
    from loop_chain import EVENT_FIELDS, LoopChain
    from ya_vo_amd import scene
    n, bad = 40, 20
    frames = [synth_frame(777, *offset(k, 30), 376, 1241) for k in range(n)]
    cfg, base = make_sequence(tmp_path, frames)
    path = os.path.join(base, "00", "image_0", f"{bad:06d}.png")
    data = open(path, "rb").read()
    with open(path, "wb") as f:
        f.write(data[:len(data) // 2])
    offsets = np.fromfile(OFFSETS, np.int8).reshape(256, 4)
    P, ev = LoopChain(oracle, scene.K_KITTI, offsets).run(frames[:bad])
    ref_events = np.array([[e[f] for f in EVENT_FIELDS] for e in ev], np.int32)
    for mode in (["--gpu-decode", "16"], []):
        pb, eb = tmp_path / "poses.bin", tmp_path / "events.bin"
        r = subprocess.run([BIN, cfg, "--poses-bin", str(pb), "--events", str(eb), "--pipeline", "2", "--readers", "4"]
                           + mode, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (mode, r.stderr[-2000:])
        stats = json.loads(r.stdout.strip().splitlines()[-1])
        assert stats["frames"] == bad, mode
        np.testing.assert_array_equal(np.fromfile(eb, np.int32).reshape(-1, len(EVENT_FIELDS)), ref_events)
        np.testing.assert_array_equal(np.fromfile(pb, np.float64).reshape(-1, 7), P)
