"""Frame upload (yv_seq_upload): PNG frames decoded on host threads into pinned staging, copied to HBM on the
caller's stream; the device bytes equal the host decode (and the source frames)."""
import numpy as np
import pytest

import ya_vo_amd as yv
from ya_vo_amd import io as yio
from test_io import _make_sequence

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stereo", [False, True])
def test_seq_upload_matches_source(ctx, tmp_path, stereo):
    import torch
    frames = _make_sequence(str(tmp_path), 9, stereo, H=37, W=53)
    seq = yio.Sequence(str(tmp_path), stereo=stereo)
    per = 2 if stereo else 1
    pitch = 37 * 53 + 11
    dev = torch.zeros((4 * per, pitch), dtype=torch.uint8, device="cuda:0")
    dev2 = torch.zeros_like(dev)
    s = torch.cuda.Stream()
    seq.upload(ctx, 1, 4, dev.data_ptr(), pitch, threads=3, stream=s.cuda_stream)
    seq.upload(ctx, 5, 4, dev2.data_ptr(), pitch, threads=3, stream=s.cuda_stream)  # the other staging slot
    s.synchronize()
    got = dev.cpu().numpy()[:, :37 * 53].reshape(-1, 37, 53)
    got2 = dev2.cpu().numpy()[:, :37 * 53].reshape(-1, 37, 53)
    np.testing.assert_array_equal(got, frames[1:5, :per].reshape(-1, 37, 53))
    np.testing.assert_array_equal(got2, frames[5:9, :per].reshape(-1, 37, 53))
    seq.upload(ctx, 0, 4, dev.data_ptr(), pitch, stream=s.cuda_stream)  # slot 0 again: waits for its copy
    s.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy()[:, :37 * 53].reshape(-1, 37, 53), frames[0:4, :per].reshape(-1, 37, 53))
    seq.close()
