"""CPU tests of the multi-GPU host logic: frame sharding with a 1-frame halo and the frame-ordered
all-gather of per-frame records, run as a world_size-2 gloo job (the GPU run uses RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ya_vo_amd.sharding import gather_frame_records, shard_frames


@pytest.mark.parametrize("n,world", [(4541, 8), (200, 3), (7, 8), (1, 2), (64, 1)])
def test_shards_cover_sequence(n, world):
    shards = [shard_frames(n, world, r) for r in range(world)]
    frames = [k for s in shards for k in s.frames]
    assert frames == list(range(n))
    sizes = [len(s.frames) for s in shards]
    assert max(sizes) - min(sizes) <= 1
    pairs = [p for s in shards for p in s.pairs()]
    assert pairs == [(k - 1, k) for k in range(1, n)]  # every temporal pair evaluated exactly once
    for s in shards:
        if len(s.frames) and s.start > 0:
            assert s.halo == s.start - 1 and s.computed.start == s.start - 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = shard_frames(n_frames, world, rank)
    # record of frame k: 12 doubles (T_cw 3x4) filled with k + j/100
    local = torch.tensor([[k + j / 100.0 for j in range(12)] for k in s.frames], dtype=torch.float64)
    full = gather_frame_records(local.reshape(-1, 12), n_frames, world, rank)
    q.put((rank, full.numpy().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [9, 2])
def test_gather_frame_records_gloo_world2(n_frames):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [[k + j / 100.0 for j in range(12)] for k in range(n_frames)]
    assert results[0] == expect and results[1] == expect
