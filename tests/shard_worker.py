"""One rank of a frame-sharded run of the device front end (tests/test_gpu_shard.py starts it as a child process):
FrameShard (ya_vo_amd/sharding.py) over frames [1 + rank*B, 1 + (rank+1)*B) of one synthetic sequence with the
halo frame rank*B, a gloo process group (the GPU runs use RCCL; gloo lets several ranks share the one GPU of a test
box), two steps (the map exchange runs one step behind), then the rank's relative poses, edge counts and the placed
shared map go to an .npz for the parent to compare with a 1-rank run of the same frames.

    python tests/shard_worker.py RANK WORLD PORT B KF_EVERY SEED OUT.npz [BACKEND]

BACKEND is gloo (default) or nccl: RCCL needs one GPU per rank, so on the 1-GPU test box it runs at WORLD 1, where the
exchange still goes through all_gather_into_tensor on the communication stream.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, B, kf_every, seed = (int(x) for x in sys.argv[1:7])
    out = sys.argv[7]
    backend = sys.argv[8] if len(sys.argv) > 8 else "gloo"
    import numpy as np
    import torch
    import torch.distributed as dist
    import ya_vo_amd as yv
    from ya_vo_amd import map as ymap
    from ya_vo_amd import scene
    from ya_vo_amd.sharding import FrameShard, shard_images
    from ya_vo_amd.synth import synth_stereo_batch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world,
                            **({"device_id": torch.device("cuda", dev)} if backend == "nccl" else {}))
    ctx = yv.Context(dev)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"),
                                      np.int8))
    first = 1 + rank * B
    fr = synth_stereo_batch(seed, B + 1, start=first - 1)
    d = torch.from_numpy(shard_images(fr[2:], fr[0])).to(f"cuda:{dev}")
    max_kf = max(ymap.max_keyframes(B, 1 + r * B, kf_every) for r in range(world))
    T_right = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
    shard = FrameShard(ctx, B, first, scene.K_KITTI, T_right, halo=True, world=world, rank=rank, backend=backend,
                       kf_every=kf_every, max_kf=max_kf)
    for _ in range(2):
        shard.step(d.data_ptr())
    shard.drain()
    v = shard.batch.view()
    np.savez(out, poses=shard.poses(), placed=shard.placed_map(),
             edge_count=ctx.download(v.edge_count, np.int32, shard.n_tracks),
             inliers=ctx.download(v.track_inliers, np.int32, shard.n_tracks))
    dist.barrier()
    shard.close()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
