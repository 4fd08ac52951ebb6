"""One rank of the frame-sharded sequence front end (tests/test_gpu_sequence_shard.py starts it as a child process):
ya_vo_amd.sequence.SequenceShard over its shard of one synthetic stereo sequence (shard_range: N frames per rank,
overlapping by one frame), a gloo process group (several ranks share the test box's one GPU; the bench uses RCCL),
then the shard's local trajectory, BA log and the placed blocks go to an .npz for the parent to compare with the CPU
oracle loop over the same frames.

    python tests/sequence_shard_worker.py RANK WORLD PORT N CHUNK SEED OUT.npz [BACKEND]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, n, chunk, seed = (int(x) for x in sys.argv[1:7])
    out = sys.argv[7]
    backend = sys.argv[8] if len(sys.argv) > 8 else "gloo"
    import numpy as np
    import torch
    import torch.distributed as dist
    import ya_vo_amd as yv
    from ya_vo_amd import scene
    from ya_vo_amd.sequence import SequenceShard, shard_range
    from ya_vo_amd.synth import synth_sequence

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    import datetime
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120),
                            **({"device_id": torch.device("cuda", dev)} if backend == "nccl" else {}))
    ctx = yv.Context(dev)
    ctx.set_brief_offsets(np.fromfile(os.path.join(ROOT, "tests", "golden", "brief_offsets_mt19937_42.bin"),
                                      np.int8))
    first, end = shard_range(rank, world, n)
    fr = synth_sequence(seed, n, stereo=True, start=first)
    d = torch.from_numpy(fr.reshape(2 * n, *fr.shape[2:])).to(f"cuda:{dev}")
    T_right = np.array([0, 0, 0, 1, 0, -0.54, 0], np.float64)
    sh = SequenceShard(ctx, rank, world, n, chunk, scene.K_KITTI, T_right)
    for c in range(n // chunk):
        sh.process_chunk(d[2 * c * chunk:2 * (c + 1) * chunk])
    sh.finish()
    np.savez(out, local=sh.local_trajectory(), placed=sh.placed_blocks(), trajectory=sh.trajectory(),
             ba_log=np.array(sh.fe.ba_log, np.float64).reshape(-1, 4))
    dist.barrier()
    sh.close()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
