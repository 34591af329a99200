"""Multi-GPU path on the CPU: world_size 2 over gloo.  Each rank renders its
tile shard (logical tile k -> rank k % world, dealt diagonally; the render_tiles layout) with the CPU
oracle, the shards are gathered to rank 0 with torch.distributed, and the
frame is rebuilt with the host mirror of pt_unshard_device.  The result must
equal the single-process render bit for bit (per-(pixel, sample) RNG keys
make any partition exact)."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent
W, H, SPP, DEPTH, SEED = 40, 27, 2, 8, 5


def _worker(rank, world, port, q):
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import oracle
    from conftest import load_package
    pt = load_package()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    text = (ROOT / "scenes" / "cornell_box.json").read_text()
    sc = oracle.Scene(text, seed=1)
    per = pt.shard_tiles(W, H, 0, world)
    idx = pt.shard_pixels(W, H, rank, world)
    assert len(idx) == pt.shard_tiles(W, H, rank, world) * 256
    shard = np.zeros((per * 256, 3))
    ok = idx >= 0
    shard[: len(idx)][ok] = sc.render(W, H, SPP, DEPTH, SEED, pixels=idx[ok].astype(np.uint32), threads=2)
    t = torch.from_numpy(shard)
    glist = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, glist, dst=0)
    if rank == 0:
        g = torch.stack(glist).numpy()
        q.put(pt.unshard_host(g, W, H, world))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_render_equals_full_frame(world):
    import socket
    import oracle
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    text = (ROOT / "scenes" / "cornell_box.json").read_text()
    ref = oracle.Scene(text, seed=1).render(W, H, SPP, DEPTH, SEED)
    assert np.array_equal(frame, ref)


def test_shard_pixels_partition(pt):
    for w, h, world in [(1920, 1080, 8), (37, 21, 3), (16, 16, 2)]:
        seen = np.concatenate([pt.shard_pixels(w, h, r, world) for r in range(world)])
        seen = np.sort(seen[seen >= 0])
        assert np.array_equal(seen, np.arange(w * h))
