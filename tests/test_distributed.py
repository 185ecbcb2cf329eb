"""Multi-process (gloo, CPU) tests of the N>1 path: 16x16 tiles dealt
round-robin to ranks (tile t -> rank t % world, slot t // world), each rank's
packed tiles exchanged by the ONE gather bench.py uses (rt.gather_tiles), and
rank 0's unpack.  The per-rank tiles are cut from an oracle image here (the
device render of a tile set is covered by test_gpu_parity's
test_tile_partition_matches_single); the test pins the layout contract the
HIP unpack kernel and the gather share."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def pack_rank(img, rank, world, rt):
    H, W, _ = img.shape
    tx, ty, n, per = rt.tile_layout(W, H, world)
    out = np.zeros((per, 256, 3))
    for slot in range(per):
        t = rank + slot * world
        if t >= n:
            continue
        x0, y0 = (t % tx) * 16, (t // tx) * 16
        blk = np.zeros((16, 16, 3))
        part = img[y0:y0 + 16, x0:x0 + 16]
        blk[:part.shape[0], :part.shape[1]] = part
        out[slot] = blk.reshape(256, 3)
    return out


def unpack(gathered, H, W, world, rt):
    """numpy statement of rt::unpack_kernel (render.hip)."""
    tx, ty, n, per = rt.tile_layout(W, H, world)
    img = np.zeros((H, W, 3))
    for y in range(H):
        for x in range(W):
            t = (y // 16) * tx + x // 16
            img[y, x] = gathered[t % world, t // world, (y % 16) * 16 + (x % 16)]
    return img


def _worker(rank, world, port, img, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from conftest import load_package
    rt = load_package()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H, W, _ = img.shape
        tiles = torch.from_numpy(pack_rank(img, rank, world, rt))
        per = tiles.shape[0]
        gathered = torch.zeros((world, per, 256, 3), dtype=torch.float64) if rank == 0 else None
        out = rt.gather_tiles(tiles, gathered, rank, world)
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks timing reduction
        if rank == 0:
            q.put((unpack(out.numpy(), H, W, world, rt), float(t.item())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape", [(2, (40, 70)), (3, (33, 50))])
def test_tile_gather_roundtrip(world, shape):
    img = np.random.default_rng(world).random(shape + (3,))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, img, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, tmax = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert np.array_equal(res, img)
    assert tmax == world


def test_tile_layout_covers_every_pixel_once(rt):
    for W, H, world in [(1920, 1080, 8), (3840, 2160, 8), (70, 45, 3), (16, 16, 5)]:
        tx, ty, n, per = rt.tile_layout(W, H, world)
        owners = np.arange(n) % world
        assert per * world >= n and all((owners == r).sum() <= per for r in range(world))
        assert tx * 16 >= W and ty * 16 >= H
