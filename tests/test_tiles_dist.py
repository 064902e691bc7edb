"""The multi-rank path of bench.py on CPU: world_size 2 and 3 over gloo. Each rank fills ONLY the
rows it owns (what crt_render_async does for its tiling); TileGather must assemble the full frame
on every rank. Also checks the row partition covers every row exactly once."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cpp_raytracer_amd.tiles import TileGather, digests_agree, frame_digest, owned_rows


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def reference_frame(h, w):
    r = torch.arange(h, dtype=torch.float64).view(h, 1, 1)
    c = torch.arange(w, dtype=torch.float64).view(1, w, 1)
    k = torch.arange(3, dtype=torch.float64).view(1, 1, 3)
    return r * 1000 + c + k / 10


def worker(rank, world, port, h, w, rb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        want = reference_frame(h, w)
        frame = torch.full((h, w, 3), float("nan"), dtype=torch.float64)
        mine = owned_rows(h, rb, world, rank)
        frame[mine] = want[mine]  # "render" only the owned rows
        g = TileGather(h, w, world, rank, "cpu", row_block=rb)
        out = g.gather(frame)
        # the packed route bench.py takes: the rank's rows only, in order (CRT_TILING_PACKED)
        tile = g.new_tile()
        tile[: len(mine)] = want[mine]
        out2 = g.gather_packed(tile)
        q.put((rank, bool(torch.equal(out, want)) and bool(torch.equal(out2, want))))
    finally:
        dist.destroy_process_group()


# row_block 4 is what bench.py and crt_render use (800 rows deal exactly over 1, 2, 4, 8 ranks);
# 16 and 3 cover other block sizes and short last blocks
@pytest.mark.parametrize("world,h,w,rb", [(2, 800, 12, 4), (3, 77, 5, 4), (2, 9, 4, 4), (4, 90, 3, 4),
                                          (2, 800, 12, 16), (3, 77, 5, 3)])
def test_tile_gather_assembles_frame(world, h, w, rb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, h, w, rb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res


@pytest.mark.parametrize("h,rb,world", [(800, 4, 8), (2160, 4, 8), (1080, 4, 8), (675, 4, 3), (5, 4, 4),
                                        (800, 16, 8), (5, 16, 4)])
def test_row_partition_covers_every_row_once(h, rb, world):
    rows = sorted(r for k in range(world) for r in owned_rows(h, rb, world, k))
    assert rows == list(range(h))


def digest_worker(rank, world, port, h, w, corrupt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        want = reference_frame(h, w)
        mine = owned_rows(h, 4, world, rank)
        g = TileGather(h, w, world, rank, "cpu", row_block=4)
        tile = g.new_tile()
        tile[: len(mine)] = want[mine]
        if corrupt == "tile" and rank == 1:  # a wrong tile: every rank assembles the same wrong frame
            tile[0, 0, 0] += 1
        out = g.gather_packed(tile)
        if corrupt == "frame" and rank == 1:  # one rank's frame differs after the gather
            out[h // 2, w // 2, 1] += 1
        d = frame_digest(out)
        agree, every = digests_agree(d, "cpu")
        q.put((rank, d, agree, every))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("corrupt", ["none", "tile", "frame"])
def test_frame_digest_self_check(world, corrupt):
    """bench.py's frame self-check (frame_check): at N = 2, 3 every rank's digest equals the N=1
    digest of the same frame and ranks_agree holds; a corrupted tile changes the digest on every
    rank (ranks agree, N=1 mismatch); a frame corrupted on one rank flips ranks_agree."""
    h, w = 98, 16
    n1 = frame_digest(reference_frame(h, w))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=digest_worker, args=(r, world, port, h, w, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    digests = [d for _, d, _, _ in res]
    assert all(every == digests for _, _, _, every in res)
    agree = {a for _, _, a, _ in res}
    assert len(agree) == 1
    if corrupt == "none":
        assert agree == {True} and digests == [n1] * world
    elif corrupt == "tile":
        assert agree == {True} and n1 not in digests
    else:
        assert agree == {False} and digests[1] != n1 and digests[0] == n1
