"""Row-tile partition of a frame over ranks and the tile gather (RCCL over xGMI on MI355X; any
torch.distributed backend works, gloo in the CPU tests).

Rows are dealt in blocks of `row_block` (default 4, the block crt_render and bench.py use): row r
belongs to rank (r // row_block) % world. Interleaving balances the >10x per-row cost variance of real scenes (the sky rows of
RTOW cost almost nothing). Every rank renders only its rows (crt_render_async with
crt_tiling{row_block, world, rank}); the frame is then assembled from equal-size padded tiles with
one all-gather. Because the RNG is per (pixel, sample) and the sample-chunk grouping depends only on
spp, the assembled frame is bit-identical for any number of ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def owned_rows(height: int, row_block: int, world: int, rank: int) -> list[int]:
    """The rows rank `rank` renders (crt_tiling semantics of include/crt_render.h)."""
    return [r for r in range(height) if (r // row_block) % world == rank]


class TileGather:
    """Gathers every rank's rows of a (h, w, 3) frame into a full frame on every rank."""

    def __init__(self, height: int, width: int, world: int, rank: int, device, row_block: int = 4,
                 dtype=torch.float64, group=None):
        self.h, self.w, self.world, self.rank, self.group = height, width, world, rank, group
        rows = [owned_rows(height, row_block, world, k) for k in range(world)]
        self.max_rows = max(len(r) for r in rows)
        self.mine = torch.tensor(rows[rank], dtype=torch.long, device=device)
        self.n_mine = len(rows[rank])
        # where each gathered tile row lands in the frame (padding rows are dropped)
        dst, src = [], []
        for k, rk in enumerate(rows):
            for i, r in enumerate(rk):
                dst.append(r)
                src.append(k * self.max_rows + i)
        self.dst = torch.tensor(dst, dtype=torch.long, device=device)
        self.src = torch.tensor(src, dtype=torch.long, device=device)
        self.tile = torch.zeros(self.max_rows, width, 3, dtype=dtype, device=device)
        self.full = torch.zeros(world * self.max_rows, width, 3, dtype=dtype, device=device)

    def gather(self, frame: torch.Tensor) -> torch.Tensor:
        """frame: this rank's (h, w, 3) buffer with its own rows rendered. Returns the assembled
        frame (a new tensor on every rank)."""
        if self.world == 1:
            return frame
        self.tile[: self.n_mine].copy_(frame.index_select(0, self.mine))
        return self.gather_packed(self.tile)

    def new_tile(self) -> torch.Tensor:
        """A (max_rows, w, 3) tile buffer: a rank renders its rows into the first n_mine rows with
        crt_tiling{row_block, world, rank, CRT_TILING_PACKED} (its share of the frame only)."""
        return torch.zeros_like(self.tile)

    def gather_packed(self, tile: torch.Tensor) -> torch.Tensor:
        """tile: this rank's owned rows in order (new_tile / CRT_TILING_PACKED). Returns the
        assembled (h, w, 3) frame on every rank: one all-gather straight into the rank-major tile
        array (no per-rank parts + concat), then one row scatter."""
        if tile.is_cuda and dist.get_backend(self.group) == "gloo":
            # the one-GPU rehearsal of the N-rank path (ranks sharing a device, which RCCL
            # refuses): gloo gathers through host memory
            full = self.full.cpu()
            dist.all_gather_into_tensor(full, tile.cpu(), group=self.group)
            self.full.copy_(full)
        else:
            dist.all_gather_into_tensor(self.full, tile, group=self.group)
        out = torch.empty(self.h, self.w, 3, dtype=tile.dtype, device=tile.device)
        out.index_copy_(0, self.dst, self.full.index_select(0, self.src))
        return out


def frame_digest(frame: torch.Tensor) -> str:
    """sha256 of an assembled (h, w, 3) float64 frame's bytes, row-major (the Image layout,
    image.h), as its first 15 hex digits (60 bits: one int64 over the wire). Frames are
    bit-identical for any rank count, so this digest is too: an N-rank run must report the N=1
    digest of the same workload."""
    import hashlib
    return hashlib.sha256(frame.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:15]


def digests_agree(digest: str, device, group=None) -> tuple[bool, list[str]]:
    """All-gather every rank's frame digest (one int64 per rank, on `device`: the process group's
    device, cuda for RCCL); returns (all ranks equal, the digests in rank order)."""
    world = dist.get_world_size(group)
    mine = torch.tensor([int(digest, 16)], dtype=torch.int64, device=device)
    every = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(every, mine, group=group)
    got = [f"{int(v):015x}" for v in every.cpu().tolist()]
    return all(g == got[0] for g in got), got
