"""Multi-GPU frame assembly: one process per GPU, 32x32 tiles dealt as a lattice
(rrt_partition_tiles: tile (tx, ty) to rank (tx + S ty) % world), one gather to rank 0.

Every rank renders the tiles rrt_partition_tiles gives it into one packed buffer (int32 words:
[n_max * T^2 * 3] f32 RGB, then [n_max * T^2] i32 sample counts; tile t's pixel (i, j) at
t * T^2 + j * T + i -- the layout rrt_render_tiles_device writes).  Rank 0 gathers the buffers
(torch.distributed: RCCL over xGMI for CUDA tensors, gloo for CPU tensors) and unpacks each
rank's tiles into the frame (rrt_unpack_tiles_device on the GPU, unpack_host() on the host).
The keyed RNG makes every pixel independent of which rank rendered it, so the assembled frame
equals a single-GPU render bit for bit."""
import numpy as np

import rrt

TILE = 32


class FramePlan:
    """Tile lists of every rank and the packed-buffer layout for a W x H frame over `world` ranks."""

    def __init__(self, frame_w, frame_h, world, tile=TILE):
        self.w, self.h, self.world, self.tile = frame_w, frame_h, world, tile
        self.rank_tiles = [rrt.partition_tiles(frame_w, frame_h, tile, q, world) for q in range(world)]
        self.n_max = max(len(t) for t in self.rank_tiles)
        self.tpix = tile * tile
        self.words = self.n_max * self.tpix * 4          # packed buffer size in 32-bit words
        self.count_offset = self.n_max * self.tpix * 3   # first count word

    def tiles(self, rank):
        return self.rank_tiles[rank]


def gather(dist, packed, rank, world):
    """Gather every rank's packed buffer (a torch int32 tensor) to rank 0; rank 0 gets the list,
    the others None.  The frame's only exchange step."""
    if world == 1:
        return [packed]
    import torch
    bufs = [torch.zeros_like(packed) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, bufs, dst=0)
    return bufs


def unpack_host(plan, bufs):
    """Host unpack of gathered packed buffers (numpy int32 arrays) into (rgb [H, W, 3] f32,
    count [H, W] i32) -- the rrt_unpack_kernel mapping."""
    rgb = np.zeros((plan.h, plan.w, 3), np.float32)
    cnt = np.zeros((plan.h, plan.w), np.int32)
    T = plan.tile
    for q, buf in enumerate(bufs):
        prgb = buf[:plan.count_offset].view(np.float32).reshape(-1, T, T, 3)
        pcnt = buf[plan.count_offset:].reshape(-1, T, T)
        for t, (x, y) in enumerate(plan.tiles(q)):
            x, y = int(x), int(y)
            tw, th = min(T, plan.w - x), min(T, plan.h - y)
            rgb[y:y + th, x:x + tw] = prgb[t, :th, :tw]
            cnt[y:y + th, x:x + tw] = pcnt[t, :th, :tw]
    return rgb, cnt
