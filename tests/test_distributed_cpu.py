"""Multi-GPU path on the CPU (gloo, world size 2): each rank renders its block-cyclic tiles with
the CPU restatement into the packed per-rank layout, rank 0 gathers and unpacks them with the
same plan the GPU bench uses (rrt_frame.py), and the assembled frame must equal the reference's
golden frame bit for bit (the keyed RNG makes pixels independent of the rank that renders them)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import rrt_frame
from golden_cases import Case

CASE = "spheres_96x72_s8_l4"  # reference golden frame with lit pixels (2.8% non-black)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path, kerr=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = Case(CASE)
    g = c.cfg
    plan = rrt_frame.FramePlan(c.frame_w, c.frame_h, world, tile=32)
    s = O.Scene(c.scene_path)
    cam = O.load_camera(c.camera_path)
    p = O.make_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                      ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                      max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], bh=g["bh"],
                      kerr=kerr)
    packed = np.zeros(plan.words, np.int32)
    prgb = packed[:plan.count_offset].view(np.float32).reshape(-1, 32, 32, 3)
    pcnt = packed[plan.count_offset:].reshape(-1, 32, 32)
    for t, (x, y) in enumerate(plan.tiles(rank)):
        x, y = int(x), int(y)
        tw, th = min(32, c.frame_w - x), min(32, c.frame_h - y)
        rgb, cnt, _, _ = O.render(s, cam, p, x, y, tw, th, threads=2)
        prgb[t, :th, :tw] = rgb
        pcnt[t, :th, :tw] = cnt
    bufs = rrt_frame.gather(dist, torch.from_numpy(packed), rank, world)
    if rank == 0:
        rgb, cnt = rrt_frame.unpack_host(plan, [b.numpy() for b in bufs])
        np.savez(out_path, rgb=rgb, cnt=cnt)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_reference_frame(tmp_path, world):
    out = str(tmp_path / "frame.npz")
    mp.spawn(_rank_main, args=(world, _free_port(), out), nprocs=world, join=True)
    c = Case(CASE)
    d = np.load(out)
    assert np.array_equal(d["rgb"].view(np.uint32), c.px["rgb"].view(np.uint32))
    assert np.array_equal(d["cnt"], c.px["count"])
    assert c.px["rgb"].max() > 0


def test_gather_kerr_frame_is_partition_independent(tmp_path):
    """The Kerr spacetime on 2 ranks: the assembled frame equals one
    single-process render of the whole frame (parity against the reference: unpinned)."""
    out = str(tmp_path / "frame.npz")
    kerr = (0.9, (0.0, 1.0, 0.0))
    mp.spawn(_rank_main, args=(2, _free_port(), out, kerr), nprocs=2, join=True)
    c = Case(CASE)
    g = c.cfg
    p = O.make_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                      ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                      max_tolerance=g["max_tolerance"], bh=g["bh"], kerr=kerr)
    rgb, cnt, _, _ = O.render(O.Scene(c.scene_path), O.load_camera(c.camera_path), p, 0, 0, c.frame_w, c.frame_h)
    d = np.load(out)
    assert np.array_equal(d["rgb"].view(np.uint32), rgb.view(np.uint32))
    assert np.array_equal(d["cnt"], cnt)
    assert not np.array_equal(rgb, c.px["rgb"])


def test_plan_layout():
    plan = rrt_frame.FramePlan(1920, 1080, 8)
    assert plan.n_max == max(len(plan.tiles(q)) for q in range(8)) and sum(len(plan.tiles(q)) for q in range(8)) == 60 * 34
    assert plan.n_max <= 60 * 34 // 8 + 1  # the lattice deal's shares differ by at most one tile here
    assert plan.words == plan.n_max * 1024 * 4


@pytest.mark.parametrize("world", [2, 3, 4, 5, 6, 7, 8])
def test_tile_deal_matches_frame_plan(world):
    """The library's block-cyclic deal (rrt_partition_tiles for bench.py's ranks, rrt_region_tiles
    for rrt_group_render's members) against rrt_frame.FramePlan, on the BASELINE frame sizes and a
    ragged region: every tile of the frame or region exactly once, tile (tx, ty) to rank
    (tx + S ty) % world with S = 1, 1, 1, 2, 1, 3, 3 for world 2..8 (the integer nearest 0.382 world
    prime to it), row by row; no rank owns a whole column; a rank may get no tile; the packed
    layout's capacity holds the largest share; unpacking a synthetic packed frame through the plan
    restores every pixel."""
    import rrt

    S = {2: 1, 3: 1, 4: 1, 5: 2, 6: 1, 7: 3, 8: 3}[world]
    for W, H in [(480, 360), (1920, 1080), (3840, 2160), (100, 40)]:
        plan = rrt_frame.FramePlan(W, H, world)
        tw, th = (W + 31) // 32, (H + 31) // 32
        order = [(tx * 32, ty * 32) for ty in range(th) for tx in range(tw)]
        for q in range(world):
            want = np.array([(x, y) for x, y in order if (x // 32 + S * (y // 32)) % world == q],
                            np.uint32).reshape(-1, 2)
            if th > 1 and tw >= world:  # every column's tiles spread over the ranks
                assert len({int(y) for x, y in want.tolist() if x == 0}) < th
            assert np.array_equal(plan.tiles(q), want)
            assert np.array_equal(rrt.region_tiles(0, 0, W, H, 32, q, world), want)
        assert plan.n_max == max(len(plan.tiles(q)) for q in range(world))
        assert sorted(map(tuple, np.concatenate([plan.tiles(q) for q in range(world)]).tolist())) == sorted(order)
    # bench.py's cfg5 split: 16-px tiles of the 4K frame, the same rule
    W, H, T = 3840, 2160, 16
    plan = rrt_frame.FramePlan(W, H, world, T)
    got = np.concatenate([plan.tiles(q) for q in range(world)])
    assert len(got) == (W // T) * (H // T) == len({tuple(t) for t in got.tolist()})
    for q in range(world):
        assert all((x // T + S * (y // T)) % world == q for x, y in plan.tiles(q).tolist())
    # a region (rrt_group_render): tiles from the region's origin, the same deal
    x0, y0, w, h = 70, 13, 200, 65
    rt = [rrt.region_tiles(x0, y0, w, h, 32, q, world) for q in range(world)]
    full = [tuple(t) for q in range(world) for t in rt[q].tolist()]
    assert len(full) == len(set(full)) == ((w + 31) // 32) * ((h + 31) // 32)
    assert all(x0 <= x < x0 + w and y0 <= y < y0 + h and (x - x0) % 32 == 0 and (y - y0) % 32 == 0 for x, y in full)
    if world > len(full):
        assert any(len(t) == 0 for t in rt)
    # packed layout round trip (rrt_frame.unpack_host, the rrt_unpack_kernel mapping)
    W, H = 100, 40
    plan = rrt_frame.FramePlan(W, H, world)
    rng = np.random.default_rng(world)
    frame = rng.random((H, W, 3), dtype=np.float32)
    cnt = rng.integers(1, 1 << 20, (H, W), dtype=np.int32)
    bufs = []
    for q in range(world):
        b = np.full(plan.words, -1, np.int32)
        prgb = b[:plan.count_offset].view(np.float32).reshape(-1, 32, 32, 3)
        pcnt = b[plan.count_offset:].reshape(-1, 32, 32)
        for t, (x, y) in enumerate(plan.tiles(q)):
            x, y = int(x), int(y)
            tw, th = min(32, W - x), min(32, H - y)
            prgb[t, :th, :tw] = frame[y:y + th, x:x + tw]
            pcnt[t, :th, :tw] = cnt[y:y + th, x:x + tw]
        bufs.append(b)
    rgb2, cnt2 = rrt_frame.unpack_host(plan, bufs)
    assert np.array_equal(rgb2.view(np.uint32), frame.view(np.uint32)) and np.array_equal(cnt2, cnt)
