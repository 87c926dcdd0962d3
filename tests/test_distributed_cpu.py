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
    assert plan.n_max == len(plan.tiles(0)) and sum(len(plan.tiles(q)) for q in range(8)) == 60 * 34
    assert plan.words == plan.n_max * 1024 * 4
