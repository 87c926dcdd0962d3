#!/usr/bin/env python3
"""A/B kernel variants on one device, interleaved rounds in one process (methodology rule 24).

Renders a golden workload with each variant, checks it against the reference's golden frame
(bit-exact), and reports the HIP-event kernel time per variant (median / min over rounds).
Usage: python3 tools/ab_kernels.py [--case cfg3_bunny_1080p_s64] [--rounds 3] VARIANT...
VARIANT = name:flags:variant, e.g. lean2:0:2  mega2:4:2  lean2x:8:2 (flags: rrt.h RRT_RENDER_*)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402  (first: one shared HIP runtime)
import rrt  # noqa: E402
from golden_cases import Case  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg3_bunny_1080p_s64")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--grids", type=int, nargs="*", default=[0],
                    help="empty-space grid resolutions to A/B (0 = library default)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    c = Case(a.case)
    g = c.cfg
    rs = {}
    for gr in a.grids:
        r = rrt.Renderer(0, free_grid_res=gr)
        r.set_scene(rrt.SceneFile(c.scene_path))
        r.set_camera(rrt.load_camera(c.camera_path))
        r.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
        rs[gr] = r
    keys = [(v, gr) for gr in a.grids for v in a.variants]
    W, H, ts = c.frame_w, c.frame_h, 32
    tiles = rrt.partition_tiles(W, H, ts, 0, 1)
    n = len(tiles) * ts * ts
    prgb = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
    pcnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    frgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    fcnt = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    times = {k: [] for k in keys}
    exact = {}
    for rnd in range(a.rounds):
        for k in keys:
            v, gr = k
            r = rs[gr]
            name, flags, var = v.split(":")
            p = rrt.render_params(W, H, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                                  ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                                  max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"],
                                  flags=int(flags), variant=int(var))
            r.render_tiles_device(p, tiles, ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
            ms = r.stats().last_kernel_ms
            times[k].append(ms)
            if rnd == 0:
                r.unpack_tiles_device(tiles, ts, W, H, prgb.data_ptr(), pcnt.data_ptr(), frgb.data_ptr(),
                                      fcnt.data_ptr(), stream=s)
                torch.cuda.synchronize()
                got = frgb.cpu().numpy().reshape(H, W, 3)
                exact[k] = bool(np.array_equal(got.view(np.uint32), c.px["rgb"].view(np.uint32)) and
                                np.array_equal(fcnt.cpu().numpy().reshape(H, W), c.px["count"]))
    samples = int(c.px["count"].astype(np.int64).sum())
    out = {(v if len(a.grids) == 1 else f"{v}@grid{gr}"):
           {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)), "exact": exact[(v, gr)],
            "msamples_per_s": samples / (np.median(t) * 1e-3) / 1e6} for (v, gr), t in times.items()}
    print(json.dumps({"case": a.case, "results": out}, indent=1))


if __name__ == "__main__":
    main()
