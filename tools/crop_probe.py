#!/usr/bin/env python3
"""Diagnostic: time one small region of a golden workload with several kernel paths and print its
per-pixel work counters (executed and reference).  Usage:
  python3 tools/crop_probe.py --case cfg3_bunny_1080p_s64 --region 960 600 20 15 [--flags 0 128 ...]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
import rrt  # noqa: E402
from golden_cases import Case  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg3_bunny_1080p_s64")
    ap.add_argument("--region", type=int, nargs=4, default=[960, 600, 20, 15])
    ap.add_argument("--flags", nargs="+", default=["0", str(rrt.RRT_RENDER_PER_PIXEL), str(rrt.RRT_RENDER_NO_MISS_PROOF)],
                    help="flags[:variant] per run (variant = waves/SIMD of the build)")
    ap.add_argument("--no-counters", action="store_true")
    a = ap.parse_args()
    c = Case(a.case)
    g = c.cfg
    x0, y0, w, h = a.region
    r = rrt.Renderer(0)
    r.set_scene(rrt.SceneFile(c.scene_path))
    r.set_envmap(c.envmap)
    r.set_camera(rrt.load_camera(c.camera_path))
    r.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
    out = {}

    def params(fl, var=0):
        return rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                                 ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                                 max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=fl,
                                 variant=var)
    for spec in a.flags:
        fl, _, var = spec.partition(":")
        ts = []
        for _ in range(3):
            t0 = time.time()
            rgb, cnt, _, _ = r.render(params(int(fl), int(var or 0)), x0, y0, w, h)
            ts.append((r.stats().last_kernel_ms, time.time() - t0))
        out[spec] = {"kernel_ms": [round(t[0], 3) for t in ts], "kernel": r.stats().kernel.decode()}
    for mode, fl in (() if a.no_counters else (("executed", rrt.RRT_RENDER_COUNT_EXECUTED), ("reference", 0))):
        rgb, cnt, draws, ctr = r.render(params(fl), x0, y0, w, h, counters=True)
        ms = r.stats().last_kernel_ms
        box = ctr[..., 0].astype(np.int64)
        i = np.unravel_index(np.argmax(box), box.shape)
        out[mode] = {"kernel_ms": ms, "aabb_max": int(box.max()), "at": [int(i[1]) + x0, int(i[0]) + y0],
                     "ctr_at_max": [int(v) for v in ctr[i]], "count_at_max": int(cnt[i]),
                     "aabb_sum": int(box.sum()), "micro_sum": int(ctr[..., 1].astype(np.int64).sum())}
    print(json.dumps({"case": a.case, "region": a.region, "results": out}, indent=1))


if __name__ == "__main__":
    main()
