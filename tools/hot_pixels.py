#!/usr/bin/env python3
"""Diagnostic: the costliest pixels of a golden workload by per-pixel work counters (executed and
reference-algorithm AABB tests, micro steps, primitive tests), to find straggler pixels.
Usage: python3 tools/hot_pixels.py [--case cfg3_bunny_1080p_s64] [--top 20]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (first: one shared HIP runtime)
import rrt  # noqa: E402
from golden_cases import Case  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg3_bunny_1080p_s64")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    c = Case(a.case)
    g = c.cfg
    r = rrt.Renderer(0)
    r.set_scene(rrt.SceneFile(c.scene_path))
    r.set_envmap(c.envmap)
    r.set_camera(rrt.load_camera(c.camera_path))
    r.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
    out = {}
    for mode, fl in (("executed", rrt.RRT_RENDER_COUNT_EXECUTED), ("reference", 0)):
        p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                              ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                              max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=fl)
        rgb, cnt, draws, ctr = r.render(p, 0, 0, c.frame_w, c.frame_h, counters=True)
        ctr = ctr.astype(np.int64)
        box = ctr[..., 0]
        order = np.argsort(box.ravel())[::-1][:a.top]
        ys, xs = np.unravel_index(order, box.shape)
        out[mode] = {
            "total_aabb": int(box.sum()), "total_micro": int(ctr[..., 1].sum()), "total_prim": int(ctr[..., 2].sum()),
            "aabb_quantiles_per_pixel": [int(v) for v in np.quantile(box, [0.5, 0.9, 0.99, 0.999, 1.0])],
            "top_share_of_aabb": float(box.ravel()[order].sum() / max(box.sum(), 1)),
            "top": [{"x": int(x), "y": int(y), "aabb": int(box[y, x]), "micro": int(ctr[y, x, 1]),
                     "prim": int(ctr[y, x, 2]), "q": int(ctr[y, x, 3]), "count": int(cnt[y, x]),
                     "rgb": [float(v) for v in rgb[y, x]]} for x, y in zip(xs, ys)]}
    print(json.dumps({"case": a.case, "results": out}, indent=1))


if __name__ == "__main__":
    main()
