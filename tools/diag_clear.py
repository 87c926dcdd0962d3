#!/usr/bin/env python3
"""Diagnostic: how much of the geodesic march the empty-space grid removes (cfg3 by default).
Renders with RRT_RENDER_COUNTERS | RRT_RENDER_DIAG_CLEAR_STATS and prints per-sample micro
steps, the fraction of micro segments the grid proves clear, and the AABB tests left outside
them.  Not a parity or bench tool (the counting kernel never skips)."""
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
    ap.add_argument("--res", type=int, nargs="+", default=[0])
    a = ap.parse_args()
    c = Case(a.case)
    g = c.cfg
    out = {}
    for res in a.res:
        r = rrt.Renderer(0, free_grid_res=res)
        r.set_scene(rrt.SceneFile(c.scene_path))
        r.set_camera(rrt.load_camera(c.camera_path))
        r.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
        flags = rrt.RRT_RENDER_COUNTERS | rrt.RRT_RENDER_DIAG_CLEAR_STATS
        p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                              ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                              max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=flags)
        _, cnt, _, ct = r.render(p, 0, 0, c.frame_w, c.frame_h, counters=True)
        s = ct.reshape(-1, 4).astype(np.float64).sum(0)
        n = float(cnt.astype(np.int64).sum())
        st = r.stats()
        out[res or 128] = {"grid": list(st.grid_n), "free_cells": st.grid_free_frac,
                           "micro_per_sample": s[1] / n, "clear_frac": s[3] / s[1],
                           "aabb_per_sample": s[0] / n, "aabb_left_per_sample": s[2] / n}
        r.close()
    print(json.dumps({"case": a.case, "results": out}, indent=1))


if __name__ == "__main__":
    main()
