#!/usr/bin/env python3
"""Render one golden case (tests/golden_cases.py) through the HIP path and report time and parity.
Usage: RRT_LIB=... python3 tools/probe_case.py NAME [FLAGS]"""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
import numpy as np  # noqa: E402
import rrt  # noqa: E402
from golden_cases import Case, parity_metrics  # noqa: E402

name, flags = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0
c = Case(name)
r = rrt.Renderer(device=0)
r.set_scene(rrt.SceneFile(c.scene_path))
r.set_envmap(c.envmap)
r.set_camera(rrt.load_camera(c.camera_path))
bh = c.cfg["bh"]
r.set_black_hole(bh[:3], bh[3], bh[4])
g = c.cfg
p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                      ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                      max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=flags)
print("rendering", name, flags, os.environ.get("RRT_LIB", "in-tree"), flush=True)
t0 = time.time()
rgb, cnt, draws, _ = r.render(p, c.x0, c.y0, c.w, c.h, draws=True)
dt = time.time() - t0
s = r.stats()
print(name, "s=%.3f" % dt, "kernel", s.kernel.decode(), "heavy", s.last_heavy_pixels, parity_metrics(c.px["rgb"], rgb),
      "bit_exact", bool(np.array_equal(rgb.view(np.uint32), c.px["rgb"].view(np.uint32))),
      "count_eq", bool(np.array_equal(cnt, c.px["count"])), flush=True)
