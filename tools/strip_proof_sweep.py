#!/usr/bin/env python3
"""Sweep of the pixel pass's strip level (rrt_device.h rect_miss_proof on 8x8 strips, the numpy
mirror tests/pixel_proof_sim.py): random 8x8-aligned strips of a BASELINE framing; every pixel of
every proven strip -- its four corners and two random jitters -- is marched by the oracle
(ro_micro_chain, bit-exact with the reference), and no segment of it may come near the root box
(a violation otherwise).  Usage: python3 tools/strip_proof_sweep.py --case cfg3_bunny_1080p_s64 --strips 2000
--fov H: the case's camera with a horizontal field of view of H degrees (vertical from the frame's
aspect), to sweep wide-angle framings; small frames (e.g. --case spheres_96x72_s8) make strips that
subtend large angles."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
import oracle_lib as O  # noqa: E402
import rrt  # noqa: E402
from golden_cases import Case  # noqa: E402
from miss_proof_sim import constants  # noqa: E402
from pixel_proof_sim import prove  # noqa: E402
from test_pixel_proof import _loose_root_hit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg3_bunny_1080p_s64")
    ap.add_argument("--strips", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--fov", type=float, default=None, help="override hFov (degrees)")
    a = ap.parse_args()
    c = Case(a.case)
    bh = np.array(c.cfg["bh"], np.float64)
    r = rrt.Renderer(device=-1)
    r.set_scene(rrt.SceneFile(c.scene_path))
    boxes, _, _ = r.bvh()
    r.close()
    lo, hi = boxes[0][:3].copy(), boxes[0][3:].copy()
    K = constants(bh, lo, hi)
    cam = O.load_camera(c.camera_path)
    cols = np.array(cam.c2w, np.float64).reshape(3, 3).T.ravel().copy()
    pos = np.array(cam.pos, np.float64)
    W, H = c.frame_w, c.frame_h
    mn, mx = C.c_double(), C.c_double()
    hfov, vfov = cam.hFov, cam.vFov
    if a.fov is not None:
        hfov = a.fov
        vfov = 2.0 * np.degrees(np.arctan(np.tan(np.radians(hfov) / 2.0) * H / W))

    def ray(sx, sy):
        o, d = np.zeros(3), np.zeros(3)
        O.lib().ro_camera_ray(hfov, vfov, pos, cols, cam.nClip, cam.fClip, sx / W, sy / H, o, d,
                              C.byref(mn), C.byref(mx))
        return o, d

    g = np.random.default_rng(a.seed)
    out = np.zeros((K["steps"] + 1, 8))
    proven = rays = viol = 0
    for _ in range(a.strips):
        x0 = int(g.integers(0, W // 8)) * 8
        y0 = int(g.integers(0, H // 8)) * 8
        o, dc = ray(x0 + 4.0, y0 + 4.0)
        corners = np.array([ray(x0 + (k & 1) * 8, y0 + (k >> 1) * 8)[1] for k in range(4)])
        if not prove(K, o, dc, corners):
            continue
        proven += 1
        for j in range(8):
            for i in range(8):
                for jx, jy in [(0.0, 0.0), (1.0, 0.0), (0.0, 1.0), (1.0, 1.0), tuple(g.random(2)), tuple(g.random(2))]:
                    o2, d2 = ray(x0 + i + jx, y0 + j + jy)
                    k = O.lib().ro_micro_chain(bh, o2, d2, out, K["steps"] + 1)
                    rays += 1
                    viol += int(_loose_root_hit(lo, hi, out[:k]).any())
    rec = dict(case=a.case, hfov=hfov, strips=a.strips, proven=proven, rays_checked=rays, violations=viol)
    print(json.dumps(rec))
    if a.out:
        json.dump(rec, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
