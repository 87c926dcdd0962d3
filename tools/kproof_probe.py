#!/usr/bin/env python3
"""Diagnostic: executed work (micro steps, AABB / primitive / plane tests per sample) and kernel time
of a region of a bench.py workload with the shadow-ray proofs on and off (RRT_RENDER_NO_SHADOW_PROOF).
Usage: python3 tools/kproof_probe.py --workload cfg5 --region 1600 900 128 128"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import bench  # noqa: E402
import rrt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg5")
    ap.add_argument("--region", type=int, nargs=4, default=[1600, 900, 128, 128])
    ap.add_argument("--spp", type=int, default=0, help="override the workload's spp (0: keep)")
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    work = tempfile.mkdtemp()
    r = rrt.Renderer(0)
    scene, cam, _, _ = bench.load_workload_scene(wl, work)
    r.set_scene(scene)
    r.set_camera(rrt.camera_desc(cam))
    r.set_envmap(bench.load_workload_env(wl, work))
    kerr = wl.get("kerr")
    r.set_black_hole(*wl["bh"], **({"spin": kerr[0], "axis": kerr[1]} if kerr else {}))
    out = {}
    for name, fl in (("proof", 0), ("noproof", rrt.RRT_RENDER_NO_SHADOW_PROOF)):
        p = rrt.render_params(wl["w"], wl["h"], ns_aa=a.spp or wl["spp"], max_ray_depth=wl.get("depth", 1), flags=fl)
        ts = []
        for _ in range(2):
            rgb, cnt, _, _ = r.render(p, *a.region)
            ts.append(r.stats().last_kernel_ms)
        pc = rrt.render_params(wl["w"], wl["h"], ns_aa=a.spp or wl["spp"], max_ray_depth=wl.get("depth", 1),
                               flags=fl | rrt.RRT_RENDER_COUNT_EXECUTED)
        rgb2, cnt2, _, ctr = r.render(pc, *a.region, counters=True)
        n = float(cnt2.sum())
        ctr = ctr.astype(np.float64)
        out[name] = {"kernel_ms": ts, "samples": n, "aabb_per_sample": ctr[..., 0].sum() / n,
                     "micro_per_sample": ctr[..., 1].sum() / n, "prim_per_sample": ctr[..., 2].sum() / n,
                     "plane_per_sample": ctr[..., 3].sum() / n, "rgb_sum": float(rgb.astype(np.float64).sum()),
                     "identical_to_counting_pass": bool(np.array_equal(rgb.view(np.uint32), rgb2.view(np.uint32)))}
    print(json.dumps({"workload": a.workload, "region": a.region, "results": out}, indent=1))


if __name__ == "__main__":
    main()
