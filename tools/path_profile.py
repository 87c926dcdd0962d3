#!/usr/bin/env python3
"""Diagnostic: where the path pool kernel's (csrc/rrt_path.hip) wave time goes on a bench.py
workload -- path phase, claims, trace phase -- and the trace phase's lane use (rays dealt per
round / 64).  Needs the -DRRT_PROFILE=1 build (make prof -> tools/librrt_prof.so, via RRT_LIB)."""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import rrt  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="m3")
    ap.add_argument("--variants", type=int, nargs="+", default=[4, 3, 2])
    a = ap.parse_args()
    L = rrt.lib()
    L.rrt_prof_read_path.argtypes = [C.c_void_p]
    r = rrt.Renderer(0)
    wl = bench.WORKLOADS[a.workload]
    work = tempfile.mkdtemp()
    scene, cam, _, _ = bench.load_workload_scene(wl, work)
    r.set_scene(scene)
    r.set_camera(rrt.camera_desc(cam))
    r.set_envmap(bench.load_workload_env(wl, work))
    r.set_black_hole(*wl["bh"])
    buf = np.zeros(8, np.uint64)
    out = {}
    for v in a.variants:
        p = rrt.render_params(wl["w"], wl["h"], ns_aa=wl["spp"], max_ray_depth=wl.get("depth", 1), variant=v)
        L.rrt_prof_read_path(buf.ctypes.data)
        r.render(p, 0, 0, wl["w"], wl["h"])
        ms = r.stats().last_kernel_ms
        L.rrt_prof_read_path(buf.ctypes.data)
        path, claim, trace, rounds, rays, waves = (float(x) for x in buf[:6])
        tot = path + claim + trace
        out[v] = {"kernel": r.stats().kernel.decode(), "ms": ms, "waves": waves, "rounds_per_wave": rounds / max(waves, 1),
                  "path_phase": path / tot, "claims": claim / tot, "trace_phase": trace / tot,
                  "lanes_dealt": rays / max(rounds, 1) / 64.0,
                  "us_per_round": ms * 1e3 / max(rounds / max(waves, 1), 1)}
        print(json.dumps({str(v): out[v]}), flush=True)


if __name__ == "__main__":
    main()
