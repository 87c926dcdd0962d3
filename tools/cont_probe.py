#!/usr/bin/env python3
"""Diagnostic: every rank's launch of bench.py's N-way split of a workload, under library A/B
environment settings (NAME=VALUE,... per setting; "-" for none), one process: the launch time, its
main kernels' time, the heavy-list and continuation counts per rank.
Usage: python3 tools/cont_probe.py --workload cfg4 --world 8 - RRT_AB_CONT=0 RRT_AB_CONT_ROOM=0"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (first: one shared HIP runtime)
import bench  # noqa: E402
import rrt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg4", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", type=int, nargs="*", default=None)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    W, H, ts = wl["w"], wl["h"], 32
    r = rrt.Renderer(0)
    scene, cam, _, _ = bench.load_workload_scene(wl, tempfile.mkdtemp(prefix="rrt_cp_"))
    r.set_scene(scene)
    r.set_camera(rrt.camera_desc(cam))
    r.set_envmap(bench.load_workload_env(wl, tempfile.mkdtemp(prefix="rrt_cp_")))
    kerr = wl.get("kerr")
    r.set_black_hole(*wl["bh"], **({"spin": kerr[0], "axis": kerr[1]} if kerr else {}))
    ranks = a.ranks if a.ranks else list(range(a.world))
    sets = {k: rrt.partition_tiles(W, H, ts, k, a.world) for k in ranks}
    n = max(len(t) for t in sets.values()) * ts * ts
    prgb = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
    pcnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    p = rrt.render_params(W, H, ns_aa=wl["spp"], max_ray_depth=wl.get("depth", 1), variant=a.variant)
    res = {}
    r.render_tiles_device(p, sets[ranks[0]], ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)  # warm-up
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for st in a.settings:
            for kv in list(os.environ):
                if kv.startswith("RRT_AB_"):
                    del os.environ[kv]
            for kv in filter(None, st.split(",")):
                if kv != "-":
                    k, _, v = kv.partition("=")
                    os.environ[k] = v
            for k in ranks:
                r.render_tiles_device(p, sets[k], ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
                torch.cuda.synchronize()
                x = r.stats()
                res.setdefault(st, {}).setdefault(k, []).append(
                    (x.last_kernel_ms, x.last_main_kernel_ms, x.last_heavy_pixels, x.last_cont_pixels))
    for st, per in res.items():
        for k, v in per.items():
            v = np.array(v)
            print(json.dumps({"setting": st, "rank": k, "launch_ms": float(np.median(v[:, 0])),
                              "main_ms": float(np.median(v[:, 1])), "heavy": int(v[-1, 2]), "cont": int(v[-1, 3])}))


if __name__ == "__main__":
    main()
