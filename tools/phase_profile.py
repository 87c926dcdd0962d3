#!/usr/bin/env python3
"""Diagnostic: per-phase wave time of the depth<=1 sample-parallel (batch) kernel, from a build with
-DRRT_PROFILE=1 (make -C relativistic-ray-tracer_amd EXTRA=-DRRT_PROFILE=1), loaded through
RRT_LIB.  Prints the share of wave time spent in camera queries, miss proofs, shadow queries, their micro
steps and BVH walks (busiest lane per wave, summed over waves)."""
import argparse
import ctypes as C
import json
import os
import sys

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
    ap.add_argument("--flags", type=int, nargs="+", default=[0, rrt.RRT_RENDER_NO_MISS_PROOF])
    ap.add_argument("--tiles", type=int, nargs="*", default=None, help="x y pairs of 32x32 tiles (default: all)")
    ap.add_argument("--region", type=int, nargs=4, default=None, help="x0 y0 w h: render only this region")
    ap.add_argument("--workload", default=None, help="a bench.py workload (cfg2..cfg5, m3) instead of a golden case")
    ap.add_argument("--rank", type=int, nargs=2, default=None, metavar=("K", "N"),
                    help="rank K's tile set of bench.py's N-way split (rrt_partition_tiles)")
    a = ap.parse_args()
    L = rrt.lib()
    L.rrt_prof_read.argtypes = [C.c_void_p]
    L.rrt_prof_read_slow.argtypes = [C.c_void_p]
    r = rrt.Renderer(0)
    if a.workload:
        # bench.py's own set-up of the workload (native ingest, generated scenes / sky, Kerr)
        sys.path.insert(0, ROOT)
        import tempfile
        import bench
        wl = bench.WORKLOADS[a.workload]
        work = tempfile.mkdtemp()
        scene, cam, _, _ = bench.load_workload_scene(wl, work)
        r.set_scene(scene)
        r.set_camera(rrt.camera_desc(cam))
        r.set_envmap(bench.load_workload_env(wl, work))
        kerr = wl.get("kerr")
        r.set_black_hole(*wl["bh"], **({"spin": kerr[0], "axis": kerr[1]} if kerr else {}))
        frame_w, frame_h = wl["w"], wl["h"]
        g = dict(ns_aa=wl["spp"], max_ray_depth=wl.get("depth", 1), ns_area_light=1, samples_per_batch=32,
                 max_tolerance=0.05, direct_hemisphere=False)
        a.case = a.workload
    else:
        c = Case(a.case)
        g = c.cfg
        r.set_scene(rrt.SceneFile(c.scene_path))
        r.set_camera(rrt.load_camera(c.camera_path))
        r.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
        frame_w, frame_h = c.frame_w, c.frame_h
    tiles = rrt.partition_tiles(frame_w, frame_h, 32, 0, 1)
    if a.tiles:
        tiles = np.array(a.tiles, np.uint32).reshape(-1, 2)
    if a.rank:
        tiles = rrt.partition_tiles(frame_w, frame_h, 32, a.rank[0], a.rank[1])
        a.case = f"{a.case}_rank{a.rank[0]}of{a.rank[1]}"
    n = len(tiles) * 1024
    prgb = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
    pcnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    HDR = 24
    buf = np.zeros(HDR + 3 * 16384, np.uint64)
    out = {}
    for fl in a.flags:
        p = rrt.render_params(frame_w, frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                              ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                              max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=fl)
        L.rrt_prof_read(buf.ctypes.data)
        L.rrt_prof_read_slow(np.zeros(64, np.uint64).ctypes.data)
        if a.region:
            r.render(p, *a.region)
        else:
            r.render_tiles_device(p, tiles, 32, prgb.data_ptr(), pcnt.data_ptr())
        ms = r.stats().last_kernel_ms
        L.rrt_prof_read(buf.ctypes.data)
        tot, tq, tm, tt, tp, tsq, tst = (float(v) for v in buf[:7])
        t0, t1, nw, tex = int(buf[8]), int(buf[9]), int(buf[10]), int(buf[11])
        span = t1 - t0
        m = min(nw, 16384)
        ends = (buf[HDR:HDR + m].astype(np.float64) - t0) / span
        starts = (buf[HDR + 16384:HDR + 16384 + m].astype(np.float64) - t0) / span
        work = buf[HDR + 2 * 16384:HDR + 2 * 16384 + m]
        blocks, samples = (work >> np.uint64(32)).astype(np.int64), (work & np.uint64(0xffffffff)).astype(np.int64)
        res = blocks > 0
        np.savez(f"gpurun_out/waves_{fl}.npz", ends=ends, starts=starts, blocks=blocks, samples=samples)
        if not a.region and n <= (1 << 21):  # per-pixel elapsed ticks and rounds (batch kernel)
            L.rrt_prof_read_px.argtypes = [C.c_void_p, C.c_uint32]
            pxv = np.zeros(n, np.uint32)
            L.rrt_prof_read_px(pxv.ctypes.data, n)
            img_t = np.zeros((frame_h, frame_w), np.float32)
            img_r = np.zeros((frame_h, frame_w), np.uint8)
            sl = np.arange(n)
            xs = tiles[sl // 1024, 0].astype(np.int64) + sl % 1024 % 32
            ys = tiles[sl // 1024, 1].astype(np.int64) + sl % 1024 // 32
            ok = (xs < frame_w) & (ys < frame_h)
            img_t[ys[ok], xs[ok]] = (pxv[ok] >> 8) / (span / ms)
            img_r[ys[ok], xs[ok]] = pxv[ok] & 255
            # when each pixel stopped, as a fraction of the kernel's span (-1: not rendered here)
            L.rrt_prof_read_px_end.argtypes = [C.c_void_p, C.c_uint32]
            pxe = np.zeros(n, np.uint32)
            L.rrt_prof_read_px_end(pxe.ctypes.data, n)
            img_e = np.full((frame_h, frame_w), -1.0, np.float32)
            rel = ((pxe.astype(np.int64) - (t0 & 0xffffffff)) % (1 << 32)) / span
            got = ok & (pxv > 0)
            img_e[ys[got], xs[got]] = rel[got]
            np.savez_compressed(f"gpurun_out/px_{a.case}_{fl}.npz", ms=img_t, rounds=img_r, end=img_e)
        slow = np.zeros(64, np.uint64)
        L.rrt_prof_read_slow(slow.ctypes.data)
        slow_px = []
        for v in sorted((int(x) for x in slow if x), reverse=True)[:16]:
            sl, ticks = v & 0xffffff, v >> 38
            t_i, rr = sl // 1024, sl % 1024
            slow_px.append({"x": int(tiles[t_i][0]) + rr % 32, "y": int(tiles[t_i][1]) + rr // 32,
                            "ms": ticks / (span / ms), "rounds": (v >> 31) & 127, "steps": (v >> 24) & 127})
        out[fl] = {"kernel_ms": ms, "ticks_per_ms": span / ms, "waves": nw, "waves_with_work": int(res.sum()),
                   "exhausted_at": (tex - t0) / span, "wave_cycles": tot,
                   "camera_query": tq / tot, "micro_all": tm / tot, "camera_walk": tt / tot,
                   "miss_proof": tp / tot, "shadow_query": tsq / tot, "shadow_walk": tst / tot,
                   "outside_queries_and_proof": 1 - (tq + tp + tsq) / tot,
                   "claim": float(buf[16]) / tot, "chain": float(buf[17]) / tot, "shade_incl_shadow": float(buf[18]) / tot,
                   "fold": float(buf[19]) / tot,
                   # lanes active in each phase (lane sum / (64 x busiest lane), summed over waves)
                   "lane_use": {k: float(buf[i]) / (64.0 * float(buf[j])) if buf[j] else None for k, i, j in
                                (("total", 15, 0), ("camera_query", 12, 1), ("micro", 23, 2), ("camera_walk", 21, 3),
                                 ("miss_proof", 14, 4), ("shadow_query", 13, 5), ("shadow_walk", 22, 6),
                                 ("shade", 20, 18))},
                   "slowest_pixels": slow_px,
                   "busy_frac_working_waves": float(((ends - starts)[res]).sum() / max(res.sum(), 1)),
                   "working_wave_end_q": [round(float(q), 3) for q in np.quantile(ends[res], [0.05, 0.25, 0.5, 0.75, 0.95, 1.0])],
                   "working_wave_start_q": [round(float(q), 3) for q in np.quantile(starts[res], [0.05, 0.5, 0.95, 1.0])],
                   "claims_per_wave": float(blocks[res].mean()), "rounds_per_wave": float(samples[res].mean())}
    print(json.dumps({"case": a.case, "results": out}, indent=1))


if __name__ == "__main__":
    main()
