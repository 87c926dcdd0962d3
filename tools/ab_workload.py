#!/usr/bin/env python3
"""A/B kernel variants (rrt_render_params.variant = waves per SIMD, flags) on a bench.py workload,
interleaved rounds in one process; prints the HIP-event kernel time per variant.
Usage: python3 tools/ab_workload.py --workload cfg5 --rounds 2 3 4 5   (VARIANT, VARIANT:FLAGS or
VARIANT:FLAGS:RRT_AB_X=V,... -- library A/B switches the launch reads from the environment)
--world N: time each of the N ranks' tile sets (bench.py's block-cyclic split) on this one GPU and
report the slowest rank per variant (the N-GPU frame's kernel time, without the gather)."""
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
    ap.add_argument("--workload", default="cfg5", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--tile", type=int, default=32, help="tile size of the split (bench.py: 32)")
    ap.add_argument("--split", default="lib", help="lib (rrt_partition_tiles) or latS: rank = (tx + S ty) % world")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    W, H, ts = wl["w"], wl["h"], a.tile
    work = tempfile.mkdtemp(prefix="rrt_ab_")
    r = rrt.Renderer(0)
    scene, cam, _, _ = bench.load_workload_scene(wl, work)
    r.set_scene(scene)
    r.set_camera(rrt.camera_desc(cam))
    r.set_envmap(bench.load_workload_env(wl, work))
    kerr = wl.get("kerr")
    r.set_black_hole(*wl["bh"], **({"spin": kerr[0], "axis": kerr[1]} if kerr else {}))
    if a.split == "lib":
        sets = [rrt.partition_tiles(W, H, ts, k, a.world) for k in range(a.world)]
    else:  # A/B of other splits: a 2-D lattice of tiles over the ranks
        sm = int(a.split[3:])
        tw, th = (W + ts - 1) // ts, (H + ts - 1) // ts
        sets = [np.array([(tx * ts, ty * ts) for ty in range(th) for tx in range(tw) if (tx + sm * ty) % a.world == k],
                         np.uint32).reshape(-1, 2) for k in range(a.world)]
    n = max(len(t) for t in sets) * ts * ts
    prgb = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
    pcnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    times, sums = {v: [] for v in a.variants}, {}
    per_rank = {v: [[] for _ in sets] for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            var, _, rest = v.partition(":")
            fl, _, envs = rest.partition(":")  # VARIANT:FLAGS:NAME=VALUE,... (library A/B switches read per launch)
            for kv in os.environ.copy():
                if kv.startswith("RRT_AB_"):
                    del os.environ[kv]
            for kv in filter(None, envs.split(",")):
                k, _, val = kv.partition("=")
                os.environ[k] = val
            p = rrt.render_params(W, H, ns_aa=wl["spp"], max_ray_depth=wl.get("depth", 1), variant=int(var), flags=int(fl or 0))
            worst, tot_rgb, tot_cnt = 0.0, 0.0, 0
            for k, tiles in enumerate(sets):
                r.render_tiles_device(p, tiles, ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
                torch.cuda.synchronize()
                ms = r.stats().last_kernel_ms
                per_rank[v][k].append(ms)
                worst = max(worst, ms)
                m = len(tiles) * ts * ts
                tot_rgb += float(prgb[:3 * m].double().sum().item())
                tot_cnt += int(pcnt[:m].long().sum().item())
            times[v].append(worst)
            sums[v] = (tot_rgb, tot_cnt)
            print(v, times[v][-1], r.stats().kernel.decode(), flush=True)
    # diagnostic flags change outputs; environment switches (third field) do not
    same = len(set(s for v, s in sums.items() if v.split(":")[1:2] in ([], ["0"], [""]))) <= 1
    print(json.dumps({"workload": a.workload, "identical_outputs": same,
                      "median_ms": {v: float(np.median(t)) for v, t in times.items()},
                      **({"world": a.world, "rank_median_ms": {v: [float(np.median(x)) for x in pr] for v, pr in per_rank.items()}}
                         if a.world > 1 else {}),
                      "sums": {v: list(x) for v, x in sums.items()}}))


if __name__ == "__main__":
    main()
