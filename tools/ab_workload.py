#!/usr/bin/env python3
"""A/B kernel variants (rrt_render_params.variant = waves per SIMD, flags) on a bench.py workload,
interleaved rounds in one process; prints the HIP-event kernel time per variant.
Usage: python3 tools/ab_workload.py --workload cfg5 --rounds 2 3 4 5   (VARIANT, VARIANT:FLAGS or
VARIANT:FLAGS:RRT_AB_X=V,... -- library A/B switches the launch reads from the environment)
--world N: time each of the N ranks' tile sets (bench.py's block-cyclic split) on this one GPU and
report the slowest rank per variant (the N-GPU frame's kernel time, without the gather).
Outputs: every rank's packed buffer is poisoned (NaN radiance, count -1) before its launch and
unpacked into a full frame (itself poisoned per variant); variants are compared by the SHA-256 of
that frame's bits ("identical_outputs"), and the frame is checked bit for bit against the
workload's reference goldens where it has them ("verified", bench.verify_frame)."""
import argparse
import hashlib
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
    ap.add_argument("--tile", type=int, default=0, help="tile size of the split (default: bench.py's for the workload)")
    ap.add_argument("--split", default="lib", help="lib (rrt_partition_tiles), latS: rank = (tx + S ty) %% world, "
                    "serS: serpentine index k, rank = (k + S ty) %% world")
    ap.add_argument("--rotate", action="store_true", help="round r renders the ranks from rank r %% world on "
                    "(a rank's time must not depend on its place in the sequence)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    wl = bench.WORKLOADS[a.workload]
    W, H, ts = wl["w"], wl["h"], a.tile or wl.get("tile", bench.TILE)
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
    elif a.split.startswith("ser"):  # serpentine order, tile k of row ty to rank (k + S ty) % world
        sm = int(a.split[3:])
        tw, th = (W + ts - 1) // ts, (H + ts - 1) // ts
        order = [((i if ty % 2 == 0 else tw - 1 - i), ty) for ty in range(th) for i in range(tw)]
        sets = [np.array([(tx * ts, ty * ts) for k, (tx, ty) in enumerate(order) if (k + sm * ty) % a.world == q],
                         np.uint32).reshape(-1, 2) for q in range(a.world)]
    else:  # A/B of other splits: a 2-D lattice of tiles over the ranks
        sm = int(a.split[3:])
        tw, th = (W + ts - 1) // ts, (H + ts - 1) // ts
        sets = [np.array([(tx * ts, ty * ts) for ty in range(th) for tx in range(tw) if (tx + sm * ty) % a.world == k],
                         np.uint32).reshape(-1, 2) for k in range(a.world)]
    n = max(len(t) for t in sets) * ts * ts
    prgb = torch.zeros(n * 3, dtype=torch.float32, device="cuda")
    pcnt = torch.zeros(n, dtype=torch.int32, device="cuda")
    frgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    fcnt = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    times, sums, digests, verified = {v: [] for v in a.variants}, {}, {}, {}
    # warm-up (the first launch of a process loads the kernels): rank 0's tiles once, untimed
    r.render_tiles_device(rrt.render_params(W, H, ns_aa=wl["spp"], max_ray_depth=wl.get("depth", 1)), sets[0], ts,
                          prgb.data_ptr(), pcnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    per_rank = {v: [[] for _ in sets] for v in a.variants}
    for rnd in range(a.rounds):
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
            worst = 0.0
            frgb.view(torch.int32).fill_(-1)
            fcnt.fill_(-1)
            seq = [(rnd + j) % len(sets) for j in range(len(sets))] if a.rotate else range(len(sets))
            for k in seq:
                tiles = sets[k]
                prgb.view(torch.int32).fill_(-1)  # poison: stale slots of an earlier rank cannot leak
                pcnt.fill_(-1)
                r.render_tiles_device(p, tiles, ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
                torch.cuda.synchronize()
                ms = r.stats().last_kernel_ms
                per_rank[v][k].append(ms)
                worst = max(worst, ms)
                r.unpack_tiles_device(tiles, ts, W, H, prgb.data_ptr(), pcnt.data_ptr(), frgb.data_ptr(),
                                      fcnt.data_ptr(), stream=s)
            torch.cuda.synchronize()
            times[v].append(worst)
            fr, fc = frgb.cpu().numpy(), fcnt.cpu().numpy()
            sums[v] = (float(fr.astype(np.float64).sum()), int(fc.astype(np.int64).sum()))
            dg = hashlib.sha256(fr.tobytes() + fc.tobytes()).hexdigest()[:16]
            if digests.setdefault(v, dg) != dg:
                digests[v] = "varies"  # a variant whose rounds differ: not deterministic
            if v not in verified:
                verified[v] = bench.verify_frame(a.workload, fr.reshape(H, W, 3), fc.reshape(H, W))
            print(v, times[v][-1], r.stats().kernel.decode(), flush=True)
    # diagnostic flags change outputs; environment switches (third field) do not
    plain = [d for v, d in digests.items() if v.split(":")[1:2] in ([], ["0"], [""])]
    same = len(set(plain)) <= 1 and "varies" not in plain
    print(json.dumps({"workload": a.workload, "identical_outputs": same, "digests": digests,
                      "verified": {v: x[0] for v, x in verified.items()},
                      "median_ms": {v: float(np.median(t)) for v, t in times.items()},
                      **({"world": a.world, "rank_median_ms": {v: [float(np.median(x)) for x in pr] for v, pr in per_rank.items()}}
                         if a.world > 1 else {}),
                      "sums": {v: list(x) for v, x in sums.items()}}))


if __name__ == "__main__":
    main()
