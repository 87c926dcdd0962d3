#!/usr/bin/env python3
"""Sweep of the Kerr shadow-ray occlusion proof's margin (rrt_device.h kerr_occluded_proof,
rrt_host.cpp RRT_KPROOF_*) over its envelope, on the CPU restatement (tests/kerr_proof_sim.py):
random holes (r_s, delta_theta, spin a/M, spin axis, position) in the Cornell-box scenes, random
shadow rays from surface points.  For every ray the proof calls occluded, the restatement's exact
shadow query must return true (a violation otherwise), and the exact march's points must stay
within delta of the coarse chords (the worst deviation / delta is reported: the margin's headroom).
Usage: python3 tools/kerr_proof_sweep.py [--configs 24] [--rays 300] [--out profiles/r04_kerr_proof_sweep.json]"""
import argparse
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
from kerr_proof_sim import constants, deviation, quads, run  # noqa: E402
from shadow_proof_sim import occluders  # noqa: E402

SCENES = ["cfg3_bunny_1080p_s64", "cfg2_spheres_1080p_s64_flat", "empty_64x48_s8", "coil_96x72_s8"]


def shadow_rays(T, n, g, eps=1e-11):
    """random surface points (area-weighted) and directions uniform over the hemisphere facing the room"""
    area = 0.5 * np.linalg.norm(np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]), axis=1)
    t = g.choice(len(T), n, p=area / area.sum())
    u, v = g.random(n), g.random(n)
    flip = u + v > 1
    u, v = np.where(flip, 1 - u, u), np.where(flip, 1 - v, v)
    hp = T[t, 0] + u[:, None] * (T[t, 1] - T[t, 0]) + v[:, None] * (T[t, 2] - T[t, 0])
    nn = np.cross(T[t, 1] - T[t, 0], T[t, 2] - T[t, 0])
    nn /= np.linalg.norm(nn, axis=1)[:, None]
    d = g.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    # the hemisphere facing the room's centre (a shading normal points into the room)
    ctr = 0.5 * (T.reshape(-1, 3).min(0) + T.reshape(-1, 3).max(0))
    side = np.where(((ctr - hp) * nn).sum(1) < 0, -1.0, 1.0)
    d = np.where(((d * nn).sum(1) * side)[:, None] < 0, -d, d)
    return hp + eps * d, d


def sweep(n_configs, n_rays, seed, only=None):
    g = np.random.default_rng(seed)
    setups = []
    for name in SCENES:
        c = Case(name)
        sf = O.Scene(c.scene_path)
        lib_sf = rrt.SceneFile(c.scene_path)
        r = rrt.Renderer(device=-1)
        r.set_scene(lib_sf)
        boxes, _, _ = r.bvh()
        r.close()
        lo, hi = boxes[0][:3].copy(), boxes[0][3:].copy()
        T = lib_sf.triangles()
        faces, w = occluders(T, lo, hi)
        setups.append((name, sf, T, lo, hi, quads(T, faces, lo, hi), w))
    out = []
    for k in range(n_configs):
        name, sf, T, lo, hi, pieces, w = setups[k % len(setups)]
        ext = hi - lo
        while True:  # a hole inside the room whose envelope admits the proof
            cpos = lo + ext * (0.2 + 0.6 * g.random(3))
            rs = float(g.choice([0.08, 0.1, 0.15, 0.2, 0.3]))
            dt = float(g.choice([0.02, 0.05, 0.1]))
            bh = (float(cpos[0]), float(cpos[1]), float(cpos[2]), rs, dt)
            K = constants(bh, lo, hi, w)
            if K["in_envelope"]:
                break
        spin = float(g.choice([0.0, 0.5, 0.9, 0.99]))
        axis = g.normal(size=3) if g.random() < 0.5 else np.array([0.0, 1.0, 0.0])
        axis = tuple(float(x) for x in axis / np.linalg.norm(axis))
        p = O.make_params(64, 64, bh=bh, kerr=(spin, axis))
        o, d = shadow_rays(T, n_rays, g)
        if only is not None and k != only:
            continue
        proven = viol = 0
        worst, worst_ray = 0.0, None
        for i in range(n_rays):
            ok, rows, extra = run(K, pieces, bh, spin, axis, o[i], d[i])
            if not ok:
                continue
            proven += 1
            if not O.shadow_query(sf, p, o[i], d[i]):
                viol += 1
            dv = deviation(bh, spin, axis, o[i], d[i], extra) / K["delta"]
            if dv > worst:
                worst, worst_ray = dv, [o[i].tolist(), d[i].tolist()]
        rec = dict(scene=name, bh=bh, spin=spin, axis=axis, rays=n_rays, proven=proven, violations=viol,
                   worst_deviation_over_delta=worst, worst_ray=worst_ray)
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, default=24)
    ap.add_argument("--rays", type=int, default=300)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", type=int, default=None, help="run only configuration k (its rays as in the full run)")
    a = ap.parse_args()
    recs = sweep(a.configs, a.rays, a.seed, a.only)
    summary = dict(configs=len(recs), rays=sum(r["rays"] for r in recs), proven=sum(r["proven"] for r in recs),
                   violations=sum(r["violations"] for r in recs),
                   worst_deviation_over_delta=max(r["worst_deviation_over_delta"] for r in recs), records=recs)
    print(json.dumps({k: v for k, v in summary.items() if k != "records"}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
