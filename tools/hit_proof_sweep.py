#!/usr/bin/env python3
"""Sweep of the camera-ray hit proof and the zero-sample proof (rrt_device.h camera_hit_proof,
zero_sample_proof; numpy mirror tests/hit_proof_sim.py) against the oracle's exact queries.

For random jittered camera rays of a golden case's framing (optionally with random holes): every ray
the hit proof takes must be a hit of the restatement's exact closest-hit query (ro_query) on a
non-emitting surface whose hit point lies within a small fraction of the margin of the proof's
crossing point Q; and for every light sample whose shadow ray from Q the occlusion proof takes
(margin scale MS), the exact shadow query from the exact hit point must be occluded.
Usage: python3 tools/hit_proof_sweep.py --case cfg3_bunny_1080p_s64 --rays 4000 [--holes 8]"""
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
from hit_proof_sim import nocc_box, prove  # noqa: E402
from miss_proof_sim import constants  # noqa: E402
from shadow_proof_sim import occluders, run as shadow_run, trigger_box  # noqa: E402

MS = 2.0  # the zero-sample proof's shadow margin scale (rrt_device.h RRT_ZERO_MS)


def scene_tables(sf):
    """per-triangle bsdf type (SceneFile.triangles() order) and the area lights' vectors"""
    d = rrt.SceneDesc.from_address(sf.desc())
    btype = [C.cast(d.bsdfs, C.POINTER(C.c_uint32))[15 * i] for i in range(d.n_bsdfs)]
    tb, spheres = [], []
    for i in range(d.n_objects):
        o = d.objects[i]
        if o.kind == 0:
            tb += [btype[o.bsdf]] * o.n_triangles
        else:
            spheres.append((np.array(o.center[:]), float(o.radius)))
    lights = []
    for i in range(d.n_lights):
        L = d.lights[i]
        if L.type == 0:
            lights.append((np.array(L.radiance[:], np.float32), np.array([[L.v[k][j] for j in range(3)] for k in range(4)])))
    return np.array(tb), lights, spheres


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg3_bunny_1080p_s64")
    ap.add_argument("--rays", type=int, default=4000)
    ap.add_argument("--holes", type=int, default=0, help="random holes (else the case's own)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    c = Case(a.case)
    sf = rrt.SceneFile(c.scene_path)
    T = sf.triangles()
    tb, lights, spheres = scene_tables(sf)
    r = rrt.Renderer(device=-1)
    r.set_scene(sf)
    boxes, _, _ = r.bvh()
    r.close()
    lo, hi = boxes[0][:3].copy(), boxes[0][3:].copy()
    faces, w = occluders(T, lo, hi)
    emit = [sum(1 << i for i, t in enumerate(faces[f]) if tb[t[4]] == 1) for f in range(6)]
    nlo, nhi = nocc_box(T, faces, spheres)
    osc = O.Scene(c.scene_path)
    cam = O.load_camera(c.camera_path)
    cols = np.array(cam.c2w, np.float64).reshape(3, 3).T.ravel().copy()
    pos = np.array(cam.pos, np.float64)
    W, H = c.frame_w, c.frame_h
    g = np.random.default_rng(a.seed)
    holes = [tuple(c.cfg["bh"])]
    ext = hi - lo
    for _ in range(a.holes):
        cp = lo + ext * (0.2 + 0.6 * g.random(3))
        holes.append((float(cp[0]), float(cp[1]), float(cp[2]), float(g.choice([0.05, 0.1, 0.2, 0.3])),
                      float(g.choice([0.05, 0.1, 0.2]))))
    mn, mx = C.c_double(), C.c_double()
    tot = dict(rays=0, proven=0, hit_violations=0, max_dev=0.0, light_samples=0, zero_proven=0, zero_violations=0)
    per = []
    for bh in holes:
        K = constants(np.array(bh), lo, hi)
        box = trigger_box(K, w)
        p = O.make_params(W, H, bh=bh)
        n_pr = n_z = 0
        for _ in range(a.rays // len(holes)):
            o, d = np.zeros(3), np.zeros(3)
            O.lib().ro_camera_ray(cam.hFov, cam.vFov, pos, cols, cam.nClip, cam.fClip, g.random(), g.random(), o, d,
                                  C.byref(mn), C.byref(mx))
            tot["rays"] += 1
            ok, ti, Q, j = prove(K, faces, box, emit, nlo, nhi, o, d)
            if not ok:
                continue
            tot["proven"] += 1
            n_pr += 1
            hit, hp, nn, bsdf = O.query(osc, p, o, d)
            dev = float(np.linalg.norm(hp - Q)) if hit else np.inf
            tot["max_dev"] = max(tot["max_dev"], dev)
            if not hit or tb[ti] == 1 or dev > 1e-7:
                tot["hit_violations"] += 1
                print("HIT VIOLATION", bh, o.tolist(), d.tolist(), hit, dev, flush=True)
                continue
            for rad, v in lights:
                rands = g.integers(0, 2 ** 31 - 1, 2).astype(np.int32)
                wq, we = np.zeros(3), np.zeros(3)
                Lq, Le = np.zeros(3, np.float32), np.zeros(3, np.float32)
                dist, pdf = C.c_float(), C.c_float()
                O.lib().ro_area_sample(rad, np.ascontiguousarray(v.ravel()), np.ascontiguousarray(Q), rands, Lq, wq,
                                       C.byref(dist), C.byref(pdf))
                O.lib().ro_area_sample(rad, np.ascontiguousarray(v.ravel()), np.ascontiguousarray(hp), rands, Le, we,
                                       C.byref(dist), C.byref(pdf))
                tot["light_samples"] += 1
                proven, _, _, _, _ = shadow_run(K, faces, box, (Q + 1e-11 * wq)[None], wq[None], ms=MS)
                if proven[0]:
                    tot["zero_proven"] += 1
                    n_z += 1
                    if not O.shadow_query(osc, p, hp + 1e-11 * we, we):
                        tot["zero_violations"] += 1
                        print("ZERO VIOLATION", bh, hp.tolist(), we.tolist(), flush=True)
        per.append(dict(bh=bh, rays=a.rays // len(holes), proven=n_pr, zero_proven=n_z))
    out = dict(case=a.case, ms=MS, **tot, holes=per)
    print(json.dumps(out))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
