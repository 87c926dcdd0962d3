"""Soundness sweep of the three result-identical proofs (rrt_device.h camera_miss_proof,
pixel_miss_proof, shadow_occluded_proof) beyond the BASELINE framings.

TEST INFRASTRUCTURE ONLY (tools/proof_sweep.py writes profiles/r03_proof_sweep.json;
tests/test_proof_envelope.py runs a small sweep).  Each configuration draws a Cornell-box scene, a
black hole (centre inside or outside the room, r_s, delta_theta), a camera (position, aim, field
of view) and a resolution, then checks the numpy mirrors of the proofs (tests/*_proof_sim.py)
against the C restatement's bit-exact march of the reference (oracle ro_micro_chain, blackhole.cpp
/ bvh.cpp):

* camera proof: on random jittered camera rays, the recurrence's deviation from the reference's
  points over the proof's margin (headroom = 1 / that), and every accepted ray's reference
  segments fail the root-box test;
* pixel proof: on random pixels, every proven pixel's corner and jittered rays miss the root box
  (loose slab test);
* shadow proof: on shadow rays from random surface points towards the area light, the
  deviation / margin, and every accepted ray's reference chain is uncaptured through the proof's
  segment whose triangle test (triangle.cpp) accepts the proof's triangle.
"""
import ctypes as C
import os

import numpy as np

import oracle_lib as O
from miss_proof_sim import constants, run as miss_run
from pixel_proof_sim import prove as pixel_prove
from shadow_proof_sim import occluders, run as shadow_run, trigger_box

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CB_SCENES = ["CBbunny", "CBspheres_lambertian", "CBspheres", "CBcoil", "CBgems", "CBempty",
             "CBspheres_microfacet_al_ag"]
EPS = 1e-11

# the envelope the proofs are enabled in (rrt_host.cpp proof_envelope): delta_theta and the
# hole's Schwarzschild radius relative to the root box's largest extent
DT_RANGE = (0.04, 0.6)     # include/rrt.h RRT_PROOF_DT_MIN / _MAX
RS_OVER_BOX_MAX = 0.5      # include/rrt.h RRT_PROOF_RS_OVER_EXTENT


def _scene(name):
    import rrt
    sf = rrt.SceneFile(os.path.join(GOLD, "scenes", name + ".rrts"))
    r = rrt.Renderer(device=-1)
    r.set_scene(sf)
    boxes, _, _ = r.bvh()
    r.close()
    return sf, boxes[0][:3].copy(), boxes[0][3:].copy()


def draw_config(g, scene=None, dt_range=DT_RANGE, rs_max=RS_OVER_BOX_MAX):
    """A random configuration: scene, hole (cx, cy, cz, r_s, dt), camera (pos, c2w columns, hFov,
    vFov) and frame size."""
    name = scene or CB_SCENES[g.integers(len(CB_SCENES))]
    sf, lo, hi = _scene(name)
    ext = hi - lo
    mid = 0.5 * (lo + hi)
    # hole: inside the room (60%) or outside it, up to 1.5 room sizes from its centre
    if g.random() < 0.6:
        c = lo + ext * (0.15 + 0.7 * g.random(3))
    else:
        c = mid + ext * (g.random(3) - 0.5) * 3.0
        c[2] = max(c[2], hi[2] + 0.1 * ext[2]) if g.random() < 0.5 else c[2]
    scale = float(ext.max())
    rs = float(g.uniform(0.0, rs_max * scale))
    dt = float(g.uniform(*dt_range))
    # camera in front of the open side (+z), aimed near the room's centre
    pos = mid + np.array([g.uniform(-0.6, 0.6) * ext[0], g.uniform(-0.4, 0.4) * ext[1],
                          hi[2] + g.uniform(0.8, 3.0) * ext[2]])
    target = mid + (g.random(3) - 0.5) * 0.3 * ext
    z = pos - target
    z /= np.linalg.norm(z)
    x = np.cross([0.0, 1.0, 0.0], z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    hfov = float(g.uniform(30.0, 70.0))
    W = int(g.choice([96, 320, 640, 1280, 1920, 3840]))
    H = int(W * 9 // 16)
    vfov = float(np.degrees(2 * np.arctan(np.tan(np.radians(hfov) / 2) * H / W)))
    return dict(scene=name, sf=sf, lo=lo, hi=hi, bh=np.array([*c, rs, dt], np.float64),
                pos=pos, cols=np.concatenate([x, y, z]), hfov=hfov, vfov=vfov, W=W, H=H)


def _ray(cfg, sx, sy):
    o, d = np.zeros(3), np.zeros(3)
    mn, mx = C.c_double(), C.c_double()
    O.lib().ro_camera_ray(cfg["hfov"], cfg["vfov"], cfg["pos"], cfg["cols"], 0.01, 1e4, sx / cfg["W"], sy / cfg["H"],
                          o, d, C.byref(mn), C.byref(mx))
    return o, d


def _chains(bh, o, d, steps):
    n = len(o)
    rows = np.zeros((n, steps + 1, 8))
    nrow = np.zeros(n, int)
    out = np.zeros((steps + 1, 8))
    for i in range(n):
        k = O.lib().ro_micro_chain(bh, o[i], d[i], out, steps + 1)
        rows[i, :k] = out[:k]
        nrow[i] = k
    return rows, nrow


def _root_hit(lo, hi, rw):
    t0, t1 = C.c_double(), C.c_double()
    return O.lib().ro_bbox_intersect(lo, hi, rw[0:3].copy(), rw[3:6].copy(), 0.0, rw[6], C.byref(t0),
                                     C.byref(t1)) != 0


def _loose_root_hit(lo, hi, rows):
    o, d, mt = rows[:, 0:3], rows[:, 3:6], rows[:, 6]
    with np.errstate(all="ignore"):
        t0 = (lo[None] - o) / d
        t1 = (hi[None] - o) / d
    tmin = np.nanmax(np.minimum(t0, t1), axis=1)
    tmax = np.nanmin(np.maximum(t0, t1), axis=1)
    tol = 1e-9 * (1.0 + np.abs(tmin) + np.abs(tmax))
    return (tmin <= tmax + tol) & (tmax >= -tol) & (tmin <= mt + tol)


def check_camera(cfg, n, g):
    K = constants(cfg["bh"], cfg["lo"], cfg["hi"])
    xs = g.integers(0, cfg["W"], n) + g.random(n)
    ys = g.integers(0, cfg["H"], n) + g.random(n)
    od = [_ray(cfg, x, y) for x, y in zip(xs, ys)]
    o = np.array([a for a, _ in od])
    d = np.array([b for _, b in od])
    rows, nrow = _chains(cfg["bh"], o, d, K["steps"])
    step0_clear = np.array([not _root_hit(K["lo"], K["hi"], rows[i, 0]) for i in range(n)])
    proven, pts, mrg = miss_run(K, o, d, step0_clear)
    worst = 0.0
    for k in range(2, K["steps"] + 1):
        ref = np.where((nrow > k)[:, None], rows[:, min(k, K["steps"]), 0:3], np.nan)
        last = nrow == k
        endp = rows[np.arange(n), np.maximum(nrow - 1, 0)]
        ref = np.where(last[:, None], endp[:, 0:3] + endp[:, 3:6] * endp[:, 6:7], ref)
        with np.errstate(all="ignore"):
            dev = np.linalg.norm(pts[k] - ref, axis=1) / mrg[k]
        ok = np.isfinite(dev)
        if ok.any():
            worst = max(worst, float(dev[ok].max()))
    bad = sum(1 for i in np.nonzero(proven)[0] if any(_root_hit(K["lo"], K["hi"], rows[i, k]) for k in range(nrow[i])))
    return {"rays": n, "proven": float(proven.mean()), "worst_dev_over_margin": worst, "violations": int(bad)}


def check_pixel(cfg, n, g, n_jit=6):
    K = constants(cfg["bh"], cfg["lo"], cfg["hi"])
    out = np.zeros((K["steps"] + 1, 8))
    proven = bad = 0
    for _ in range(n):
        px, py = int(g.integers(0, cfg["W"])), int(g.integers(0, cfg["H"]))
        o, dc = _ray(cfg, px + 0.5, py + 0.5)
        corners = np.array([_ray(cfg, px + (k & 1), py + (k >> 1))[1] for k in range(4)])
        if not pixel_prove(K, o, dc, corners):
            continue
        proven += 1
        jit = [(float(k & 1), float(k >> 1)) for k in range(4)] + [tuple(g.random(2)) for _ in range(n_jit)]
        for jx, jy in jit:
            o2, d2 = _ray(cfg, px + jx, py + jy)
            k = O.lib().ro_micro_chain(cfg["bh"], o2, d2, out, K["steps"] + 1)
            if _loose_root_hit(K["lo"], K["hi"], out[:k]).any():
                bad += 1
                break
    return {"pixels": n, "proven": proven / n, "violations": bad}


def check_shadow(cfg, n, g):
    K = constants(cfg["bh"], cfg["lo"], cfg["hi"])
    T = cfg["sf"].triangles()
    faces, w = occluders(T, cfg["lo"], cfg["hi"])
    if not any(len(f) for f in faces):
        return {"rays": 0, "proven": 0.0, "worst_dev_over_margin": 0.0, "violations": 0}
    box = trigger_box(K, w)
    area = 0.5 * np.linalg.norm(np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]), axis=1)
    t = g.choice(len(T), n, p=area / area.sum())
    u, v = g.random(n), g.random(n)
    flip = u + v > 1
    u, v = np.where(flip, 1 - u, u), np.where(flip, 1 - v, v)
    hp = T[t, 0] + u[:, None] * (T[t, 1] - T[t, 0]) + v[:, None] * (T[t, 2] - T[t, 0])
    ls = [lv for ty, _, lv in cfg["sf"].lights() if ty in (0, 1)]
    kind = [ty for ty, _, _ in cfg["sf"].lights() if ty in (0, 1)]
    if not ls:
        return {"rays": 0, "proven": 0.0, "worst_dev_over_margin": 0.0, "violations": 0}
    li = g.integers(0, len(ls), n)
    pos = np.array([ls[i][0] for i in li])
    isarea = np.array([kind[i] == 0 for i in li])[:, None]
    dx = np.where(isarea, np.array([ls[i][2] for i in li]), 0.0)
    dy = np.where(isarea, np.array([ls[i][3] for i in li]), 0.0)
    p = pos + (g.random(n) - 0.5)[:, None] * dx + (g.random(n) - 0.5)[:, None] * dy
    wi = p - hp
    wi /= np.linalg.norm(wi, axis=1)[:, None]
    o, d = hp + EPS * wi, wi
    rows, nrow = _chains(cfg["bh"], o, d, K["steps"])
    proven, step, tri, pts, mrg = shadow_run(K, faces, box, o, d)
    worst = 0.0
    for k in range(1, K["steps"] + 1):
        ok = (nrow > k) & np.isfinite(mrg[k])
        if ok.any():
            dev = np.linalg.norm(pts[k][ok] - rows[ok, k, 0:3], axis=1) / mrg[k][ok]
            worst = max(worst, float(dev.max()))
    hit_p, nrm, zero_n = np.zeros(3), np.zeros(3), np.zeros(9)
    bad = 0
    for i in np.nonzero(proven)[0]:
        k = step[i]
        if not (nrow[i] > k and not rows[i, :k + 1, 7].any()):
            bad += 1
            continue
        mt = C.c_double(rows[i, k, 6])
        if O.lib().ro_tri_intersect(T[tri[i]].ravel().copy(), zero_n, rows[i, k, 0:3].copy(), rows[i, k, 3:6].copy(),
                                    C.byref(mt), hit_p, nrm) != 1:
            bad += 1
    return {"rays": n, "proven": float(proven.mean()), "worst_dev_over_margin": worst, "violations": int(bad)}


def sweep(n_cfg, seed, n_cam=600, n_pix=80, n_shadow=600, log=None, dt_range=DT_RANGE, rs_max=RS_OVER_BOX_MAX):
    g = np.random.default_rng(seed)
    res = []
    for i in range(n_cfg):
        cfg = draw_config(g, dt_range=dt_range, rs_max=rs_max)
        r = {"scene": cfg["scene"], "bh": [float(v) for v in cfg["bh"]], "camera_pos": [float(v) for v in cfg["pos"]],
             "hfov": cfg["hfov"], "frame": [cfg["W"], cfg["H"]],
             "box": [float(v) for v in np.concatenate([cfg["lo"], cfg["hi"]])],
             "camera": check_camera(cfg, n_cam, g), "pixel": check_pixel(cfg, n_pix, g),
             "shadow": check_shadow(cfg, n_shadow, g)}
        res.append(r)
        if log:
            log(i, r)
    return res
