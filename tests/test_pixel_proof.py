"""The pixel miss proof (rrt_device.h pixel_miss_proof) against the CPU restatement
of the reference's march (oracle ro_camera_ray / ro_micro_chain, bit-exact with
part1_code.cpp:182-187 and blackhole.cpp / bvh.cpp): on random pixels of the BASELINE framings,

* every ray of a proven pixel -- its four corners and random jitters -- misses: none of its
  reference segments before the capture reaches the root box (a loose slab test, so a proven
  segment must clear it by more than rounding);
* the proof accepts most pixels where the frame is empty.

The GPU parity tests then check whole frames bit-exactly with the pass on (default) and off.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import rrt
from golden_cases import Case
from miss_proof_sim import constants
from pixel_proof_sim import prove

CASES = [("cfg1_spheres_480x360_s8", 0.0), ("cfg2_spheres_1080p_s64_flat", 0.6), ("cfg3_bunny_1080p_s64", 0.6),
         ("cfg4_knot_4k_s256_crop", 0.8)]
N_PIX = 600
N_JIT = 6


def _loose_root_hit(lo, hi, rows):
    """Segments rows [k, 8] (o, d, max_t) whose slab test against [lo, hi] passes or nearly does."""
    o, d, mt = rows[:, 0:3], rows[:, 3:6], rows[:, 6]
    with np.errstate(all="ignore"):
        t0 = (lo[None] - o) / d
        t1 = (hi[None] - o) / d
    tmin = np.nanmax(np.minimum(t0, t1), axis=1)
    tmax = np.nanmin(np.maximum(t0, t1), axis=1)
    tol = 1e-9 * (1.0 + np.abs(tmin) + np.abs(tmax))
    return (tmin <= tmax + tol) & (tmax >= -tol) & (tmin <= mt + tol)


@pytest.mark.parametrize("name,min_share", CASES)
def test_proven_pixels_miss(name, min_share):
    c = Case(name)
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

    def ray(sx, sy):
        o, d = np.zeros(3), np.zeros(3)
        O.lib().ro_camera_ray(cam.hFov, cam.vFov, pos, cols, cam.nClip, cam.fClip, sx / W, sy / H, o, d,
                              C.byref(mn), C.byref(mx))
        return o, d

    g = np.random.default_rng(5)
    pxs = g.integers(0, W, N_PIX)
    pys = g.integers(0, H, N_PIX)
    out = np.zeros((K["steps"] + 1, 8))
    proven = 0
    for px, py in zip(pxs, pys):
        o, dc = ray(px + 0.5, py + 0.5)
        corners = np.array([ray(px + (k & 1), py + (k >> 1))[1] for k in range(4)])
        if not prove(K, o, dc, corners):
            continue
        proven += 1
        jit = [(float(k & 1), float(k >> 1)) for k in range(4)] + [tuple(g.random(2)) for _ in range(N_JIT)]
        for jx, jy in jit:
            o2, d2 = ray(px + jx, py + jy)
            k = O.lib().ro_micro_chain(bh, o2, d2, out, K["steps"] + 1)
            assert not _loose_root_hit(lo, hi, out[:k]).any(), (name, px, py, jx, jy)
    print(name, "proven pixels", proven / N_PIX)
    assert proven / N_PIX >= min_share


@pytest.mark.parametrize("name,w,h,min_share", [("cfg3_bunny_1080p_s64", 8, 8, 0.3), ("cfg4_knot_4k_s256_crop", 8, 8, 0.6),
                                                ("cfg2_spheres_1080p_s64_flat", 8, 8, 0.0), ("cfg3_bunny_1080p_s64", 32, 2, 0.1)])
def test_proven_strips_miss(name, w, h, min_share):
    """The pass's strip level (rrt_strip_proof_kernel: rect_miss_proof on a w x h rectangle of
    pixels; the strips of 64 claim indices are 8 x 8, 32 x 2 with row-major claims): every pixel of a proven strip -- its corners and a
    random jitter each -- misses.  A wide strip proves less than its pixels do (its rays' v cross
    zero at different steps), so the per-pixel level stays behind it."""
    c = Case(name)
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

    def ray(sx, sy):
        o, d = np.zeros(3), np.zeros(3)
        O.lib().ro_camera_ray(cam.hFov, cam.vFov, pos, cols, cam.nClip, cam.fClip, sx / W, sy / H, o, d,
                              C.byref(mn), C.byref(mx))
        return o, d

    g = np.random.default_rng(9)
    out = np.zeros((K["steps"] + 1, 8))
    n_strips, proven, px_proven = 60, 0, 0
    for _ in range(n_strips):
        x0 = int(g.integers(0, W - w + 1)) // w * w
        y0 = int(g.integers(0, H - h + 1)) // h * h
        o, dc = ray(x0 + 0.5 * w, y0 + 0.5 * h)
        corners = np.array([ray(x0 + (k & 1) * w, y0 + (k >> 1) * h)[1] for k in range(4)])
        pix = [(x0 + i, y0 + j) for j in range(h) for i in range(w)]
        px_ok = sum(prove(K, o, ray(px + 0.5, py + 0.5)[1],
                          np.array([ray(px + (k & 1), py + (k >> 1))[1] for k in range(4)])) for px, py in pix[::7])
        px_proven += px_ok
        if not prove(K, o, dc, corners):
            continue
        proven += 1
        for px, py in pix:
            for jx, jy in [(0.0, 0.0), (1.0, 1.0), tuple(g.random(2))]:
                o2, d2 = ray(px + jx, py + jy)
                k = O.lib().ro_micro_chain(bh, o2, d2, out, K["steps"] + 1)
                assert not _loose_root_hit(lo, hi, out[:k]).any(), (name, px, py, jx, jy)
    per_px = px_proven / (n_strips * len(range(0, w * h, 7)))
    print(name, w, h, "proven strips", proven / n_strips, "pixel level (every 7th pixel)", per_px)
    assert proven / n_strips >= min_share
