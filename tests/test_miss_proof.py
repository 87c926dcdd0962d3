"""The camera-ray miss proof (rrt_device.h camera_miss_proof) against the CPU
restatement of the reference's march (oracle ro_micro_chain, bit-exact with blackhole.cpp /
bvh.cpp): on random jittered camera rays of every BASELINE framing,

* the planar recurrence stays within 1e-3 of the proof's margin of the reference's march points
  (the margin is 1e3 x the deviation the proof assumes), up to the reference's capture;
* every ray the proof accepts really misses: each of its reference segments fails the
  reference's root-box test (bbox.cpp:10-25);
* the proof accepts the bulk of the rays where most of the frame is empty (cfg2/3/4).

The GPU parity tests then check whole frames bit-exactly with the proof on (the default) and off.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import rrt
from golden_cases import Case
from miss_proof_sim import constants, run

CASES = [("cfg1_spheres_480x360_s8", 0.0), ("cfg2_spheres_1080p_s64_flat", 0.85),
         ("cfg3_bunny_1080p_s64", 0.85), ("cfg4_knot_4k_s256_crop", 0.9)]
N = 6000


def _rays(c, n, seed):
    cam = O.load_camera(c.camera_path)
    cols = np.array(cam.c2w, np.float64).reshape(3, 3).T.ravel().copy()
    pos = np.array(cam.pos, np.float64)
    g = np.random.default_rng(seed)
    xs = (g.integers(0, c.frame_w, n) + g.random(n)) / c.frame_w
    ys = (g.integers(0, c.frame_h, n) + g.random(n)) / c.frame_h
    o = np.zeros((n, 3))
    d = np.zeros((n, 3))
    mn, mx = C.c_double(), C.c_double()
    for i in range(n):
        O.lib().ro_camera_ray(cam.hFov, cam.vFov, pos, cols, cam.nClip, cam.fClip, xs[i], ys[i], o[i], d[i],
                              C.byref(mn), C.byref(mx))
    return o, d


@pytest.mark.parametrize("name,min_share", CASES)
def test_recurrence_tracks_reference_and_proven_rays_miss(name, min_share):
    c = Case(name)
    bh = c.cfg["bh"]
    r = rrt.Renderer(device=-1)
    r.set_scene(rrt.SceneFile(c.scene_path))
    boxes, _, _ = r.bvh()
    r.close()
    lo, hi = boxes[0][:3].copy(), boxes[0][3:].copy()
    K = constants(bh, lo, hi)
    o, d = _rays(c, N, 7)
    bha = np.array(bh, np.float64)
    rows = np.zeros((N, K["steps"] + 1, 8))
    nrow = np.zeros(N, int)
    out = np.zeros((64, 8))
    for i in range(N):
        k = O.lib().ro_micro_chain(bha, o[i], d[i], out, 64)
        rows[i, :k] = out[:k]
        nrow[i] = k
    t0, t1 = C.c_double(), C.c_double()

    def root_hit(i, k):
        rw = rows[i, k]
        return O.lib().ro_bbox_intersect(lo, hi, rw[0:3].copy(), rw[3:6].copy(), 0.0, rw[6], C.byref(t0),
                                         C.byref(t1)) != 0

    step0_clear = np.array([not root_hit(i, 0) for i in range(N)])
    proven, pts, mrg = run(K, o, d, step0_clear)
    # deviation of the recurrence from the reference, wherever the proof was still running
    worst = 0.0
    for k in range(2, K["steps"] + 1):
        ref = np.where((nrow > k)[:, None], rows[:, min(k, K["steps"]), 0:3], np.nan)
        last = nrow == k  # the end point of the final (pre-capture) segment
        endp = rows[np.arange(N), np.maximum(nrow - 1, 0)]
        ref = np.where(last[:, None], endp[:, 0:3] + endp[:, 3:6] * endp[:, 6:7], ref)
        dev = np.linalg.norm(pts[k] - ref, axis=1) / mrg[k]
        ok = np.isfinite(dev)
        if ok.any():
            worst = max(worst, float(dev[ok].max()))
    print(name, "proven share", proven.mean(), "worst deviation / margin", worst)
    assert worst < 1e-3
    # accepted rays really miss: no pre-capture reference segment passes the root test
    for i in np.nonzero(proven)[0]:
        for k in range(nrow[i]):
            assert not root_hit(i, k), (name, i, k)
    assert proven.mean() >= min_share
