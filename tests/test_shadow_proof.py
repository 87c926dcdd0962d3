"""The shadow-ray occlusion proof (rrt_device.h shadow_occluded_proof) against the
CPU restatement of the reference's march (oracle ro_micro_chain / ro_tri_intersect, bit-exact with
blackhole.cpp / bvh.cpp / triangle.cpp), on shadow rays from random surface points of the BASELINE
Cornell-box scenes towards random points of their area lights:

* the host's occluder table (rrt_get_occluders) is the numpy mirror's (tests/shadow_proof_sim.py);
* the recurrence stays within 1e-3 of the proof's margin of the reference's march points;
* every ray the proof calls occluded really is: the reference's chain is not captured up to the
  proof's segment, and the reference's triangle test accepts that segment against the proof's
  triangle -- so the reference's shadow query (first hit before capture) returns true;
* the proof accepts the bulk of such rays.

The GPU parity tests then check whole frames bit-exactly with the proof on (default) and off.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import rrt
from golden_cases import Case
from miss_proof_sim import constants
from shadow_proof_sim import occluders, run, trigger_box

CASES = [("cfg3_bunny_1080p_s64", 0.8), ("cfg4_knot_240x135_s16", 0.7), ("cfg1_spheres_480x360_s8", 0.6),
         ("cfg2_spheres_1080p_s64_flat", 0.6),
         ("spheres_bh_96x72_s8", 0.0)]
N = 3000
EPS = 1e-11


def _shadow_rays(T, lights, n, seed):
    g = np.random.default_rng(seed)
    area = 0.5 * np.linalg.norm(np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]), axis=1)
    t = g.choice(len(T), n, p=area / area.sum())
    u, v = g.random(n), g.random(n)
    flip = u + v > 1
    u, v = np.where(flip, 1 - u, u), np.where(flip, 1 - v, v)
    hp = T[t, 0] + u[:, None] * (T[t, 1] - T[t, 0]) + v[:, None] * (T[t, 2] - T[t, 0])
    # area lights: a uniform point of the rectangle (light.cpp sample_L); point lights: the point
    ls = [lv for ty, _, lv in lights if ty in (0, 1)]
    kind = [ty for ty, _, _ in lights if ty in (0, 1)]
    li = g.integers(0, len(ls), n)
    pos = np.array([ls[i][0] for i in li])
    area = np.array([kind[i] == 0 for i in li])[:, None]
    dx = np.where(area, np.array([ls[i][2] for i in li]), 0.0)
    dy = np.where(area, np.array([ls[i][3] for i in li]), 0.0)
    p = pos + (g.random(n) - 0.5)[:, None] * dx + (g.random(n) - 0.5)[:, None] * dy
    wi = p - hp
    wi /= np.linalg.norm(wi, axis=1)[:, None]
    return hp + EPS * wi, wi


def _setup(name):
    c = Case(name)
    sf = rrt.SceneFile(c.scene_path)
    r = rrt.Renderer(device=-1)
    r.set_scene(sf)
    boxes, _, _ = r.bvh()
    tris_dev, counts = r.occluders()
    r.close()
    lo, hi = boxes[0][:3].copy(), boxes[0][3:].copy()
    return c, sf, lo, hi, tris_dev, counts


@pytest.mark.parametrize("name,_share", CASES)
def test_occluder_table_matches_mirror(name, _share):
    c, sf, lo, hi, tris_dev, counts = _setup(name)
    faces, _ = occluders(sf.triangles(), lo, hi)
    assert [len(f) for f in faces] == counts.tolist()
    for f, tris in enumerate(faces):
        for i, (n, d, en, eo, _) in enumerate(tris):
            ref = np.concatenate([n, [d], en.ravel(), eo])
            np.testing.assert_allclose(tris_dev[f, i], ref, rtol=1e-12, atol=1e-14)
    # a Cornell box: floor, ceiling and at least two walls carry triangles
    assert counts[1] >= 1 and counts[4] >= 1 and (counts > 0).sum() >= 4


@pytest.mark.parametrize("lead", [0, 2])
@pytest.mark.parametrize("name,min_share", CASES)
def test_occluded_rays_really_hit_before_capture(name, min_share, lead):
    """lead: the exact segments the query marches before the proof takes over from the
    reference's state (the start of segment `lead` and the previous segment's direction)."""
    c, sf, lo, hi, _, _ = _setup(name)
    T = sf.triangles()
    faces, w = occluders(T, lo, hi)
    bh = np.array(c.cfg["bh"], np.float64)
    K = constants(bh, lo, hi)
    box = trigger_box(K, w)
    o, d = _shadow_rays(T, sf.lights(), N, 11)
    rows = np.zeros((N, K["steps"] + 1, 8))
    nrow = np.zeros(N, int)
    out = np.zeros((K["steps"] + 1, 8))
    for i in range(N):
        k = O.lib().ro_micro_chain(bh, o[i], d[i], out, K["steps"] + 1)
        rows[i, :k] = out[:k]
        nrow[i] = k
    if lead:  # rays whose first `lead` reference segments neither hit a wall nor were captured
        keep = (nrow > lead) & ~rows[:, :lead, 7].any(1)
        o2, d2 = rows[:, lead, 0:3].copy(), rows[:, lead - 1, 3:6].copy()
        o, d = o2[keep], d2[keep]
        rows, nrow = rows[keep][:, lead:], nrow[keep] - lead
    K = dict(K, steps=K["steps"] - lead)
    proven, step, tri, pts, mrg = run(K, faces, box, o, d)
    # deviation of the recurrence from the reference's points while the proof ran
    worst = 0.0
    for k in range(1, K["steps"] + 1):
        ok = (nrow > k) & np.isfinite(mrg[k])
        if ok.any():
            dev = np.linalg.norm(pts[k][ok] - rows[ok, k, 0:3], axis=1) / mrg[k][ok]
            worst = max(worst, float(dev.max()))
    print(name, lead, "proven share", proven.mean(), "worst deviation / margin", worst)
    assert worst < 1e-3
    # every proven ray: no capture through the proof's segment, and the reference's triangle test
    # accepts that segment against the proof's triangle
    hit_p, nrm = np.zeros(3), np.zeros(3)
    zero_n = np.zeros(9)
    for i in np.nonzero(proven)[0]:
        k = step[i]
        assert nrow[i] > k and not rows[i, :k + 1, 7].any(), (name, i, k)
        mt = C.c_double(rows[i, k, 6])
        assert O.lib().ro_tri_intersect(T[tri[i]].ravel().copy(), zero_n, rows[i, k, 0:3].copy(),
                                        rows[i, k, 3:6].copy(), C.byref(mt), hit_p, nrm) == 1, (name, i, k)
    assert proven.mean() >= min_share
