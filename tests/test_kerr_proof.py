"""The Kerr shadow-ray occlusion proof (rrt_device.h kerr_occluded_proof) on the CPU
restatement's marches (tests/kerr_proof_sim.py mirrors the device proof on ro_kerr_chain_st):

* the host's Kerr envelope constants are the mirror's;
* every ray the proof calls occluded is occluded by the restatement's exact query, and the exact
  march's chords stay within a third of the margin delta of the coarse chords (a small sweep of the
  envelope; tools/kerr_proof_sweep.py runs the full one -> profiles/r04_kerr_proof_sweep.json);
* on the cfg5 hole (a/M 0.9, r_s 0.1, delta_theta 0.1) the proof takes the bulk of the shadow rays
  that end on a wall.

The GPU parity tests (tests/test_gpu_kerr.py) then check the cfg5 framing bit-exactly with the
proof on (default) and off ("noproof").
"""
import os
import sys

import numpy as np

import oracle_lib as O
import rrt
from golden_cases import Case
from kerr_proof_sim import constants, deviation, quads, run
from shadow_proof_sim import occluders

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
from kerr_proof_sweep import shadow_rays, sweep  # noqa: E402


def _hdr(name):
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "..", "relativistic-ray-tracer_amd", "csrc", "rrt_host.cpp")) as f:
        src = f.read()
    for line in src.splitlines():
        if line.startswith("#define " + name + " "):
            return float(line.split()[2])
    raise KeyError(name)


def test_envelope_constants_match_the_library():
    import kerr_proof_sim as K
    assert K.STRETCH == _hdr("RRT_KPROOF_STRETCH") and K.NEAR_M == _hdr("RRT_KPROOF_NEAR_M")
    assert K.DELTA_M == _hdr("RRT_KPROOF_DELTA_M") and K.DT_MIN == _hdr("RRT_KPROOF_DT_MIN")
    assert K.DT_MAX == _hdr("RRT_KPROOF_DT_MAX") and K.SPIN_MAX == _hdr("RRT_KPROOF_SPIN_MAX")
    assert K.REACH_M == _hdr("RRT_KPROOF_REACH_M")
    assert K.CENTRE_LO == _hdr("RRT_KPROOF_CENTRE_LO") and K.CENTRE_HI == _hdr("RRT_KPROOF_CENTRE_HI")
    assert K.RS_LO == _hdr("RRT_KPROOF_RS_LO") and K.RS_HI == _hdr("RRT_KPROOF_RS_HI")


def test_envelope_excludes_unswept_holes():
    """Holes outside the swept region (centre near a wall or outside the room, r_s outside the swept
    range) get no proof."""
    lo, hi, w = np.array([-1.0, 0.0, -1.0]), np.array([1.0, 1.5, 1.0]), np.zeros(6)
    assert constants((0.0, 1.0, 0.0, 0.1, 0.1), lo, hi, w)["in_envelope"]
    assert not constants((0.0, 1.45, 0.0, 0.1, 0.1), lo, hi, w)["in_envelope"]   # near the ceiling
    assert not constants((0.0, 1.0, 3.0, 0.1, 0.1), lo, hi, w)["in_envelope"]    # outside the room
    assert not constants((0.0, 1.0, 0.0, 0.05, 0.1), lo, hi, w)["in_envelope"]   # r_s below the sweep's
    assert not constants((0.0, 1.0, 0.0, 0.4, 0.1), lo, hi, w)["in_envelope"]    # and above


def test_small_envelope_sweep_sound():
    recs = sweep(4, 60, seed=17)
    assert sum(r["proven"] for r in recs) > 0
    assert sum(r["violations"] for r in recs) == 0
    assert max(r["worst_deviation_over_delta"] for r in recs) < 1 / 3


def test_cfg5_hole_proves_most_wall_rays():
    c = Case("cfg3_bunny_1080p_s64")  # CBbunny, cfg5's scene
    lsf = rrt.SceneFile(c.scene_path)
    r = rrt.Renderer(device=-1)
    r.set_scene(lsf)
    boxes, _, _ = r.bvh()
    r.close()
    lo, hi = boxes[0][:3].copy(), boxes[0][3:].copy()
    T = lsf.triangles()
    faces, w = occluders(T, lo, hi)
    pieces = quads(T, faces, lo, hi)
    assert [len(p) for p in pieces] == [1, 1, 0, 1, 2, 1]  # walls as quads, the light apart; z- open
    bh, spin, axis = (0.0, 1.0, 0.0, 0.1, 0.1), 0.9, (0.0, 1.0, 0.0)
    K = constants(bh, lo, hi, w)
    assert K["in_envelope"]
    sf = O.Scene(c.scene_path)
    p = O.make_params(64, 64, bh=bh, kerr=(spin, axis))
    o, d = shadow_rays(T, 200, np.random.default_rng(3))
    occ = proven = 0
    for i in range(len(o)):
        hit = O.shadow_query(sf, p, o[i], d[i])
        ok, _, extra = run(K, pieces, bh, spin, axis, o[i], d[i])
        occ += hit
        if ok:
            proven += 1
            assert hit, i
            assert deviation(bh, spin, axis, o[i], d[i], extra) < K["delta"] / 3
    print("occluded", occ, "proven", proven)
    assert proven >= 0.6 * occ
