"""The proofs' validated envelope (include/rrt.h RRT_PROOF_*): the library enables the
camera-ray, pixel and shadow-ray proofs only for Schwarzschild holes with delta_theta in
[RRT_PROOF_DT_MIN, RRT_PROOF_DT_MAX] and r_s <= RRT_PROOF_RS_OVER_EXTENT x the room's largest
extent -- the ranges tools/proof_sweep.py validated (profiles/r03_proof_sweep.json) -- and a small
random sweep inside it finds the proofs sound against the reference's march."""
import os
import re

import numpy as np
import pytest

import proof_sweep as P
import rrt

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLD = os.path.join(ROOT, "tests", "golden")


def _header_constants():
    src = open(os.path.join(ROOT, "include", "rrt.h")).read()
    return {k: float(re.search(rf"#define RRT_PROOF_{k} ([0-9.]+)", src).group(1))
            for k in ("DT_MIN", "DT_MAX", "RS_OVER_EXTENT")}


def test_sweep_ranges_are_the_library_envelope():
    h = _header_constants()
    assert P.DT_RANGE == (h["DT_MIN"], h["DT_MAX"])
    assert P.RS_OVER_BOX_MAX == h["RS_OVER_EXTENT"]


@pytest.mark.parametrize("bh,inside", [
    (((0.0, 1.0, 0.0), 0.1, 0.1), True),     # the reference's default hole (BASELINE configs)
    (((0.0, 1.0, 0.0), 0.0, 0.1), True),     # cfg2's flat limit
    (((0.3, 1.2, -0.2), 0.25, 0.05), True),  # golden bunny_B1
    (((0.0, 1.0, 0.0), 0.1, 0.02), False),   # finer steps than validated
    (((0.0, 1.0, 0.0), 0.1, 0.9), False),    # coarser steps than validated
    (((0.0, 1.0, 0.0), 1.5, 0.1), False),    # a hole larger than half the room
])
def test_library_envelope(bh, inside):
    r = rrt.Renderer(device=-1)
    r.set_scene(rrt.SceneFile(os.path.join(GOLD, "scenes", "CBbunny.rrts")))
    r.set_black_hole(*bh)
    assert r.proof_envelope() == inside
    if bh[1] > 0:
        r.set_black_hole(*bh, spin=0.5, axis=(0.0, 1.0, 0.0))  # Kerr: never
        assert not r.proof_envelope()
    r.close()


def test_small_sweep_inside_the_envelope():
    res = P.sweep(6, 77, n_cam=200, n_pix=30, n_shadow=200)
    for r in res:
        for k in ("camera", "pixel", "shadow"):
            assert r[k]["violations"] == 0, (r["scene"], r["bh"], k, r[k])
        assert r["camera"]["worst_dev_over_margin"] < 1e-3, r
        assert r["shadow"]["worst_dev_over_margin"] < 1e-3, r
    assert np.mean([r["camera"]["proven"] for r in res]) > 0.05
