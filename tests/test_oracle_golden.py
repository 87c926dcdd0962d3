"""The CPU restatement against the reference's per-pixel outputs (tests/golden/<case>/px.npz,
rendered by the compiled reference under the same keyed RNG).  Bit-exact: RGB, sample counts,
RNG draw counts and the reference's own work counters (AABB tests, micro steps)."""
import os

import numpy as np
import pytest

import oracle_lib as O
from golden_cases import SMALL, Case


def render_case(c, rows=None, counters=True):
    s = O.Scene(c.scene_path)
    if c.envmap is not None:
        s.set_envmap(c.envmap)
    cam = O.load_camera(c.camera_path)
    g = c.cfg
    p = O.make_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                      ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                      max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], bh=g["bh"])
    y0, h = (c.y0, c.h) if rows is None else (c.y0 + rows[0], rows[1] - rows[0])
    return O.render(s, cam, p, c.x0, y0, c.w, h, counters=counters)


@pytest.mark.parametrize("name", SMALL)
def test_case_bit_exact(name):
    c = Case(name)
    rgb, cnt, draws, ctr = render_case(c)
    px = c.px
    assert np.array_equal(rgb.view(np.uint32), px["rgb"].view(np.uint32)), name
    assert np.array_equal(cnt, px["count"])
    assert np.array_equal(draws, px["draws"])
    if "bbox_tests" in px:
        assert np.array_equal(ctr[..., 0], px["bbox_tests"])
        assert np.array_equal(ctr[..., 1], px["micro_steps"])
    if "prim_tests_total" in c.info and name == "spheres_96x72_s40_m3":
        # recorded with -t 1, where the reference's (racy) total_isects counter is exact
        assert int(ctr[..., 2].astype(np.int64).sum()) == c.info["prim_tests_total"]


@pytest.mark.parametrize("name,rows", [("cfg3_bunny_1080p_s64", (368, 380)),
                                       ("cfg2_spheres_1080p_s64_flat", (672, 684))])
def test_baseline_frames_band(name, rows):
    """A band of rows through the middle of the 1080p BASELINE frames (the full frames are
    checked by test_baseline_frames_full, marked slow)."""
    c = Case(name)
    rgb, cnt, draws, _ = render_case(c, rows=rows, counters=False)
    px = c.px
    sl = slice(rows[0], rows[1])
    assert np.array_equal(rgb.view(np.uint32), px["rgb"][sl].view(np.uint32))
    assert np.array_equal(cnt, px["count"][sl])
    assert np.array_equal(draws, px["draws"][sl])
    assert (rgb.sum(-1) > 0).any()


@pytest.mark.slow
@pytest.mark.parametrize("name", ["cfg1_spheres_480x360_s8", "cfg2_spheres_1080p_s64_flat", "cfg3_bunny_1080p_s64"])
def test_baseline_frames_full(name):
    c = Case(name)
    rgb, cnt, draws, _ = render_case(c, counters=False)
    assert np.array_equal(rgb.view(np.uint32), c.px["rgb"].view(np.uint32))
    assert np.array_equal(cnt, c.px["count"])
