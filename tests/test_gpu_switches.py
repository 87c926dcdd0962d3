"""GPU: the reference's compile-time switches as run-time flags (include/rrt.h RRT_RENDER_THIN_LENS,
RRT_RENDER_NO_ADAPTIVE, RRT_RENDER_ENV_HEMI, RRT_RENDER_MICROFACET_HEMI, RRT_RENDER_ILLUM; the V_SW
kernel build) against the CPU restatement with the same switches, bit for bit (RGB, sample counts,
RNG draws).  Parity against the reference is unpinned for non-default switch values (see
tests/test_switches_oracle.py); the default values are the reference build and are pinned by every
golden."""
import numpy as np
import pytest

import oracle_lib as ol
import rrt
from golden_cases import Case

pytestmark = pytest.mark.gpu

# (golden case for scene / camera / settings, overrides, oracle switches, GPU flags)
CASES = [
    ("spheres_96x72_s64_a16", {}, dict(adaptive=False), rrt.RRT_RENDER_NO_ADAPTIVE),
    ("spheres_96x72_s1", {}, dict(illum=0), rrt.RRT_RENDER_ILLUM(0)),
    # (CBspheres' shadow rays all end on the light's own emitter mesh -- the reference drops the
    # shadow ray's max_t -- so its direct light is zero: ILLUM 1 / 3 run on the lit bunny)
    ("bunny_160x120_s16", {}, dict(illum=1), rrt.RRT_RENDER_ILLUM(1)),
    ("bunny_160x120_s16", {"max_ray_depth": 3}, dict(illum=3), rrt.RRT_RENDER_ILLUM(3)),
    ("spheres_96x72_s8_l4", {"max_ray_depth": 2}, dict(illum=3), rrt.RRT_RENDER_ILLUM(3)),
    ("spheres_96x72_s8_l4", {"max_ray_depth": 1}, dict(illum=3), rrt.RRT_RENDER_ILLUM(3)),
    ("spheres_96x72_s8_l4", {}, dict(thin_lens=True), rrt.RRT_RENDER_THIN_LENS),
    ("bunny_160x120_s16", {}, dict(thin_lens=True, adaptive=False), rrt.RRT_RENDER_THIN_LENS | rrt.RRT_RENDER_NO_ADAPTIVE),
    ("env_spheres_96x72_s32_l2", {}, dict(env_hemi=True), rrt.RRT_RENDER_ENV_HEMI),
    ("env_spheres_96x72_s16_m2", {}, dict(env_hemi=True, illum=3), rrt.RRT_RENDER_ENV_HEMI | rrt.RRT_RENDER_ILLUM(3)),
    ("bunnycu_96x72_s8_m2", {}, dict(microfacet_hemi=True), rrt.RRT_RENDER_MICROFACET_HEMI),
    ("spheres_96x72_s8_hemi", {}, dict(illum=1, adaptive=False), rrt.RRT_RENDER_ILLUM(1) | rrt.RRT_RENDER_NO_ADAPTIVE),
]


@pytest.fixture(scope="module")
def gpu():
    r = rrt.Renderer(device=0)
    yield r
    r.close()


def settings(c, over):
    g = dict(c.cfg)
    g.update(over)
    return g


@pytest.mark.parametrize("name,over,osw,flags", CASES)
def test_switch_matches_restatement(gpu, name, over, osw, flags):
    c = Case(name)
    g = settings(c, over)
    s = ol.Scene(c.scene_path)
    if c.envmap is not None:
        s.set_envmap(c.envmap)
    op = ol.make_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                        ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                        max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], bh=g["bh"], **osw)
    ref_rgb, ref_cnt, ref_draws, _ = ol.render(s, ol.load_camera(c.camera_path), op, c.x0, c.y0, c.w, c.h, threads=16)
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(c.envmap)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    gpu.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
    p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                          ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                          max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=flags)
    rgb, cnt, draws, _ = gpu.render(p, c.x0, c.y0, c.w, c.h, draws=True)
    print(name, osw, "kernel", gpu.stats().kernel.decode(), "mean", rgb.mean(axis=(0, 1)))
    assert float(ref_rgb.max()) > 0
    assert "rrt_render_kernel<true, false, 4" in gpu.stats().kernel.decode()
    assert np.array_equal(rgb.view(np.uint32), ref_rgb.view(np.uint32))
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(draws, ref_draws)


def test_switches_rejected_where_not_built(gpu):
    """Kerr has no switch build, and ILLUM 3 at depth 0 is rejected: the reference's recursion depth is
    unbounded there (size_t Ray::depth wraps; only Russian roulette ends it), beyond RRT_MAX_DEPTH."""
    c = Case("spheres_96x72_s1")
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(None)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    gpu.set_black_hole((0.0, 1.0, 0.0), 0.1, 0.1, spin=0.5)
    p = rrt.render_params(c.frame_w, c.frame_h, flags=rrt.RRT_RENDER_NO_ADAPTIVE)
    with pytest.raises(rrt.RRTError) as e:
        gpu.render(p, 0, 0, 8, 8)
    assert e.value.code == rrt.RRT_E_INVALID
    gpu.set_black_hole((0.0, 1.0, 0.0), 0.1, 0.1)
    p = rrt.render_params(c.frame_w, c.frame_h, max_ray_depth=0, flags=rrt.RRT_RENDER_ILLUM(3))
    with pytest.raises(rrt.RRTError) as e:
        gpu.render(p, 0, 0, 8, 8)
    assert e.value.code == rrt.RRT_E_INVALID
