"""GPU: the path pool kernel (csrc/rrt_path.hip, RRT_RENDER_WAVEFRONT: an A/B variant for
max_ray_depth >= 2; the per-pixel loop is the default) against the
CPU restatement, bit for bit (RGB, sample counts, RNG draws), on settings the depth >= 2 goldens
do not cover: hemisphere-sampled direct light at depth 3, several light samples a vertex (the
vertex's rays go out one a round), one sample a pixel, the delta BSDFs at depth 5, and a clipped
region.  The goldens themselves run through it in tests/test_gpu_parity.py ("pathpool" variant).
Reference: part1_code.cpp:15-163."""
import numpy as np
import pytest

import oracle_lib as ol
import rrt
from golden_cases import Case

pytestmark = pytest.mark.gpu

# (golden case for scene / camera, setting overrides, region (x0, y0, w, h) or None)
CASES = [
    ("spheres_96x72_s40_m3", {"direct_hemisphere": True, "ns_aa": 16}, None),
    ("bunny_160x120_s16", {"max_ray_depth": 3, "ns_area_light": 4, "ns_aa": 8}, None),
    ("spheres_96x72_s40_m3", {"ns_aa": 1}, None),
    ("glass_mirror_96x72_s16_m4", {"max_ray_depth": 5}, None),
    ("env_spheres_96x72_s16_m2", {"max_ray_depth": 3, "ns_area_light": 2}, None),
    ("spheres_96x72_s40_m3", {}, (13, 7, 50, 41)),
]


@pytest.fixture(scope="module")
def gpu():
    r = rrt.Renderer(device=0)
    yield r
    r.close()


@pytest.mark.parametrize("name,over,region", CASES)
def test_path_kernel_matches_restatement(gpu, name, over, region):
    c = Case(name)
    g = dict(c.cfg)
    g.update(over)
    x0, y0, w, h = region if region else (c.x0, c.y0, c.w, c.h)
    s = ol.Scene(c.scene_path)
    if c.envmap is not None:
        s.set_envmap(c.envmap)
    op = ol.make_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                        ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                        max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], bh=g["bh"])
    ref_rgb, ref_cnt, ref_draws, _ = ol.render(s, ol.load_camera(c.camera_path), op, x0, y0, w, h, threads=16)
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(c.envmap)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    gpu.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
    p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                          ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                          max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"],
                          flags=rrt.RRT_RENDER_WAVEFRONT)
    rgb, cnt, draws, _ = gpu.render(p, x0, y0, w, h, draws=True)
    kernel = gpu.stats().kernel.decode()
    print(name, over, region, kernel, "mean", rgb.mean(axis=(0, 1)))
    assert "rrt_path_kernel" in kernel
    assert float(ref_rgb.max()) > 0
    assert np.array_equal(cnt, ref_cnt)
    assert np.array_equal(draws, ref_draws)
    assert np.array_equal(rgb.view(np.uint32), ref_rgb.view(np.uint32))


def test_path_kernel_waves_budgets_agree(gpu):
    """The 2 / 3 / 4 waves-per-SIMD builds (variant byte) and the per-pixel-loop kernel (the
    depth >= 2 default) give the same frame."""
    c = Case("spheres_96x72_s40_m3")
    g = c.cfg
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(None)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    gpu.set_black_hole(g["bh"][:3], g["bh"][3], g["bh"][4])
    outs = {}
    wf = rrt.RRT_RENDER_WAVEFRONT
    for name, flags, variant in (("loop", 0, 0), ("w2", wf, 2), ("w3", wf, 3), ("w4", wf, 4)):
        p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                              ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                              max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"],
                              flags=flags, variant=variant)
        outs[name] = gpu.render(p, c.x0, c.y0, c.w, c.h, draws=True)
        print(name, gpu.stats().kernel.decode())
    for name in ("w2", "w3", "w4"):
        for a, b in zip(outs["loop"][:3], outs[name][:3]):
            assert np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def test_path_kernel_rejected_where_not_built(gpu):
    """Depth <= 1 has no path pool kernel: the flag fails loudly."""
    c = Case("spheres_96x72_s1")
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(None)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    gpu.set_black_hole((0.0, 1.0, 0.0), 0.1, 0.1)
    p = rrt.render_params(c.frame_w, c.frame_h, max_ray_depth=1, flags=rrt.RRT_RENDER_WAVEFRONT)
    with pytest.raises(rrt.RRTError) as e:
        gpu.render(p, 0, 0, 8, 8)
    assert e.value.code == rrt.RRT_E_INVALID
