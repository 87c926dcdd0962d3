"""The run-time proof audit (include/rrt.h rrt_set_proof_audit).

The renderer skips marches whose results its proofs determine -- the camera-ray miss proof, the
shadow-ray occlusion proof, the pixel pass's pixel and strip proofs, the Kerr occlusion proof --
with margins validated by sweeps.  A counting launch with the audit set re-marches proven rays
exactly: here every one of them (every_log2 = 0) on frames whose proofs all fire, and no proof may
be contradicted.  The audit must not change the frame."""
import numpy as np
import pytest

import rrt
from golden_cases import Case

pytestmark = pytest.mark.gpu
COUNT_X = rrt.RRT_RENDER_COUNTERS | rrt.RRT_RENDER_COUNT_EXECUTED


@pytest.fixture(scope="module")
def gpu():
    r = rrt.Renderer(device=0)
    yield r
    r.close()


def _setup(gpu, c, spin=None, axis=(0.0, 1.0, 0.0), bh=None):
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(c.envmap)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    b = bh or c.cfg["bh"]
    gpu.set_black_hole(b[:3], b[3], b[4], spin=spin, axis=axis)


def _params(c, flags):
    g = c.cfg
    return rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                             ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                             max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=flags)


# (case, region, whether the region holds proven camera rays / pixels: the small frames' narrow
# fields of view see only the room, so there the shadow proof is what runs)
AUDIT_CASES = [("cfg3_bunny_1080p_s64", (832, 412, 256, 256), False), ("cfg3_bunny_1080p_s64", (0, 0, 192, 192), True),
               ("cfg2_spheres_1080p_s64_flat", (1600, 800, 128, 128), True), ("bunny_160x120_s16", None, False),
               ("bunny_B1_160x120_s16", None, False), ("spheres_B2_160x120_s16", None, False)]
# (the point-light scenes -- cfg4's knot -- and the empty room carry no occluder for the shadow
# proof, and their small frames see no misses: nothing to audit there)


@pytest.mark.parametrize("name,region,misses", AUDIT_CASES)
def test_audit_schwarzschild_proofs(gpu, name, region, misses):
    c = Case(name)
    _setup(gpu, c)
    p = _params(c, COUNT_X)
    x0, y0, w, h = region or (0, 0, c.frame_w, c.frame_h)
    gpu.set_proof_audit(-1)
    a0 = gpu.render(p, x0, y0, w, h, counters=True)
    gpu.set_proof_audit(0)   # every proven ray and pixel
    a1 = gpu.render(p, x0, y0, w, h, counters=True)
    gpu.set_proof_audit(-1)
    t = gpu.proof_audit()
    print(name, region, t)
    assert np.array_equal(a0[0].view(np.uint32), a1[0].view(np.uint32)) and np.array_equal(a0[1], a1[1])
    ref = c.px["rgb"][y0 - c.y0:y0 - c.y0 + h, x0 - c.x0:x0 - c.x0 + w]
    assert np.array_equal(a0[0].view(np.uint32), ref.view(np.uint32))  # the reference's frame
    if misses:
        assert t["camera"]["checked"] > 0 and t["pixel"]["checked"] > 0 and t["strip"]["checked"] > 0, t
    assert t["zero"]["checked"] == 0, t  # reserved kind: no zero-sample proof in the product
    assert sum(v["checked"] for v in t.values()) > 0, t
    assert all(v["violations"] == 0 for v in t.values()), t


def test_audit_kerr_proof(gpu):
    c = Case("bunny_160x120_s16")
    _setup(gpu, c, spin=0.9)
    gpu.set_proof_audit(0)
    gpu.render(_params(c, COUNT_X), 0, 0, c.frame_w, c.frame_h, counters=True)
    gpu.set_proof_audit(-1)
    t = gpu.proof_audit()
    print(t)
    assert t["kerr"]["checked"] > 0 and t["kerr"]["violations"] == 0, t
    assert t["camera"]["checked"] == 0  # Kerr has no camera proof


def test_audit_off_outside_counting(gpu):
    """Only counting launches audit: a plain render leaves the tallies at zero."""
    c = Case("bunny_160x120_s16")
    _setup(gpu, c)
    gpu.set_proof_audit(0)
    gpu.render(_params(c, 0), 0, 0, c.frame_w, c.frame_h)
    gpu.set_proof_audit(-1)
    t = gpu.proof_audit()
    assert all(v["checked"] == 0 for v in t.values()), t
