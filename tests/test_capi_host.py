"""C ABI (include/rrt.h, librrt.so) host-side checks that need no GPU: every declared symbol is
exported, the scene/camera file loaders, the reference BVH build (node-for-node against the
reference's own BVH dump), the multi-GPU tile partition, and error handling."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import rrt
from golden_cases import GOLD, Case

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SCENES = sorted(f[:-5] for f in os.listdir(os.path.join(GOLD, "scenes")) if f.endswith(".rrts"))


def test_exports_match_header():
    hdr = open(os.path.join(ROOT, "include", "rrt.h")).read()
    declared = set(re.findall(r"\b(rrt_[a-z_]+)\s*\(", hdr))
    assert declared == set(rrt.EXPORTS), declared ^ set(rrt.EXPORTS)
    L = rrt.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.rrt_abi_version() == 1


@pytest.fixture(scope="module")
def host_ctx():
    r = rrt.Renderer(device=-1)
    yield r
    r.close()


@pytest.mark.parametrize("scene", SCENES)
def test_bvh_matches_reference(host_ctx, scene):
    sf = rrt.SceneFile(os.path.join(GOLD, "scenes", scene + ".rrts"))
    host_ctx.set_scene(sf)
    boxes, nodes, prims = host_ctx.bvh()
    ref = np.load(os.path.join(GOLD, "scenes", scene + "_bvh.npz"))
    assert np.array_equal(boxes.view(np.uint64), ref["boxes"].view(np.uint64))
    assert np.array_equal(nodes, ref["nodes"])
    assert np.array_equal(prims, ref["prims"])
    s = host_ctx.stats()
    assert s.n_nodes == len(ref["nodes"]) and s.n_leaf_refs == len(ref["prims"])


def test_bunny_bvh_shape(host_ctx):
    host_ctx.set_scene(rrt.SceneFile(os.path.join(GOLD, "scenes", "CBbunny.rrts")))
    s = host_ctx.stats()
    # CBbunny 28,588 prims, 19,103 nodes, max depth 19
    assert (s.n_prims, s.n_nodes, s.max_depth) == (28588, 19103, 19)


def test_camera_loader_matches_reference_record():
    c = Case("cfg3_bunny_1080p_s64")
    cam = rrt.load_camera(c.camera_path)
    raw = np.fromfile(c.camera_path, dtype="<f8", offset=8)
    assert cam.hFov == raw[0] and cam.vFov == raw[1] and cam.nClip == raw[3] and cam.fClip == raw[4]
    assert list(cam.pos) == list(raw[5:8]) and list(cam.c2w) == list(raw[16:25])
    # SURVEY Appendix C known values for CBbunny @ 1920x1080
    assert cam.hFov == 95.304258666083385 and cam.vFov == 63.361022388069181


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_covers_frame_once(world):
    W, H, ts = 1920, 1080, 32
    seen = {}
    for r in range(world):
        for x, y in rrt.partition_tiles(W, H, ts, r, world):
            assert (x, y) not in seen
            seen[(int(x), int(y))] = r
    assert len(seen) == ((W + ts - 1) // ts) * ((H + ts - 1) // ts)
    sizes = [sum(1 for v in seen.values() if v == r) for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def test_partition_load_balance_cfg3():
    """Block-cyclic tiles balance the spatially concentrated cfg3 work:
    per-rank sum of reference work (samples) within a few % of the mean at 8 ranks."""
    c = Case("cfg3_bunny_1080p_s64")
    work = c.px["count"].astype(np.int64) + 64 * (c.px["rgb"].sum(-1) > 0)
    tot = []
    for r in range(8):
        t = 0
        for x, y in rrt.partition_tiles(1920, 1080, 32, r, 8):
            t += work[y:y + 32, x:x + 32].sum()
        tot.append(t)
    assert max(tot) / np.mean(tot) < 1.05


def test_errors(host_ctx):
    with pytest.raises(rrt.RRTError) as e:
        host_ctx.render(rrt.render_params(8, 8), 0, 0, 8, 8)
    assert e.value.code in (rrt.RRT_E_INVALID, rrt.RRT_E_NO_DEVICE)
    assert rrt.lib().rrt_partition_tiles(64, 64, 32, 2, 2, None, 0) == rrt.RRT_E_INVALID
    with pytest.raises(rrt.RRTError):
        rrt.SceneFile("/nonexistent.rrts")
    st = rrt.SpacetimeDesc()
    st.delta_theta = 0.0
    assert rrt.lib().rrt_set_spacetime(host_ctx.h, C.byref(st)) == rrt.RRT_E_INVALID
