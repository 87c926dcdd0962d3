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
    declared = set(re.findall(r"\b(rrt_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(rrt.EXPORTS), declared ^ set(rrt.EXPORTS)
    L = rrt.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.rrt_abi_version() == 5


def test_proof_audit_needs_a_device():
    """rrt_set_proof_audit: a host-only context cannot audit (no renders); off (< 0) is always
    accepted; the tallies of a context that never audited are zero."""
    r = rrt.Renderer(device=-1)
    with pytest.raises(rrt.RRTError) as e:
        r.set_proof_audit(10)
    assert e.value.code == rrt.RRT_E_NO_DEVICE
    with pytest.raises(rrt.RRTError) as e:
        r.set_proof_audit(31)
    assert e.value.code == rrt.RRT_E_INVALID
    r.set_proof_audit(-1)
    assert all(v == {"checked": 0, "violations": 0} for v in r.proof_audit().values())
    r.close()


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
    # the lattice deal: every row dealt cyclically (shares differ by one a row), every `world`
    # consecutive rows give each rank the same share, so the leftover rows bound the difference
    assert max(sizes) - min(sizes) <= max(1, (H + ts - 1) // ts % world)


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


class _SceneDescHead(C.Structure):  # include/rrt.h rrt_scene_desc
    _fields_ = [("n_objects", C.c_uint32), ("n_bsdfs", C.c_uint32), ("n_lights", C.c_uint32),
                ("reserved", C.c_uint32), ("objects", C.c_void_p), ("bsdfs", C.c_void_p), ("lights", C.c_void_p)]


def _bad_scene_after_good(ctx):
    """Load a valid scene, then a desc whose objects name BSDFs that do not exist: the second
    rrt_set_scene must fail and leave the context with NO scene (not the first one's device
    buffers paired with the emptied host tables)."""
    sf = rrt.SceneFile(os.path.join(GOLD, "scenes", "CBspheres_lambertian.rrts"))
    ctx.set_scene(sf)
    good = _SceneDescHead.from_address(sf.desc())
    bad = _SceneDescHead(good.n_objects, 0, good.n_lights, 0, good.objects, None, good.lights)
    assert rrt.lib().rrt_set_scene(ctx.h, C.byref(bad)) == rrt.RRT_E_INVALID
    return sf


def test_failed_set_scene_leaves_no_scene():
    r = rrt.Renderer(device=-1)
    try:
        _bad_scene_after_good(r)
        assert rrt.lib().rrt_get_bvh(r.h, None, None, None) == rrt.RRT_E_INVALID
        assert rrt.lib().rrt_get_clean_tree(r.h, None, None, None, None) == rrt.RRT_E_INVALID
    finally:
        r.close()


@pytest.mark.parametrize("kind,r_s,spin,ok", [(1, 0.1, 0.0, True), (1, 0.1, 0.999, True), (1, 0.1, 1.0, False),
                                              (1, 0.1, -0.1, False), (1, 0.0, 0.5, False), (2, 0.1, 0.5, False),
                                              (0, 0.1, 7.0, True)])
def test_spacetime_validation(host_ctx, kind, r_s, spin, ok):
    """Kerr needs r_s > 0 and spin a/M in [0, 1); unknown metric kinds are rejected; the spin is
    ignored for Schwarzschild."""
    st = rrt.SpacetimeDesc()
    st.kind, st.r_s, st.delta_theta, st.spin = kind, r_s, 0.1, spin
    st.center[1] = 1.0
    rc = rrt.lib().rrt_set_spacetime(host_ctx.h, C.byref(st))
    assert (rc == rrt.RRT_OK) == ok, rrt.lib().rrt_last_error(host_ctx.h)


def _seg_dist(p, a, b):
    ab = b - a
    t = np.clip(((p - a) * ab).sum(-1) / np.maximum((ab * ab).sum(-1), 1e-300), 0.0, 1.0)
    d = p - (a + t[..., None] * ab)
    return np.sqrt((d * d).sum(-1))


def _tri_dist(p, a, b, c):
    """Euclidean distance from points p [m,1,3] to triangles a, b, c [1,t,3] -> [m,t]."""
    n = np.cross(b - a, c - a)
    nn = np.maximum((n * n).sum(-1), 1e-300)
    w = p - a
    h = (w * n).sum(-1) / nn
    q = p - h[..., None] * n                     # projection onto the plane
    def side(u, v):
        return (np.cross(v - u, q - u) * n).sum(-1)
    inside = (side(a, b) >= 0) & (side(b, c) >= 0) & (side(c, a) >= 0)
    d_in = np.abs(h) * np.sqrt(nn)
    d_edge = np.minimum(np.minimum(_seg_dist(p, a, b), _seg_dist(p, b, c)), _seg_dist(p, c, a))
    return np.where(inside, d_in, d_edge)


def _scene_prims(path):
    """Triangles (a, b, c) and spheres (centre, r) of a .rrts file (include/rrt_scene_format.h)."""
    raw = open(path, "rb").read()
    nb, no, _, _ = np.frombuffer(raw, "<u4", 4, 8)
    off = 24 + 64 * int(nb)
    tris, sph = [], []
    for _ in range(int(no)):
        kind, _, a, b = np.frombuffer(raw, "<u4", 4, off)
        off += 16
        if kind == 0:
            pos = np.frombuffer(raw, "<f8", 3 * int(a), off).reshape(-1, 3)
            off += 48 * int(a)
            idx = np.frombuffer(raw, "<u4", 3 * int(b), off).reshape(-1, 3)
            off += 12 * int(b)
            tris.append(pos[idx])
        else:
            v = np.frombuffer(raw, "<f8", 4, off)
            off += 32
            sph.append(v)
    return (np.concatenate(tris) if tris else np.zeros((0, 3, 3))), np.array(sph).reshape(-1, 4)


@pytest.mark.parametrize("scene", ["CBbunny", "CBspheres_lambertian", "CBcoil", "CBgems"])
def test_free_grid_is_conservative(host_ctx, scene):
    """Empty-space grid: from any point p, the free radius (k - 2) * h_free that
    the kernel reads for p's cell never exceeds p's true distance to the nearest primitive, and
    (for the floating-point hit region of Triangle::intersect) to the nearest triangle plane
    inside that triangle's leaf box -- so a skipped micro segment meets no primitive test that
    could accept it, and skipping it is result-identical.  The GPU parity tests check the
    rendered frames bit for bit with and without the grid."""
    path = os.path.join(GOLD, "scenes", scene + ".rrts")
    host_ctx.set_scene(rrt.SceneFile(path))
    g = host_ctx.free_grid()
    assert g is not None
    k, g0, inv_h, h_free = g
    tris, sph = _scene_prims(path)
    rng = np.random.default_rng(7)
    n = np.array(k.shape[::-1])
    span = n / inv_h
    pts = g0 + rng.uniform(-0.02, 1.02, size=(600, 3)) * span
    if len(tris):  # points hugging primitives, where the bound is tight
        t = tris[rng.integers(0, len(tris), 600)]
        wts = rng.dirichlet([1, 1, 1], 600)
        pts = np.concatenate([pts, (wts[:, :, None] * t).sum(1) + rng.normal(0, 4 / inv_h, (600, 3))])
    f = (pts - g0) * inv_h                       # same arithmetic as segment_clear()
    inside = np.all((f >= 0) & (f < n), axis=1)
    pts, f = pts[inside], f[inside]
    idx = f.astype(np.int64)
    free = (k[idx[:, 2], idx[:, 1], idx[:, 0]].astype(np.float64) - 2) * h_free
    assert (free > 0).mean() > 0.2
    dist = np.full(len(pts), np.inf)
    for i in range(0, len(pts), 64):
        p = pts[i:i + 64, None, :]
        if len(tris):
            dist[i:i + 64] = _tri_dist(p, tris[None, :, 0], tris[None, :, 1], tris[None, :, 2]).min(1)
        if len(sph):
            ds = np.sqrt(((p - sph[None, :, :3]) ** 2).sum(-1)) - sph[None, :, 3]
            dist[i:i + 64] = np.minimum(dist[i:i + 64], np.maximum(ds, 0).min(1))
    assert (dist - free).min() >= 0.0, (dist - free).min()
    s = host_ctx.stats()
    assert list(s.grid_n) == list(n) and 0.0 < s.grid_free_frac < 1.0


@pytest.mark.parametrize("scene", ["CBbunny", "CBcoil", "CBgems"])
def test_big_leaf_masks_are_conservative(host_ctx, scene):
    """Oversized-leaf masks: where a cell's bit for oversized leaf b is clear,
    every point of the cell is at least `reach` from every primitive of b, so a segment shorter
    than reach that starts there cannot be accepted by them and the walk may skip b."""
    path = os.path.join(GOLD, "scenes", scene + ".rrts")
    host_ctx.set_scene(rrt.SceneFile(path))
    bm = host_ctx.big_masks()
    assert bm is not None
    mask, reach = bm
    k, g0, inv_h, h_free = host_ctx.free_grid()
    assert mask.shape == k.shape and abs(reach - (rrt_internal_reach() - 1) * h_free) < 1e-15
    _, _, _, big = host_ctx.clean_tree()
    _, _, leaf_prims = host_ctx.bvh()
    tris, sph = _scene_prims(path)
    assert len(sph) == 0
    rng = np.random.default_rng(11)
    n = np.array(k.shape[::-1])
    span = n / inv_h
    pts = g0 + rng.uniform(-0.02, 1.02, size=(1500, 3)) * span
    t = tris[rng.integers(0, len(tris), 1500)]
    wts = rng.dirichlet([1, 1, 1], 1500)
    pts = np.concatenate([pts, (wts[:, :, None] * t).sum(1) + rng.normal(0, 12 / inv_h, (1500, 3))])
    f = (pts - g0) * inv_h                       # same arithmetic as grid_cell()
    inside = np.all((f >= 0) & (f < n), axis=1)
    pts, f = pts[inside], f[inside]
    idx = f.astype(np.int64)
    m = mask[idx[:, 2], idx[:, 1], idx[:, 0]]
    skipped = 0
    for b, (first, count, _) in enumerate(big):
        clear = (m >> np.uint32(b)) & 1 == 0
        if not clear.any():
            continue
        bt = tris[leaf_prims[first:first + count]]
        p = pts[clear][:, None, :]
        d = _tri_dist(p, bt[None, :, 0], bt[None, :, 1], bt[None, :, 2]).min(1)
        assert d.min() >= reach, (b, d.min(), reach)
        skipped += int(clear.sum())
    assert skipped > 0.3 * len(pts) * len(big)  # the masks do cull most leaves


def rrt_internal_reach():
    import re
    src = open(os.path.join(os.path.dirname(rrt.__file__), "csrc", "rrt_internal.h")).read()
    return int(re.search(r"#define RRT_BIG_REACH (\d+)", src).group(1))


@pytest.mark.parametrize("scene", ["CBbunny", "CBcoil", "CBgems"])
def test_clean_walk_matches_reference_walk(host_ctx, scene):
    """The clean-tree walk (oversized leaves listed apart, inner boxes refit), with and without the
    plane cull in front of primitive tests, returns the same closest hit (leaf slot and t, bit for
    bit) as the reference walk, on segments aimed at primitives, grazing them, inside the room
    and far outside."""
    from walk_sim import Walker
    path = os.path.join(GOLD, "scenes", scene + ".rrts")
    host_ctx.set_scene(rrt.SceneFile(path))
    ct = host_ctx.clean_tree()
    assert ct is not None and len(ct[3]) > 0
    boxes, nodes, prims = host_ctx.bvh()
    tris, _ = _scene_prims(path)
    t = tris[prims.astype(np.int64)]
    geo = np.concatenate([t[:, 0], t[:, 1] - t[:, 0], t[:, 2] - t[:, 0]], 1)
    w = Walker(boxes, nodes, geo, ct)
    w.planes(1e-9 * max(1.0, float(np.abs(boxes[0]).max())))
    rng = np.random.default_rng(3)
    lo, hi = boxes[0, :3], boxes[0, 3:]
    n_hit = 0
    for i in range(400):
        if i % 4 == 0:    # far away, long
            o = lo + rng.uniform(-2, 3, 3) * (hi - lo)
            L = rng.uniform(0.1, 20)
        else:             # near a primitive, short, often grazing
            k = rng.integers(len(t))
            tgt = rng.dirichlet([1, 1, 1]) @ t[k]
            o = tgt + rng.normal(0, 0.05, 3)
            L = rng.uniform(0.01, 0.3)
        dv = rng.normal(size=3)
        if i % 7 == 0:
            dv[rng.integers(3)] = 0.0  # axis-parallel component
        d = dv / np.linalg.norm(dv)
        o, d = tuple(float(v) for v in o), tuple(float(v) for v in d)
        ref = w.reference(o, d, float(L))
        got = w.clean(o, d, float(L))
        assert ref[:2] == got[:2], (i, ref, got)
        got = w.clean(o, d, float(L), cull=True)
        assert ref[:2] == got[:2], (i, ref, got)
        n_hit += ref[0] >= 0
    assert n_hit > 20


@pytest.mark.parametrize("scene", ["CBbunny", "CBcoil", "CBgems"])
def test_search_walk_matches_reference_walk(host_ctx, scene):
    """traverse_free (search tree): the SAH hierarchy holds exactly the clean tree's
    leaves (the reference's leaf boxes and slot runs) under inner boxes that contain them, and its
    walk at the full max_t followed by the ordered replay of the accepted primitives -- in windows
    of 4 slots, and of 1 to exercise the window edges -- returns the reference walk's closest hit
    (leaf slot and t, bit for bit) and its any-hit answer."""
    from walk_sim import Walker
    path = os.path.join(GOLD, "scenes", scene + ".rrts")
    host_ctx.set_scene(rrt.SceneFile(path))
    ct = host_ctx.clean_tree()
    st = host_ctx.search_tree()
    assert st is not None
    sb, sn = st
    cb, cn = ct[0], ct[1]
    leaves_clean = sorted((int(r[1]), int(r[2]), tuple(cb[i])) for i, r in enumerate(cn) if r[2] > 0)
    leaves_search = sorted((int(r[1]), int(r[2]), tuple(sb[i])) for i, r in enumerate(sn) if r[2] > 0)
    # the search tree holds the clean tree's leaves plus the local oversized ones (box diagonal at
    # most a quarter of the root's); the room-spanning ones stay on the walk's list
    bb, bg = ct[2], ct[3]
    root = host_ctx.bvh()[0][0]
    rd = float(np.linalg.norm(root[3:] - root[:3]))
    local = sorted((int(bg[i, 0]), int(bg[i, 1]), tuple(bb[i])) for i in range(len(bg))
                   if np.linalg.norm(bb[i, 3:] - bb[i, :3]) <= 0.25 * rd)
    assert leaves_search == sorted(leaves_clean + local)
    assert len(local) < len(bg)
    # pre-order with skip pointers; every inner box contains its subtree
    n = len(sn)
    end = [0] * n
    for i in range(n - 1, -1, -1):
        end[i] = i + 1 if sn[i][2] > 0 else end[end[i + 1]]
        assert sn[i][0] == (end[i] if end[i] < n else -1)
        if sn[i][2] == 0:
            sub = sb[i + 1:end[i]]
            assert (sb[i][:3] <= sub[:, :3]).all() and (sb[i][3:] >= sub[:, 3:]).all()
    boxes, nodes, prims = host_ctx.bvh()
    tris, _ = _scene_prims(path)
    t = tris[prims.astype(np.int64)]
    geo = np.concatenate([t[:, 0], t[:, 1] - t[:, 0], t[:, 2] - t[:, 0]], 1)
    w = Walker(boxes, nodes, geo, ct)
    w.planes(1e-9 * max(1.0, float(np.abs(boxes[0]).max())))
    w.set_search_tree(st)
    rng = np.random.default_rng(5)
    lo, hi = boxes[0, :3], boxes[0, 3:]
    n_hit = n_multi = 0
    for i in range(300):
        if i % 3 == 0:    # long segments through the geometry: several accepted primitives
            k = rng.integers(len(t))
            tgt = rng.dirichlet([1, 1, 1]) @ t[k]
            dv = rng.normal(size=3)
            dv /= np.linalg.norm(dv)
            o = tgt - dv * rng.uniform(0.2, 1.0)
            L = rng.uniform(0.5, 2.5)
        elif i % 3 == 1:  # near a primitive, short, often grazing
            k = rng.integers(len(t))
            tgt = rng.dirichlet([1, 1, 1]) @ t[k]
            o = tgt + rng.normal(0, 0.05, 3)
            L = rng.uniform(0.01, 0.3)
            dv = rng.normal(size=3)
        else:             # anywhere in and around the room
            o = lo + rng.uniform(-0.5, 1.5, 3) * (hi - lo)
            L = rng.uniform(0.05, 5)
            dv = rng.normal(size=3)
        if i % 7 == 0:
            dv[rng.integers(3)] = 0.0
        d = dv / np.linalg.norm(dv)
        o, d = tuple(float(v) for v in o), tuple(float(v) for v in d)
        ref = w.reference(o, d, float(L))
        for window in (4, 1):
            got = w.search(o, d, float(L), window=window)
            assert ref[:2] == got[:2], (i, window, ref, got)
            if window == 1:
                n_multi += w.windows > 2  # two or more primitives accepted at the full max_t
        anyh = w.search(o, d, float(L), any_hit=True)
        assert (anyh[0] >= 0) == (ref[0] >= 0), (i, ref, anyh)
        n_hit += ref[0] >= 0
    assert n_hit > 30 and n_multi > 10, (n_hit, n_multi)


def test_group_rejects_host_contexts():
    """rrt_group_create needs device contexts (a host-only context cannot render)."""
    import ctypes as C
    L = rrt.lib()
    h = C.c_void_p()
    cfg = rrt.DeviceCfg()
    cfg.device = -1
    assert L.rrt_create(C.byref(h), C.byref(cfg)) == 0
    arr = (C.c_void_p * 2)(h.value, h.value)
    g = C.c_void_p()
    L.rrt_group_create.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    assert L.rrt_group_create(arr, 2, C.byref(g)) == rrt.RRT_E_NO_DEVICE
    assert L.rrt_group_create(None, 0, C.byref(g)) == rrt.RRT_E_INVALID
    L.rrt_destroy(h)


@pytest.mark.parametrize("scene", ["CBbunny", "CBspheres_lambertian", "CBcoil", "CBgems"])
def test_search_tree4_covers_the_search_tree(host_ctx, scene):
    """The 4-wide walk's nodes (rrt_host.cpp build_free4): every search-tree leaf below the root is a
    leaf child of exactly one node, with its slot run; every inner child is a node reached once; each
    child's f32 box contains the f64 boxes of every search-tree node below it (a conservative
    pre-test: it never fails a box the exact test passes)."""
    sf = rrt.SceneFile(os.path.join(GOLD, "scenes", scene + ".rrts"))
    host_ctx.set_scene(sf)
    sboxes, snodes = host_ctx.search_tree()
    b4, k4 = host_ctx.search_tree4()
    if len(snodes) < 3:
        assert len(b4) == 0
        return
    assert 0 < len(b4) <= 65535
    leaves = [i for i in range(len(snodes)) if snodes[i, 2] != 0]
    seen, reached = [], [0]

    def below(i):  # search-tree nodes of i's subtree (pre-order: i .. skip(i) - 1)
        end = snodes[i, 0] if snodes[i, 0] >= 0 else len(snodes)
        return range(i, end)

    def node_box_cover(n4, j, subtree_root):
        b = b4[n4, j].astype(np.float64)
        for s in below(subtree_root):
            assert np.all(b[:3] <= sboxes[s, :3]) and np.all(b[3:] >= sboxes[s, 3:]), (n4, j, s)

    # map each 4-wide child back to a search-tree subtree: leaves by index, inner nodes by the union
    # of the leaves they reach
    def walk(n4):
        leaf_set = []
        for j in range(4):
            child, first, count = k4[n4, j]
            if count < 0:
                continue
            if count > 0:
                assert snodes[child, 2] == count and snodes[child, 1] == first
                seen.append(int(child))
                node_box_cover(n4, j, child)
                leaf_set.append(int(child))
            else:
                reached.append(int(child))
                sub = walk(child)
                for s in sub:
                    bb = b4[n4, j].astype(np.float64)
                    assert np.all(bb[:3] <= sboxes[s, :3]) and np.all(bb[3:] >= sboxes[s, 3:])
                leaf_set += sub
        return leaf_set
    walk(0)
    assert sorted(seen) == leaves
    assert sorted(reached) == list(range(len(b4)))
