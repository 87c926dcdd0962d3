"""GPU parity: the HIP path (through the C ABI) against the reference's golden outputs.

Every case (Case.exact) must be bit-exact, including the per-pixel sample counts and RNG draw
counts: the bounce, hemisphere, environment and microfacet paths' sin/cos/acos/atan2/sinf/cosf/
exp/log/erf/atan/tan are the host C library's own routines restated on the device
(rrt_glibm.h).  (check() keeps the north-star bound -- max per-pixel L2 of linear HDR RGB <= 1e-4
-- for any case marked inexact.)"""
import os

import numpy as np
import pytest

import rrt
from golden_cases import SMALL, Case, parity_metrics

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def gpu():
    r = rrt.Renderer(device=0)
    yield r
    r.close()


def render(gpu, c, draws=True, counters=False, flags=0):
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(c.envmap)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    bh = c.cfg["bh"]
    gpu.set_black_hole(bh[:3], bh[3], bh[4])
    g = c.cfg
    p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                          ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                          max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"], flags=flags)
    return gpu.render(p, c.x0, c.y0, c.w, c.h, draws=draws, counters=counters)


def check(c, rgb, cnt, draws):
    m = parity_metrics(c.px["rgb"], rgb)
    print(c.name, m, "count_eq", float(np.mean(cnt == c.px["count"])))
    if c.exact:
        assert np.array_equal(rgb.view(np.uint32), c.px["rgb"].view(np.uint32)), m
        assert np.array_equal(cnt, c.px["count"])
        if draws is not None:
            assert np.array_equal(draws, c.px["draws"])
    else:
        # north star: per-pixel L2 <= 1e-4, on every pixel
        assert m["max"] <= TOL, m
        assert np.array_equal(cnt, c.px["count"]), m
    return m


# every kernel path must meet the same bar: default (sample-parallel kernel, clean-tree BVH walk,
# empty-space grid), the reference-tree walk without the grid, the lane-per-pixel per-sample
# kernel and the per-pixel-loop kernel; the sample-parallel
# kernel also with one chip-wide claim queue, one queue per XCD, and in list order; and the
# default path with every camera ray marched exactly (no miss proof) and with every shadow ray
# marched exactly (no occlusion proof); at depth >= 2 also the per-sample refill kernel
VARIANTS = {"default": 0, "plain": rrt.RRT_RENDER_NO_CLEAN | rrt.RRT_RENDER_NO_SKIP,
            "onequeue": rrt.RRT_RENDER_ONE_QUEUE, "xcdqueues": rrt.RRT_RENDER_XCD_QUEUES,
            "ordered": rrt.RRT_RENDER_ORDERED, "noproof": rrt.RRT_RENDER_NO_MISS_PROOF,
            "prepass": rrt.RRT_RENDER_PREPASS, "striped": rrt.RRT_RENDER_STRIPED_QUEUES,
            "perpixel": rrt.RRT_RENDER_PER_PIXEL, "loop": rrt.RRT_RENDER_PIXEL_LOOP,
            "noshadowproof": rrt.RRT_RENDER_NO_SHADOW_PROOF,
            "nopixelproof": rrt.RRT_RENDER_NO_PIXEL_PROOF, "nosearch": rrt.RRT_RENDER_NO_SEARCH_TREE,
            "deepsample": rrt.RRT_RENDER_DEEP_SAMPLE, "noheavy": rrt.RRT_RENDER_NO_HEAVY,
            "heavy": rrt.RRT_RENDER_HEAVY}
# the path pool kernel (RRT_RENDER_WAVEFRONT) exists for depth >= 2 only
DEEP_VARIANTS = {"pathpool": rrt.RRT_RENDER_WAVEFRONT}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("name", SMALL)
def test_small_cases(gpu, name, variant):
    c = Case(name)
    rgb, cnt, draws, _ = render(gpu, c, flags=VARIANTS[variant])
    print(variant, end=" ")
    check(c, rgb, cnt, draws)


@pytest.mark.parametrize("variant", sorted(DEEP_VARIANTS))
@pytest.mark.parametrize("name", [n for n in SMALL if Case(n).cfg["max_ray_depth"] >= 2])
def test_small_deep_cases(gpu, name, variant):
    c = Case(name)
    rgb, cnt, draws, _ = render(gpu, c, flags=DEEP_VARIANTS[variant])
    assert "rrt_path_kernel" in gpu.stats().kernel.decode()
    print(variant, end=" ")
    check(c, rgb, cnt, draws)


PROOFS = {"proofs": 0,
          "noproofs": rrt.RRT_RENDER_NO_MISS_PROOF | rrt.RRT_RENDER_NO_SHADOW_PROOF | rrt.RRT_RENDER_NO_PIXEL_PROOF,
          "nocamproof": rrt.RRT_RENDER_NO_MISS_PROOF, "noshadowproof": rrt.RRT_RENDER_NO_SHADOW_PROOF,
          "nopixelproof": rrt.RRT_RENDER_NO_PIXEL_PROOF, "nosearch": rrt.RRT_RENDER_NO_SEARCH_TREE,
          "noheavy": rrt.RRT_RENDER_NO_HEAVY, "heavy": rrt.RRT_RENDER_HEAVY}


@pytest.mark.parametrize("proof", sorted(PROOFS))
@pytest.mark.parametrize("name", ["cfg1_spheres_480x360_s8", "cfg2_spheres_1080p_s64_flat", "cfg3_bunny_1080p_s64"])
def test_baseline_frames(gpu, name, proof):
    """The BASELINE.json configs, full frames, bit-exact against the reference (with the
    camera-ray miss proof and the shadow-ray occlusion proof, the default, and with either or
    both rays marched exactly)."""
    c = Case(name)
    rgb, cnt, draws, _ = render(gpu, c, flags=PROOFS[proof])
    check(c, rgb, cnt, draws)
    heavy = gpu.stats().last_heavy_pixels
    print("heavy pixels", heavy)
    if name.startswith("cfg3") and proof == "heavy":  # the hole's capture ring: slot-parallel pixels
        assert heavy > 0
    # no pass / flat / a whole frame (the heavy path runs by default for launches of <= 60% of it)
    if proof in ("noheavy", "nopixelproof", "noproofs", "proofs") or name.startswith("cfg2"):
        assert heavy == 0


def test_work_counters_closest_hit(gpu):
    """Counting variant: micro steps per pixel equal the reference's own (camera rays are
    closest-hit; shadow rays stop at the first hit on the GPU, so AABB tests are <= ref)."""
    c = Case("spheres_96x72_s1")
    rgb, cnt, draws, ctr = render(gpu, c, counters=True)
    assert np.array_equal(rgb.view(np.uint32), c.px["rgb"].view(np.uint32))
    assert np.all(ctr[..., 0] <= c.px["bbox_tests"])
    assert np.all(ctr[..., 1] <= c.px["micro_steps"])
    assert ctr[..., 0].sum() > 0.5 * c.px["bbox_tests"].sum()


def test_device_tiles_path_matches_host_path(gpu):
    """rrt_render_tiles_device (packed tiles) + rrt_unpack_tiles_device == rrt_render."""
    torch = pytest.importorskip("torch")
    c = Case("bunny_160x120_s16")
    rgb_h, cnt_h, _, _ = render(gpu, c, draws=False)
    W, H, ts = c.frame_w, c.frame_h, 32
    g = c.cfg
    p = rrt.render_params(W, H, ns_aa=g["ns_aa"])
    out_rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    out_cnt = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    for world in (1, 3):
        out_rgb.zero_(); out_cnt.zero_()
        for r in range(world):
            tiles = rrt.partition_tiles(W, H, ts, r, world)
            prgb = torch.zeros(len(tiles) * ts * ts * 3, dtype=torch.float32, device="cuda")
            pcnt = torch.zeros(len(tiles) * ts * ts, dtype=torch.int32, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            gpu.render_tiles_device(p, tiles, ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
            gpu.unpack_tiles_device(tiles, ts, W, H, prgb.data_ptr(), pcnt.data_ptr(), out_rgb.data_ptr(),
                                    out_cnt.data_ptr(), stream=s)
        torch.cuda.synchronize()
        assert np.array_equal(out_rgb.cpu().numpy().reshape(H, W, 3).view(np.uint32), rgb_h.view(np.uint32))
        assert np.array_equal(out_cnt.cpu().numpy().reshape(H, W), cnt_h)


@pytest.mark.parametrize("world", [2, 8])
def test_rank_tiles_cfg3_heavy_path(gpu, world):
    """Every rank's tile set of the cfg3 frame (bench.py's block-cyclic split over `world` GPUs),
    rendered on this GPU through the device path, unpacked into one frame: bit-exact against the
    reference's frame.  A rank's launch covers <= 60% of the frame, so the heavy pixels' kernel
    runs beside the batch kernel (its pixels straddle the hole's capture ring)."""
    torch = pytest.importorskip("torch")
    c = Case("cfg3_bunny_1080p_s64")
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(c.envmap)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    bh = c.cfg["bh"]
    gpu.set_black_hole(bh[:3], bh[3], bh[4])
    W, H, ts, g = c.frame_w, c.frame_h, 32, c.cfg
    p = rrt.render_params(W, H, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"], ns_area_light=g["ns_area_light"],
                          samples_per_batch=g["samples_per_batch"], max_tolerance=g["max_tolerance"])
    out_rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    out_cnt = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    heavy = 0
    for r in range(world):
        tiles = rrt.partition_tiles(W, H, ts, r, world)
        prgb = torch.zeros(len(tiles) * ts * ts * 3, dtype=torch.float32, device="cuda")
        pcnt = torch.zeros(len(tiles) * ts * ts, dtype=torch.int32, device="cuda")
        gpu.render_tiles_device(p, tiles, ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
        torch.cuda.synchronize()
        heavy += gpu.stats().last_heavy_pixels
        gpu.unpack_tiles_device(tiles, ts, W, H, prgb.data_ptr(), pcnt.data_ptr(), out_rgb.data_ptr(),
                                out_cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    print("world", world, "heavy pixels", heavy)
    assert heavy > 0
    rgb = out_rgb.cpu().numpy().reshape(H, W, 3)
    assert np.array_equal(rgb.view(np.uint32), c.px["rgb"].view(np.uint32))
    assert np.array_equal(out_cnt.cpu().numpy().reshape(H, W), c.px["count"])


def test_tonemap(gpu):
    torch = pytest.importorskip("torch")
    c = Case("cfg1_spheres_480x360_s8")
    rgb = torch.from_numpy(c.px["rgb"].reshape(-1).copy()).cuda()
    out = torch.zeros(c.w * c.h, dtype=torch.int32, device="cuda")
    gpu.tonemap_device(c.w * c.h, rgb.data_ptr(), out.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(c.h, c.w)
    # HDRImageBuffer::toColor + ImageBuffer::update_pixel (image.h:53-62, 183-198), float pow
    s = c.px["rgb"].astype(np.float32) * np.float32(np.sqrt(2.0))
    v = np.power(s, np.float32(1.0) / np.float32(2.2)).astype(np.float32)
    v = np.where(v < 1, v, np.float32(1)).astype(np.float32)
    q = (v * np.float32(255)).astype(np.uint32)
    want = 0xFF000000 | (q[..., 2] << 16) | (q[..., 1] << 8) | q[..., 0]
    diff = np.abs(((got >> 0) & 255).astype(int) - (want & 255).astype(int))
    assert diff.max() <= 1 and np.mean(got == want) > 0.999


def test_render_after_failed_set_scene():
    """A failed second rrt_set_scene leaves no scene: rrt_render reports RRT_E_INVALID instead of
    launching over the previous scene's device buffers."""
    from test_capi_host import _bad_scene_after_good

    r = rrt.Renderer(device=0)
    try:
        _bad_scene_after_good(r)
        r.set_camera(rrt.load_camera(Case("spheres_96x72_s1").camera_path))
        with pytest.raises(rrt.RRTError) as e:
            r.render(rrt.render_params(16, 16), 0, 0, 16, 16)
        assert e.value.code == rrt.RRT_E_INVALID
    finally:
        r.close()


def test_two_streams_one_context(gpu):
    """rrt_render_tiles_device on two streams of one context: the second launch waits for the
    first (the context's workspace is fenced), so both frames equal the golden one."""
    import torch

    c = Case("spheres_96x72_s8_l4")
    assert c.exact
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(None)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    bh = c.cfg["bh"]
    gpu.set_black_hole(bh[:3], bh[3], bh[4])
    g = c.cfg
    p = rrt.render_params(c.frame_w, c.frame_h, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"],
                          ns_area_light=g["ns_area_light"], samples_per_batch=g["samples_per_batch"],
                          max_tolerance=g["max_tolerance"], direct_hemisphere=g["direct_hemisphere"])
    ts = 32
    tiles = np.array([(x, y) for y in range(0, c.frame_h, ts) for x in range(0, c.frame_w, ts)], np.uint32)
    n = len(tiles) * ts * ts
    outs = []
    streams = [torch.cuda.Stream(device=0), torch.cuda.Stream(device=0)]
    for s in streams:
        rgb = torch.empty(n * 3, dtype=torch.float32, device="cuda:0")
        cnt = torch.empty(n, dtype=torch.int32, device="cuda:0")
        gpu.render_tiles_device(p, tiles, ts, rgb.data_ptr(), cnt.data_ptr(), stream=s.cuda_stream)
        outs.append((rgb, cnt))
    torch.cuda.synchronize()
    frames = []
    for rgb, cnt in outs:
        fr = np.zeros((c.frame_h, c.frame_w, 3), np.float32)
        rg = rgb.cpu().numpy().reshape(len(tiles), ts, ts, 3)
        for t, (x, y) in enumerate(tiles):
            h, w = min(ts, c.frame_h - y), min(ts, c.frame_w - x)
            fr[y:y + h, x:x + w] = rg[t, :h, :w]
        frames.append(fr[c.y0:c.y0 + c.h, c.x0:c.x0 + c.w])
    assert np.array_equal(frames[0].view(np.uint32), frames[1].view(np.uint32))
    assert np.array_equal(frames[0].view(np.uint32), c.px["rgb"].view(np.uint32))


# Continuations: pixels of >= 3 adaptive steps that have not stopped at a check are
# handed from the batch kernel to waiting heavy blocks (by default in launches of <= 60% of the
# frame: the crops).  Modes: the library default; "eager" hands over every pixel that did not stop
# (RRT_AB_CONT_MIN=1), in any launch (RRT_AB_CONT=1), with room for 64 heavy blocks from the
# launch's start; "off" (RRT_AB_CONT=0).  Read by the library at every launch.
CONT_MODES = {"default": {}, "eager": {"RRT_AB_CONT": "1", "RRT_AB_CONT_MIN": "1", "RRT_AB_CONT_ROOM": "64"},
              "off": {"RRT_AB_CONT": "0"}}
CONT_CASES = ["cfg4_knot_4k_s256_crop", "cfg4_knot_4k_s256_crop2", "cfg4_knot_4k_s256_crop3", "spheres_96x72_s64_a16"]


@pytest.fixture
def cont_env():
    keys = {k for m in CONT_MODES.values() for k in m}
    saved = {k: os.environ.get(k) for k in keys}

    def set_mode(mode):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(CONT_MODES[mode])

    yield set_mode
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("mode", sorted(CONT_MODES))
@pytest.mark.parametrize("name", CONT_CASES)
def test_continuations(gpu, cont_env, name, mode):
    """Bit-exact with the batch kernel's pixels resumed by the heavy kernel from their folded sums."""
    cont_env(mode)
    c = Case(name)
    rgb, cnt, draws, _ = render(gpu, c)
    st = gpu.stats()
    print(name, mode, "continuations", st.last_cont_pixels, "heavy", st.last_heavy_pixels, st.kernel.decode())
    check(c, rgb, cnt, draws)
    if mode == "off":
        assert st.last_cont_pixels == 0
    if mode == "eager":  # some pixel of each case goes past its first check
        assert st.last_cont_pixels > 0


@pytest.mark.parametrize("world", [8])
def test_rank_tiles_cfg4_crops(gpu, cont_env, world):
    """cfg4 (4K, 256 spp) split `world` ways as bench.py splits it: every rank's tiles that cover
    the three reference-rendered crops, rendered through the device path (heavy pixels and
    continuations on: a rank's launch is a small part of the frame), unpacked into one frame:
    bit-exact against the reference's crops."""
    torch = pytest.importorskip("torch")
    cont_env("default")
    cases = [Case(n) for n in CONT_CASES[:3]]
    c = cases[0]
    gpu.set_scene(rrt.SceneFile(c.scene_path))
    gpu.set_envmap(c.envmap)
    gpu.set_camera(rrt.load_camera(c.camera_path))
    bh = c.cfg["bh"]
    gpu.set_black_hole(bh[:3], bh[3], bh[4])
    W, H, ts, g = c.frame_w, c.frame_h, 32, c.cfg
    p = rrt.render_params(W, H, ns_aa=g["ns_aa"], max_ray_depth=g["max_ray_depth"], ns_area_light=g["ns_area_light"],
                          samples_per_batch=g["samples_per_batch"], max_tolerance=g["max_tolerance"])
    out_rgb = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda")
    out_cnt = torch.full((H * W,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def covers(x, y):
        return any(x < k.x0 + k.w and x + ts > k.x0 and y < k.y0 + k.h and y + ts > k.y0 for k in cases)

    n_cont = 0
    for r in range(world):
        tiles = np.array([t for t in rrt.partition_tiles(W, H, ts, r, world) if covers(int(t[0]), int(t[1]))],
                         np.uint32).reshape(-1, 2)
        if len(tiles) == 0:
            continue
        prgb = torch.zeros(len(tiles) * ts * ts * 3, dtype=torch.float32, device="cuda")
        pcnt = torch.zeros(len(tiles) * ts * ts, dtype=torch.int32, device="cuda")
        gpu.render_tiles_device(p, tiles, ts, prgb.data_ptr(), pcnt.data_ptr(), stream=s)
        torch.cuda.synchronize()
        n_cont += gpu.stats().last_cont_pixels
        gpu.unpack_tiles_device(tiles, ts, W, H, prgb.data_ptr(), pcnt.data_ptr(), out_rgb.data_ptr(),
                                out_cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    rgb = out_rgb.cpu().numpy().reshape(H, W, 3)
    cnt = out_cnt.cpu().numpy().reshape(H, W)
    print("world", world, "continuations", n_cont)
    for k in cases:
        ys, xs = slice(k.y0, k.y0 + k.h), slice(k.x0, k.x0 + k.w)
        assert np.array_equal(rgb[ys, xs].view(np.uint32), k.px["rgb"].view(np.uint32)), k.name
        assert np.array_equal(cnt[ys, xs], k.px["count"]), k.name
