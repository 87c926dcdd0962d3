"""Host-side image outputs and inputs of the PathTracer surface (no GPU):
  * rrt_tonemap_pixel == HDRImageBuffer::toColor + update_pixel: the reference's own PNG output
    (tests/golden/<case>/ref.png, written by the reference's save_image) is reproduced exactly
    from the reference's sampleBuffer;
  * rrt_write_png round-trips (PNG decoded by tests/png_util.py);
  * rrt_exr_save / rrt_exr_load round-trip, HALF channels, and the main.cpp channel mapping
    (R, G, B = file channels 2, 1, 0)."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

import rrt
from golden_cases import GOLD
from png_util import read_png


def _lib():
    L = rrt.lib()
    L.rrt_tonemap_pixel.restype = C.c_uint32
    L.rrt_tonemap_pixel.argtypes = [C.c_void_p]
    L.rrt_write_png.argtypes = [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]
    L.rrt_exr_save.argtypes = [C.c_char_p, C.c_void_p, C.c_uint32, C.c_uint32]
    L.rrt_exr_load.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_uint32),
                               C.POINTER(C.c_uint32)]
    L.rrt_exr_free.argtypes = [C.c_void_p]
    return L


def tonemap(rgb):
    L = _lib()
    h, w, _ = rgb.shape
    flat = np.ascontiguousarray(rgb.reshape(-1, 3), np.float32)
    out = np.array([L.rrt_tonemap_pixel(flat[i].ctypes.data) for i in range(len(flat))], np.uint32)
    return out.reshape(h, w)


@pytest.mark.parametrize("case", ["spheres_96x72_s8_l4", "cfg1_spheres_480x360_s8", "bunny_1080p_s64_crop"])
def test_tonemap_reproduces_reference_png(case):
    ref = read_png(os.path.join(GOLD, case, "ref.png"))
    rgb = np.load(os.path.join(GOLD, case, "px.npz"))["rgb"]
    mine = tonemap(rgb)[::-1].copy().view(np.uint8).reshape(*rgb.shape[:2], 4)  # save_image flips rows
    assert np.array_equal(mine, ref)


def test_png_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    for w, h in ((1, 1), (37, 5), (300, 260)):  # 300x260 spans several stored deflate blocks
        img = rng.integers(0, 2 ** 32, size=(h, w), dtype=np.uint64).astype(np.uint32)
        p = str(tmp_path / f"t{w}.png")
        assert _lib().rrt_write_png(p.encode(), img.ctypes.data, w, h) == 0
        back = read_png(p)
        assert np.array_equal(back, img.view(np.uint8).reshape(h, w, 4))


def _load_exr(path):
    L = _lib()
    t = C.POINTER(C.c_float)()
    w, h = C.c_uint32(), C.c_uint32()
    rc = L.rrt_exr_load(path.encode(), C.byref(t), C.byref(w), C.byref(h))
    if rc != 0:
        return rc, None
    arr = np.ctypeslib.as_array(t, shape=(h.value, w.value, 3)).copy()
    L.rrt_exr_free(t)
    return 0, arr


def test_exr_roundtrip(tmp_path):
    rng = np.random.default_rng(2)
    img = rng.random((17, 33, 3), dtype=np.float32) * 50
    p = str(tmp_path / "e.exr")
    assert _lib().rrt_exr_save(p.encode(), np.ascontiguousarray(img).ctypes.data, 33, 17) == 0
    rc, back = _load_exr(p)
    assert rc == 0 and np.array_equal(back, img)


def _write_exr(path, channels, planes, w, h, ptype):
    """EXR with the given channel names (file order) and per-channel planes [h][w]."""
    def attr(name, typ, val):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(val)) + val
    ch = b"".join(n.encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1) for n in channels) + b"\0"
    box = struct.pack("<4i", 0, 0, w - 1, h - 1)
    hdr = (struct.pack("<II", 20000630, 2) + attr("channels", "chlist", ch) + attr("compression", "compression", b"\0")
           + attr("dataWindow", "box2i", box) + attr("displayWindow", "box2i", box)
           + attr("lineOrder", "lineOrder", b"\0") + attr("pixelAspectRatio", "float", struct.pack("<f", 1))
           + attr("screenWindowCenter", "v2f", b"\0" * 8) + attr("screenWindowWidth", "float", struct.pack("<f", 1))
           + b"\0")
    dt = np.float16 if ptype == 1 else np.float32
    rows = []
    for y in range(h):
        data = b"".join(np.ascontiguousarray(pl[y], dt).tobytes() for pl in planes)
        rows.append(struct.pack("<ii", y, len(data)) + data)
    off = len(hdr) + 8 * h
    table = b""
    for r in rows:
        table += struct.pack("<Q", off)
        off += len(r)
    open(path, "wb").write(hdr + table + b"".join(rows))


def test_exr_half_and_channel_mapping(tmp_path):
    """main.cpp:69-75 takes R, G, B from channels 2, 1, 0 of the file (B, G, R when the file lists
    them alphabetically); HALF channels are widened exactly."""
    w, h = 5, 3
    rng = np.random.default_rng(3)
    planes = [rng.random((h, w)).astype(np.float16) * 10 for _ in range(3)]
    p = str(tmp_path / "h.exr")
    _write_exr(p, ["B", "G", "R"], planes, w, h, 1)
    rc, img = _load_exr(p)
    assert rc == 0
    for k, plane in zip((2, 1, 0), planes):
        assert np.array_equal(img[..., k], plane.astype(np.float32))
    # four channels A, B, G, R: the reference takes channels 2, 1, 0 = G, B, A (its quirk)
    planes4 = [np.full((h, w), v, np.float32) for v in (1.0, 2.0, 3.0, 4.0)]
    _write_exr(p, ["A", "B", "G", "R"], planes4, w, h, 2)
    rc, img = _load_exr(p)
    assert rc == 0 and np.all(img[..., 0] == 3.0) and np.all(img[..., 1] == 2.0) and np.all(img[..., 2] == 1.0)


def test_exr_rejects_compressed(tmp_path):
    p = str(tmp_path / "z.exr")
    _write_exr(p, ["B", "G", "R"], [np.zeros((2, 2), np.float32)] * 3, 2, 2, 2)
    raw = bytearray(open(p, "rb").read())
    i = raw.find(b"compression\0compression\0")
    raw[i + len(b"compression\0compression\0") + 4] = 3  # ZIP
    open(p, "wb").write(bytes(raw))
    rc, _ = _load_exr(p)
    assert rc == rrt.RRT_E_INVALID
