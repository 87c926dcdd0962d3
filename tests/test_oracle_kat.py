"""The CPU restatement (oracle/restate) against the reference's own function-level known
answers (tests/golden/kat, produced by oracle/ref/harness_kat.cpp from the compiled reference).
Bit-exact: same IEEE operations in the same order on the same x86-64 host."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle_lib as O

KAT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat")


def kat(name):
    return np.load(os.path.join(KAT, f"kat_{name}.npz"))["v"]


def same(a, b):
    """bit-equality for doubles (NaN == NaN)"""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(a, b, equal_nan=True)


def test_micro_chain():
    v = kat("micro")
    # group rows by (hole, ray0)
    keys = v[:, :11]
    starts = np.r_[0, np.nonzero(np.any(keys[1:] != keys[:-1], axis=1) & ~np.all(np.isnan(keys[1:]) & np.isnan(keys[:-1]), axis=1))[0] + 1]
    n_chains = 0
    for s in starts:
        bh = np.ascontiguousarray(v[s, 0:5])
        o = np.ascontiguousarray(v[s, 5:8])
        d = np.ascontiguousarray(v[s, 8:11])
        rows = v[s:][np.all((v[s:, :11] == v[s, :11]) | (np.isnan(v[s:, :11]) & np.isnan(v[s, :11])), axis=1)]
        out = np.zeros((128, 8))
        n = O.lib().ro_micro_chain(bh, o, d, out, 128)
        assert n >= len(rows)
        for r in rows:
            j = int(r[11])
            assert same(out[j, :7], r[12:19]), (j, out[j, :7], r[12:19])
            assert out[j, 7] == r[19]
        n_chains += 1
    assert n_chains >= 64


def test_bbox():
    v = kat("bbox")
    for r in v:
        t0, t1 = C.c_double(-7), C.c_double(-7)
        hit = O.lib().ro_bbox_intersect(np.ascontiguousarray(r[0:3]), np.ascontiguousarray(r[3:6]),
                                        np.ascontiguousarray(r[6:9]), np.ascontiguousarray(r[9:12]), r[12], r[13],
                                        C.byref(t0), C.byref(t1))
        assert hit == r[14]
        if hit:
            assert same(t0.value, r[15]) and same(t1.value, r[16])


def test_triangle():
    v = kat("tri")
    assert v[:, 25].sum() > 100  # enough hits
    for r in v:
        mt = C.c_double(r[24])
        hp, nn = np.zeros(3), np.zeros(3)
        hit = O.lib().ro_tri_intersect(np.ascontiguousarray(r[0:9]), np.ascontiguousarray(r[9:18]),
                                       np.ascontiguousarray(r[18:21]), np.ascontiguousarray(r[21:24]), C.byref(mt), hp, nn)
        assert hit == r[25]
        assert same(mt.value, r[26])
        if hit:
            assert same(hp, r[27:30]) and same(nn, r[30:33])


def test_sphere():
    v = kat("sphere")
    for k, r in enumerate(v):
        mt = C.c_double(r[10])
        hp, nn = np.zeros(3), np.zeros(3)
        want = 1 if k % 2 == 0 else 0
        hit = O.lib().ro_sphere_intersect(np.ascontiguousarray(r[0:3]), r[3], np.ascontiguousarray(r[4:7]),
                                          np.ascontiguousarray(r[7:10]), C.byref(mt), hp, nn, want)
        assert hit == r[11]
        assert same(mt.value, r[12])
        if hit and want:
            assert same(hp, r[13:16]) and same(nn, r[16:19])


def test_coord_space():
    v = kat("coord")
    for r in v:
        o2w, a, b = np.zeros(9), np.zeros(3), np.zeros(3)
        O.lib().ro_coord_space(np.ascontiguousarray(r[0:3]), np.ascontiguousarray(r[3:6]), o2w, a, b)
        assert same(o2w, r[6:15]) and same(a, r[15:18]) and same(b, r[18:21])


def test_samplers_draw_order():
    """UniformGridSampler2D draws y first (g++ evaluates Vector2D(ru(), ru()) right to left)."""
    v = kat("sampler")
    for r in v:
        out = np.zeros(3)
        pdf, used = C.c_float(), C.c_int()
        O.lib().ro_sampler(int(r[0]), np.array(r[1:3], np.int32), out, C.byref(pdf), C.byref(used))
        assert used.value == 2
        assert same(out, r[3:6]), (r[0], out, r[3:6])
        assert np.float32(pdf.value) == np.float32(r[6])
    g = v[v[:, 0] == 0]
    assert np.all(g[:, 4] == g[:, 1] / 2147483647.0)  # y <- first draw


def test_bsdf_sample_f():
    v = kat("bsdf")
    for r in v:
        f3 = np.zeros(3, np.float32)
        fe = np.zeros(3, np.float32)
        wi = np.zeros(3)
        pdf, used = C.c_float(), C.c_int()
        O.lib().ro_bsdf_sample(int(r[0]), np.ascontiguousarray(r[1:9]), np.ascontiguousarray(r[9:12]),
                               np.array(r[12:15], np.int32), f3, wi, C.byref(pdf), C.byref(used), fe)
        assert used.value == r[22], r[0]
        assert np.array_equal(f3, r[15:18].astype(np.float32)), (r[0], f3, r[15:18])
        assert same(wi, r[18:21]), (r[0], wi, r[18:21])
        assert np.float32(pdf.value) == np.float32(r[21])
        assert np.array_equal(fe, r[23:26].astype(np.float32))


def test_area_light():
    v = kat("area")
    for r in v:
        L = np.zeros(3, np.float32)
        wi = np.zeros(3)
        dist, pdf = C.c_float(), C.c_float()
        O.lib().ro_area_sample(r[0:3].astype(np.float32), np.ascontiguousarray(r[3:15]), np.ascontiguousarray(r[15:18]),
                               np.array(r[18:20], np.int32), L, wi, C.byref(dist), C.byref(pdf))
        assert np.array_equal(L, r[20:23].astype(np.float32))
        assert same(wi, r[23:26])
        assert np.float32(dist.value) == np.float32(r[26])
        assert np.float32(pdf.value) == np.float32(r[27])


def test_point_directional_hemisphere_lights():
    """PointLight / DirectionalLight / InfiniteHemisphereLight::sample_L (light.cpp:17-23, 34-42,
    49-57) with scripted draws; the light's own vector comes from the reference object (the
    ingest's construction of it is pinned by tests/test_ingest.py)."""
    v = kat("light")
    hemi_frame = np.array([[1, 0, 0], [0, 0, -1], [0, 1, 0], [0, 0, 0]], np.float64)  # light.cpp:29-31
    for r in v:
        kind = int(r[0])
        vv = hemi_frame.copy() if kind == 3 else np.zeros((4, 3))
        if kind != 3:
            vv[0] = r[7:10]
        L = np.zeros(3, np.float32)
        wi = np.zeros(3)
        dist, pdf, used = C.c_float(), C.c_float(), C.c_int()
        O.lib().ro_light_sample(kind, r[1:4].astype(np.float32), np.ascontiguousarray(vv.ravel()),
                                np.ascontiguousarray(r[10:13]), np.array(r[13:15], np.int32), L, wi,
                                C.byref(dist), C.byref(pdf), C.byref(used))
        assert np.array_equal(L, r[15:18].astype(np.float32)), r
        assert same(wi, r[18:21]), (kind, wi, r[18:21])
        assert np.float32(dist.value) == np.float32(r[21]) or (np.isinf(dist.value) and np.isinf(r[21]))
        assert np.float32(pdf.value) == np.float32(r[22])
        assert used.value == int(r[23])
    assert {int(k) for k in v[:, 0]} == {1, 2, 3}


def test_camera_ray():
    v = kat("camray")
    for r in v:
        o, d = np.zeros(3), np.zeros(3)
        mn, mx = C.c_double(), C.c_double()
        O.lib().ro_camera_ray(r[0], r[1], np.ascontiguousarray(r[2:5]), np.ascontiguousarray(r[5:14]), r[14], r[15],
                              r[16], r[17], o, d, C.byref(mn), C.byref(mx))
        assert same(o, r[18:21]) and same(d, r[21:24])
        assert mn.value == r[24] and mx.value == r[25]


def test_keyed_rng_reference_formula():
    """The keyed generator (oracle/ref/harness_common.h) restated in Python."""
    M = (1 << 64) - 1

    def mix(z):
        z ^= z >> 30; z = (z * 0xBF58476D1CE4E5B9) & M
        z ^= z >> 27; z = (z * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    for seed, x, y in [(0, 0, 0), (0, 479, 359), (7, 1919, 1079), (2 ** 40 + 3, 5, 9)]:
        key = mix((((y << 32) | x) ^ mix((seed + 0x9E3779B97F4A7C15) & M)) & M)
        assert O.lib().ro_pixel_key(seed, x, y) == key
        for n in range(5):
            want = mix((key + (n + 1) * 0x9E3779B97F4A7C15) & M) >> 33
            assert O.lib().ro_keyed_rand(key, n) == want
