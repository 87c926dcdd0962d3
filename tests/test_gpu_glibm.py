"""GPU: the device's restatement of the host C library's transcendentals (csrc/rrt_glibm.h, run
through the product library's rrt_libm_eval) returns the library's own bits.

The host side is the C library itself (oracle/restate ro_libm_eval: plain sin/cos/acos/atan2/
sinf/cosf calls, i.e. what the reference gets).  Arguments: a 2^24 stride through the 2^31 values
random_uniform() can return, taken through each reference call site (cos/sin(2 PI Xi),
sampler.cpp:53-55; acos(Xi), sampler.cpp:20; sinf/cosf of (float)acos(Xi) and (float)(2 PI Xi),
sampler.cpp:23-25), random arguments over each restated domain, the environment light's
atan2(-u.z, u.x) / acos(u.y) on random unit directions (environment_light.cpp:88-89), and every
branch boundary; and the microfacet BSDF's exp, log, erf, atan and tan (bsdf.cpp:45-96,
bsdf.h:159-191) on its sampler's arguments and on random arguments over each restated domain.
tests/test_glibm.py runs the full domains on the CPU build of the same source."""
import numpy as np
import pytest

import oracle_lib as ol
import rrt

pytestmark = pytest.mark.gpu

PI_REF = 3.14159265358979323  # misc.h:11


@pytest.fixture(scope="module")
def gpu():
    r = rrt.Renderer(device=0)
    yield r
    r.close()


def same_bits(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))


def check(gpu, fn, a, b=None):
    got = gpu.libm_eval(fn, a, b)
    want = ol.libm_eval(fn, a, b)
    ok = same_bits(got, want)
    if not ok.all():
        i = int(np.flatnonzero(~ok)[0])
        raise AssertionError(f"{fn}: {int((~ok).sum())} of {a.size} differ; first a={a[i]!r}"
                             + (f" b={b[i]!r}" if b is not None else "") + f" got {got[i]!r} want {want[i]!r}")
    return a.size


def boundaries():
    his = [0x3E400000, 0x3E500000, 0x3FEB6000, 0x400368FD, 0x419921FB, 0x3C880000, 0x3FC00000,
           0x3FD00000, 0x3FE00000, 0x3FE80000, 0x3FED8000, 0x3FEE8000, 0x3FEF0000, 0x3FF00000,
           0x7FF00000, 0x3FB00000, 0x20B00000, 0x5F300000, 0x00100000, 0]
    bits = np.array([(h << 32) + d for h in his for d in range(-64, 65) if (h << 32) + d >= 0], np.uint64)
    v = bits.view(np.float64)
    extra = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 0.126, 0.0625, PI_REF, 2.426265])
    return np.concatenate([v, -v, extra])


def test_sampler_arguments(gpu):
    k = np.arange(0, 2 ** 31, 128, dtype=np.int64) + np.random.default_rng(1).integers(0, 128, 2 ** 24)
    xi = k.astype(np.float64) / 2147483647.0          # random_uniform(): rand() / RAND_MAX
    theta = 2. * PI_REF * xi                           # sampler.cpp:53, :21
    check(gpu, "cos", theta)
    check(gpu, "sin", theta)
    check(gpu, "acos", xi)
    th_f = ol.libm_eval("acos", xi).astype(np.float32).astype(np.float64)
    check(gpu, "sinf", th_f)
    check(gpu, "cosf", th_f)
    ph_f = theta.astype(np.float32).astype(np.float64)
    check(gpu, "sinf", ph_f)
    check(gpu, "cosf", ph_f)


def test_random_arguments(gpu):
    g = np.random.default_rng(20261017)
    n = 1 << 22

    def mixed(lim):  # half value-uniform, half log-uniform magnitude (60 octaves below lim), either sign
        v = g.uniform(-lim, lim, n)
        e = g.uniform(min(-60.0, np.log2(lim) - 60.0), np.log2(lim), n)
        v[: n // 2] = np.sign(g.uniform(-1, 1, n // 2)) * 2.0 ** e[: n // 2]
        return v

    x = mixed(105414350.0)
    check(gpu, "sin", x)
    check(gpu, "cos", x)
    check(gpu, "acos", mixed(1.0))
    f = mixed(119.0).astype(np.float32).astype(np.float64)
    check(gpu, "sinf", f)
    check(gpu, "cosf", f)
    d = g.normal(size=(n, 3))
    u = d / np.sqrt((d * d).sum(-1))[:, None]          # unit directions
    check(gpu, "atan2", -u[:, 2], u[:, 0])             # environment_light.cpp:89
    check(gpu, "acos", u[:, 1])                        # environment_light.cpp:88
    check(gpu, "atan2", mixed(1e300), mixed(1e-300))


def test_branch_boundaries_and_specials(gpu):
    b = boundaries()
    # sin/cos are restated for |x| < 105414350 (high word < 0x419921FB, s_sin.c's
    # reduce_sincos range); beyond it the device calls its own sin/cos, which the sampler and
    # environment light never reach (their arguments are within [-2 pi, 2 pi])
    hi = (np.abs(b).view(np.uint64) >> np.uint64(32)).astype(np.int64)
    check(gpu, "sin", b[hi < 0x419921FB])
    check(gpu, "cos", b[hi < 0x419921FB])
    check(gpu, "acos", b)
    f = b[np.abs(b) < 120].astype(np.float32).astype(np.float64)
    check(gpu, "sinf", f)
    check(gpu, "cosf", f)
    yy, xx = np.meshgrid(b, b[::5])
    check(gpu, "atan2", yy.ravel(), xx.ravel())


def test_microfacet_functions(gpu):
    """The microfacet sampler's chain on a 2^24 stride through random_uniform()'s values (bsdf.cpp:76-86:
    log(1 - Xi), atan(sqrt(-a^2 log(1 - Xi))), tan of it, exp(-tan^2 / a^2)), each on the library's own
    inputs; then random arguments: exp over its finite range (subnormal results included), log of any
    positive double and near 1, erf, atan on the whole line, tan on its restated domain |x| <= 25."""
    k = np.arange(0, 2 ** 31, 128, dtype=np.int64) + np.random.default_rng(2).integers(0, 128, 2 ** 24)
    xi = k.astype(np.float64) / 2147483647.0
    check(gpu, "log", 1 - xi)
    lg = ol.libm_eval("log", 1 - xi)
    for alpha in (0.05, 0.25, 0.5):
        a2 = alpha * alpha
        q = np.sqrt(-a2 * lg)
        check(gpu, "atan", q)
        th = ol.libm_eval("atan", q)
        check(gpu, "tan", th)
        t = ol.libm_eval("tan", th)
        check(gpu, "exp", -t * t / a2)
    g = np.random.default_rng(20261018)
    n = 1 << 22

    def mixed(lim, octaves=60):
        v = g.uniform(-1.0, 1.0, n) * lim
        e = g.uniform(np.log2(lim) - octaves, np.log2(lim), n)
        v[: n // 2] = np.sign(g.uniform(-1, 1, n // 2)) * 2.0 ** e[: n // 2]
        return v

    check(gpu, "exp", mixed(760.0))
    check(gpu, "exp", mixed(1.0))
    check(gpu, "log", np.abs(mixed(1e308, 2000)))
    check(gpu, "log", 1.0 + mixed(0.1))
    check(gpu, "erf", mixed(7.0))
    check(gpu, "atan", mixed(20.0))
    check(gpu, "atan", mixed(1e300))
    check(gpu, "tan", mixed(3.2))
    check(gpu, "tan", mixed(25.0))
    b = boundaries()
    mb = np.array([(h << 32) + d for h in (0x3C900000, 0x40800000, 0x40900000, 0x40862E42, 0x408633CE, 0x40874910,
                                             0x3FEE0000, 0x3FF10900, 0x3FE60000, 0x00100000, 0x000FFFFF, 0x3E300000,
                                             0x3FEB0000, 0x3FF40000, 0x4006DB6E, 0x40180000, 0x00800000, 0x3E4BB67A,
                                             0x3FB00000, 0x40300000, 0x43349FF2, 0x3E4B096C, 0x3FAF212D, 0x3FE92F1A,
                                             0x40390000, 0x3FF921FB, 0x400921FB, 0x4012D97C)
                   for d in range(-64, 65)], np.uint64).view(np.float64)
    pts = np.concatenate([b, mb, -mb])
    for fn in ("exp", "log", "erf", "atan"):
        check(gpu, fn, pts)
    check(gpu, "tan", pts[~(np.abs(pts) > 25)])
