"""The device's restatement of the host C library's transcendentals (csrc/rrt_glibm.h) against the
library itself, on the CPU: the same source compiled as C must return the library's bits.

The reference calls glibc's sin/cos (sampler.cpp:53-55 cosine-weighted hemisphere sampler of every
diffuse bounce; environment_light.cpp:97-137), acos (sampler.cpp:20, bsdf.h:166,
environment_light.cpp:88), atan2 (environment_light.cpp:89), sinf/cosf (sampler.cpp:23-25) and, in
the microfacet BSDF, exp, log, erf, atan and tan (bsdf.cpp:45-96, bsdf.h:159-191).
Checked here (tests/glibm_check.c):
  * every argument the samplers can produce: Xi = k / RAND_MAX for all 2^31 k, through
    cos/sin(2 PI Xi), acos(Xi), (float)acos(Xi) and sinf/cosf of (float)acos(Xi), (float)(2 PI Xi);
  * sinf and cosf on every float of the restated domain |x| < 120;
  * the microfacet sampler's chain on all 2^31 Xi: log(1 - Xi), atan(sqrt(-a^2 log(1 - Xi))), tan of
    it and exp(-tan^2 / a^2) for three roughnesses;
  * 10^8 random arguments per function (value- and log-uniform; atan2 also on unit directions);
  * every branch boundary, zeros, infinities and NaNs.
The GPU side of the same check is tests/test_gpu_glibm.py.
"""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "relativistic-ray-tracer_amd", "csrc")


def precondition():
    """The parity precondition of rrt_glibm.h: the reference's bits are those of one
    libm build (Ubuntu GLIBC 2.35, sha-pinned by tools/gen_glibm_tables.py) on an x86-64 CPU with FMA
    and AVX2 (glibc's ifuncs then pick the FMA builds restated here).  None if it holds, else why not."""
    import hashlib
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen", os.path.join(ROOT, "tools", "gen_glibm_tables.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    if not os.path.exists(gen.LIBM):
        return f"no {gen.LIBM}"
    with open(gen.LIBM, "rb") as f:
        if hashlib.sha256(f.read()).hexdigest() != gen.LIBM_SHA256:
            return "this host's libm is not the pinned build " + gen.EXPECTED
    try:
        with open("/proc/cpuinfo") as f:
            flags = next((ln.split(":", 1)[1].split() for ln in f if ln.startswith("flags")), [])
    except OSError:
        flags = []
    if not ({"fma", "avx2"} <= set(flags)):
        return "the host CPU lacks FMA/AVX2: glibc would select other (non-FMA) builds"
    return None


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    why = precondition()
    if why:
        pytest.skip("PARITY PRECONDITION NOT MET (rrt_glibm.h restates one glibc build on FMA hosts): " + why)
    exe = str(tmp_path_factory.mktemp("glibm") / "glibm_check")
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-fopenmp", "-I", CSRC,
                    os.path.join(ROOT, "tests", "glibm_check.c"), "-o", exe, "-lm"], check=True)
    return exe


def run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=600)
    res = json.loads(r.stdout)
    print(res)
    for name, v in res.items():
        if name != "mode":
            tested, bad, first = v
            assert tested > 0 and bad == 0, f"{name}: {bad} of {tested} differ from the library (first at {first!r})"
    assert r.returncode == 0
    return res


def test_tables_are_the_librarys():
    """rrt_glibm_tables.h is what tools/gen_glibm_tables.py reads from this machine's libm."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen", os.path.join(ROOT, "tools", "gen_glibm_tables.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    import hashlib
    data = open(gen.LIBM, "rb").read()
    if hashlib.sha256(data).hexdigest() != gen.LIBM_SHA256:
        pytest.skip("a different libm build: the restatement is pinned to " + gen.EXPECTED)
    assert gen.render(data) == open(gen.OUT).read()


def test_branch_boundaries_and_specials(checker):
    run(checker, "specials")


def test_random_arguments(checker):
    res = run(checker, "random", 100_000_000, 20261017)
    assert res["sin"][0] == 100_000_000 and res["atan2"][0] == 100_000_000


def test_every_float_below_120(checker):
    run(checker, "floats", 0, 0x42F00000)            # +0 .. 120
    run(checker, "floats", 0x80000000, 0xC2F00000)   # -0 .. -120


def test_every_sampler_argument(checker):
    """All 2^31 values random_uniform() can return, through each reference call site."""
    res = run(checker, "sampler", 0, 2 ** 31)
    assert res["cos"][0] == 2 ** 31


def test_every_microfacet_sampler_argument(checker):
    """bsdf.cpp:76-86 on all 2^31 values random_uniform() can return, three roughnesses."""
    res = run(checker, "mf", 0, 2 ** 31)
    assert res["log"][0] == 2 ** 31 and res["tan"][0] == 3 * 2 ** 31
