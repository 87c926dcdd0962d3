"""The Kerr integrator (build-defined) -- parity UNPINNED.

The reference has no Kerr metric, so there is no reference output to pin against.  Instead the
CPU restatement (oracle/restate ro_kerr_chain, which the GPU must reproduce: test_gpu_kerr.py)
is pinned by physics:
  * a -> 0: the spatial path is the Schwarzschild photon orbit u'' + u = 3 M u^2, the equation
    the reference's BlackHole::next_micro_ray (blackhole.cpp:13-40) steps; checked against a
    high-accuracy solution, and against the reference stepper's own capture behaviour;
  * the photon-capture thresholds: b_c = 3 sqrt(3) M at a = 0, and the equatorial prograde /
    retrograde critical impact parameters b = -/+ a + 6 M cos(arccos(-/+ a / M) / 3) at a = 0.9
    (the asymmetric Kerr shadow);
  * the constants of motion: H = 0 (null) and L_z (axisymmetry) along the march.
"""
import numpy as np
import pytest

import oracle_lib as ol
import rrt

RS = 0.1
M = RS / 2
HOLE = (0.0, 1.0, 0.0)


def chain(o, d, spin=0.0, dt=0.1, axis=(0.0, 1.0, 0.0), rows=63):
    return ol.kerr_chain(HOLE + (RS, dt), spin, axis, np.asarray(o, float), np.asarray(d, float), max_rows=rows)


def test_frame_matches_library():
    """The restatement's local frame is the library's (rrt_kerr_frame)."""
    for axis in [(0, 1, 0), (0, 0, 1), (1, 2, 3), (0.0, -0.3, 0.95)]:
        _, fr = chain((0, 1, 3), (0, 0, -1), spin=0.5, axis=axis, rows=1)
        lib = rrt.kerr_frame(axis)
        assert np.array_equal(fr, lib), (axis, fr, lib)
        assert np.allclose(fr @ fr.T, np.eye(3), atol=1e-15)
        assert np.allclose(np.cross(fr[0], fr[1]), fr[2], atol=1e-15)


@pytest.mark.parametrize("b", [0.3, 0.5, 1.0])
def test_a0_is_the_schwarzschild_orbit(b):
    """a = 0: r(phi) along the march solves u'' + u = 3 M u^2 (= 1.5 r_s u^2, blackhole.cpp:13-15)."""
    from scipy.integrate import solve_ivp
    o = np.array([-3.0, 1.0, b])
    d = np.array([1.0, 0.0, 0.0])
    rows, fr = chain(o, d)
    assert len(rows) == 63 and rows[-1, 7] == 0  # escapes within one revolution's steps
    q = rows[:, 8:11]
    q0, d0 = fr @ (o - np.array(HOLE)), fr @ d
    n = np.cross(q0, d0)
    n /= np.linalg.norm(n)
    assert np.abs(q @ n).max() < 1e-12  # planar orbit
    e1 = q0 / np.linalg.norm(q0)
    e2 = np.cross(n, e1)
    phi = np.unwrap(np.arctan2(q @ e2, q @ e1))
    u0 = 1 / np.linalg.norm(q0)
    up0 = -u0 * (d0 @ e1) / (d0 @ e2)
    sol = solve_ivp(lambda t, y: [y[1], -y[0] + 1.5 * RS * y[0] ** 2], (0, phi[-1]), [u0, up0], rtol=1e-12,
                    atol=1e-14, dense_output=True)
    u = sol.sol(phi)[0]
    rel = np.abs(1 / np.linalg.norm(q, axis=1) - u) / u
    assert rel.max() < 1e-4, rel.max()


def test_a0_limit_is_continuous():
    """a = 1e-9 and a = 0 give the same march to ~1e-9."""
    o, d = (-2.0, 1.2, 0.3), (1.0, -0.05, 0.0)
    r0, _ = chain(o, d, spin=0.0)
    r1, _ = chain(o, d, spin=1e-9)
    assert len(r0) == len(r1)
    assert np.abs(r0[:, :3] - r1[:, :3]).max() < 1e-8


def test_a0_capture_vs_reference_stepper():
    """Capture (return false) vs the reference's own stepper (ro_micro_chain = next_micro_ray,
    pinned by the KATs).  Both capture deep inside the critical impact parameter and both let
    rays well outside it escape.  In between (0.6-0.9 b_c) the reference's fixed-angle step
    overshoots the hole and lets the ray out: its capture cross-section is smaller than the
    physical 3 sqrt(3) M, which the RK4 march resolves."""
    bc = 3 * np.sqrt(3) * M
    for f, kerr_want, ref_want in [(0.3, 1, 1), (0.6, 1, 0), (0.9, 1, 0), (1.2, 0, 0), (2.0, 0, 0)]:
        o, d = np.array([-2.0, 1.0, f * bc]), np.array([1.0, 0.0, 0.0])
        rows, _ = chain(o, d, dt=0.02, rows=2000)
        assert rows[-1, 7] == kerr_want, f
        ref = np.zeros((64, 8))
        n = ol.lib().ro_micro_chain(np.array(HOLE + (RS, 0.1)), o, d, ref, 64)
        assert ref[n - 1, 7] == ref_want, f


@pytest.mark.parametrize("spin", [0.0, 0.9])
def test_capture_thresholds(spin):
    """Equatorial critical impact parameters: b = -a + 6M cos(acos(-a/M)/3) (prograde),
    a + 6M cos(acos(a/M)/3) (retrograde); a = 0: 3 sqrt(3) M."""
    a = spin * M
    b_pro = -a + 6 * M * np.cos(np.arccos(-spin) / 3)
    b_ret = a + 6 * M * np.cos(np.arccos(spin) / 3)
    if spin == 0:
        assert np.isclose(b_pro, 3 * np.sqrt(3) * M) and np.isclose(b_ret, b_pro)
    _, fr = chain((0, 1, 3), (0, 0, -1), spin=spin, rows=1)
    ex, ey = fr[0], fr[1]
    for side, bb in [(+1, b_pro), (-1, b_ret)]:
        for f, want in [(0.95, 1), (1.05, 0)]:
            # moving along +ex from x = -2: L_z = -y p_x, so y < 0 is prograde
            o = np.array(HOLE) - 2.0 * ex - side * f * bb * ey
            rows, _ = chain(o, ex, spin=spin, dt=0.02, rows=4000)
            assert rows[-1, 7] == want, (spin, side, f)


def _H_Lz(q, p, spin):
    a = spin * M
    H, Lz = [], []
    for (x, y, z), pi in zip(q, p):
        w = x * x + y * y + z * z - a * a
        r2 = 0.5 * w + np.sqrt(0.25 * w * w + a * a * z * z)
        r = np.sqrt(r2)
        f = 2 * M * r * r2 / (r2 * r2 + a * a * z * z)
        l = np.array([(r * x + a * y) / (r2 + a * a), (r * y - a * x) / (r2 + a * a), z / r])
        L = 1 + l @ pi
        H.append(0.5 * (-1 + pi @ pi - f * L * L) / (pi @ pi))
        Lz.append(x * pi[1] - y * pi[0])
    return np.array(H), np.array(Lz)


@pytest.mark.parametrize("o,d", [((-2, 1.3, 0.4), (1, -0.1, -0.05)), ((0.5, 2.5, -1.5), (-0.1, -0.6, 0.5)),
                                 ((0.3, 1.4, 1.0), (-0.1, -0.3, -1.0))])
def test_constants_of_motion(o, d):
    d = np.array(d, float) / np.linalg.norm(d)
    rows, _ = chain(o, d, spin=0.9)
    H, Lz = _H_Lz(rows[:, 8:11], rows[:, 11:14], 0.9)
    assert np.abs(H).max() < 1e-5
    assert np.abs(Lz - Lz[0]).max() < 1e-5 * max(abs(Lz[0]), 1e-3)


def _exit_deflection(rows_o, rows_d, o, d):
    r = np.linalg.norm(rows_o - np.array(HOLE), axis=1)
    i = np.argmin(r)
    j = i + np.argmax(r[i:] > 2.0)
    return np.degrees(np.arccos(np.clip(rows_d[j] @ d, -1, 1)))


def test_a0_deflection_is_exact_reference_stepper_is_not():
    """A camera ray of the cfg3 framing passing the hole at b = 7.6 M: the exact Schwarzschild
    deflection (orbit equation to infinity) is 53.9 deg.  The Kerr march at a = 0 gives it; the
    reference's next_micro_ray converges (delta_theta -> 0) to 18.9 deg -- it re-derives u' from
    the previous chord every step and loses most of the bending.  So the Kerr renderer at a = 0
    is the physical Schwarzschild image, not the reference's."""
    from scipy.integrate import solve_ivp
    o = np.array([0.0, 0.75, -4.80234411])
    d = np.array([0.07909504, 0.04609135, 0.99580096])
    d /= np.linalg.norm(d)
    q0 = o - np.array(HOLE)
    r0 = np.linalg.norm(q0)
    e1 = q0 / r0
    n = np.cross(q0, d)
    n /= np.linalg.norm(n)
    e2 = np.cross(n, e1)
    u0, up0 = 1 / r0, -(d @ e1) / (d @ e2) / r0
    ev = lambda t, y: y[0]  # noqa: E731
    ev.terminal, ev.direction = True, -1
    bent = solve_ivp(lambda t, y: [y[1], -y[0] + 1.5 * RS * y[0] ** 2], (0, 10), [u0, up0], rtol=1e-12,
                     atol=1e-14, events=ev).t_events[0][0]
    flat = solve_ivp(lambda t, y: [y[1], -y[0]], (0, 10), [u0, up0], rtol=1e-12, atol=1e-14,
                     events=ev).t_events[0][0]
    exact = np.degrees(bent - flat)
    assert abs(exact - 53.91) < 0.01
    rows, _ = chain(o, d, dt=0.005, rows=20000)
    assert abs(_exit_deflection(rows[:, :3], rows[:, 3:6], o, d) - exact) < 0.05
    rows, _ = chain(o, d, dt=0.1, rows=200)  # the renderer's step: within half a degree
    assert abs(_exit_deflection(rows[:, :3], rows[:, 3:6], o, d) - exact) < 0.5
    ref = np.zeros((20000, 8))
    m = ol.lib().ro_micro_chain(np.array(HOLE + (RS, 0.001)), o, d, ref, 20000)
    assert abs(_exit_deflection(ref[:m, :3], ref[:m, 3:6], o, d) - 18.86) < 0.05
