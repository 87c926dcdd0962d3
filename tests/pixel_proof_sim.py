"""numpy mirror of the pixel miss proof (relativistic-ray-tracer_amd/csrc/rrt_device.h
pixel_miss_proof), one pixel at a time, given the pixel's centre and corner ray directions.

TEST INFRASTRUCTURE ONLY (tests/test_pixel_proof.py): the product runs the HIP version.

Every camera ray of a pixel starts at the camera position O and shares x = (O - c) / |O - c|;
its planar march depends on its direction only through dx = d . x, its plane through y.  The
proof runs the recurrence (tests/miss_proof_sim.py) for the pixel's least, central and largest
dx, bounds every ray's points around the central ray's, and requires each central segment to
clear the root box by the camera proof's margin plus that bound.
"""
import numpy as np

from miss_proof_sim import ETA, KAPPA, seg_clear


def prove(K, O, dc, corners):
    """True if every ray through the pixel (centre direction dc, corner directions corners [4,3])
    is a proven miss."""
    c = K["c"]
    x0 = O - c
    r0 = np.sqrt(x0 @ x0)
    u0 = 1.0 / r0
    X = x0 * u0
    dxc = dc @ X
    Yc = dc - dxc * X
    dyc = np.sqrt(Yc @ Yc)
    if not dyc > 1e-3:
        return False
    Yc = Yc / dyc
    dlo = dhi = dxc
    dY = dd = 0.0
    dymin = dyc
    for d in corners:
        dx = d @ X
        dlo, dhi = min(dlo, dx), max(dhi, dx)
        yv = d - dx * X
        dy = np.sqrt(yv @ yv)
        if not dy > 1e-3:
            return False
        dymin = min(dymin, dy)
        dY = max(dY, np.linalg.norm(yv / dy - Yc))
        dd = max(dd, np.linalg.norm(d - dc))
    if not dd <= 0.25 * dymin:  # +-X (where y turns round) kept well outside the rectangle
        return False
    slack = 2.0 * dd * dd + 1e-12
    wdx = dhi - dlo
    dlo -= 0.05 * wdx + slack
    dhi += 0.05 * wdx + slack
    dY = 1.25 * dY + slack
    if not (dlo > -1.0 and dhi < 1.0):
        return False
    dxs = np.array([dlo, dxc, dhi])
    up0 = -u0 * dxs / np.sqrt(1.0 - dxs * dxs)
    vp = np.full(3, K["rho"] * u0)
    s = u0 * K["co1"] - up0 * K["si"] / K["rho"]
    ea, eb, sig, rp, dpa, dvp = 1.0, 0.0, 1.0, r0, 0.0, 0.0
    si2 = K["si"] * K["si"]
    rho = K["rho"]
    for j in range(K["steps"]):
        up = (vp * K["co1"] - rho * s) / K["si"]
        s = np.abs(vp) / rho
        f1 = -s + K["k15"] * s * s
        u2 = s + up * (K["dt"] * 0.5)
        f2 = -u2 + K["k15"] * u2 * u2
        u3 = u2 + f1 * (K["dt"] * K["dt"] / 4.0)
        f3 = -u3 + K["k15"] * u3 * u3
        v = s + up * K["dt"] + (f1 + f2 + f3) * (K["dt"] * K["dt"] / 6.0)
        ok = bool(np.all(np.abs(v) >= KAPPA * (s + np.abs(up) * K["dt"])))
        dv = 1.5 * max(abs(v[0] - v[1]), abs(v[2] - v[1]))
        av = abs(v[1])
        if not (ok and (v[0] < 0) == (v[1] < 0) and (v[2] < 0) == (v[1] < 0) and av > 2.0 * dv):
            return False
        sg = -1.0 if vp[1] < 0.0 else 1.0
        a, b = sg * K["co1"], sig * K["si1"]
        na, nb = a * ea - b * eb, a * eb + b * ea
        sig *= sg
        r = rho / (av - dv) * (1.0 + 1e-6)
        dpb = rho * dv / (av * (av - dv)) * (1.0 + 1e-6) + r * abs(nb) * dY
        m0 = ETA * (max(rp, r) + K["scale"])
        m = m0 + max(dpa, dpb)
        rb = K["r_ball"] + m0
        far = True
        for k in range(4):
            w = v[1] + (dv if k & 1 else -dv)
            wp = vp[1] + (dvp if k & 2 else -dvp)
            D = w * w + wp * wp - 2.0 * K["co1"] * abs(wp) * w
            far = far and si2 > rb * rb * D  # the line distance, a lower bound on the segment's
        if not far:
            pa = O if j == 0 else c + (ea * rho / vp[1]) * X + (eb * rho / vp[1]) * Yc
            pb = c + (na * rho / v[1]) * X + (nb * rho / v[1]) * Yc
            if not seg_clear(pa[None], pb[None], K["lo"], K["hi"], np.array([m]))[0]:
                return False
        vp = v
        rp, dpa, dvp, ea, eb = r, dpb, dv, na, nb
    return True
