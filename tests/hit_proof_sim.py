"""numpy mirror of the camera-ray hit proof (relativistic-ray-tracer_amd/csrc/rrt_device.h
camera_hit_proof) and of the zero-sample proof built on it (rrt_sample.hip zero_sample_proof).

TEST INFRASTRUCTURE ONLY (tests/test_hit_proof.py, tools/hit_proof_sweep.py): the product runs the
HIP version.

The reference's closest-hit query (bvh.cpp:103-113) returns the first micro segment's closest hit.
The proof marches the shadow proof's planar recurrence from the camera ray itself (A = o) and accepts
"the query hits kept face triangle T at Q" when, with the shadow proof's margin m at every segment:
  * every segment up to the crossing clears the capture sphere (capture would end the query first);
  * every segment clears the box holding every primitive but the kept face triangles;
  * every kept face triangle of a face that a segment end is past is certainly untouched by that
    segment (ends > m on one side of its plane, or its plane crossing mq outside an edge), except
    one -- T -- which the crossing segment certainly crosses (ends > m on either side, the crossing
    point mq inside every edge) and which is not a light.
The reference's segment is then within the recurrence's deviation of this one, crosses T first, and
its hit point is within that deviation of Q.
"""
import numpy as np

from miss_proof_sim import ETA, KAPPA, _step0, seg_clear


def nocc_box(T, faces, spheres=()):
    """rrt_host.cpp build_occluders' box of every primitive but the kept face triangles: the other
    triangles of T and the spheres [(centre, radius)]."""
    kept = {t[4] for f in faces for t in f}
    rest = np.array([i for i in range(len(T)) if i not in kept], np.int64)
    pts = [T[rest].reshape(-1, 3)] if len(rest) else []
    for cen, rad in spheres:
        pts.append(np.array([np.asarray(cen) - rad, np.asarray(cen) + rad]))
    if not pts:
        return np.full(3, np.inf), np.full(3, -np.inf)
    P = np.concatenate(pts)
    return P.min(0), P.max(0)


def touch(tri, a, b, m):
    """occ_touch: 2 certain crossing (with the crossing point), 0 certainly untouched, 1 uncertain."""
    n, d, en, eo, _ = tri
    da = n @ a - d
    db = n @ b - d
    if (da > m and db > m) or (da < -m and db < -m):
        return 0, None
    if not ((da > m and db < -m) or (da < -m and db > m)):
        return 1, None
    q = a + (b - a) * (da / (da - db))
    mq = m * (2.0 + np.abs(b - a).sum() / abs(da - db))
    e = np.array([en[k] @ q - eo[k] for k in range(3)])
    if np.all(e >= mq):
        return 2, q
    if np.any(e <= -mq):
        return 0, None
    return 1, None


def prove(K, faces, box, emit, nlo, nhi, o, d):
    """One camera ray: (proven, hit triangle index, Q, step)."""
    c = K["c"]
    X, Y, u0, up0, _, _ = _step0(K, o[None], d[None])
    X, Y, u0, up0 = X[0], Y[0], float(u0[0]), float(up0[0])
    vprev = K["rho"] * u0
    s = u0 * K["co1"] - up0 * K["si"] / K["rho"]
    ea, eb, sig, rp = 1.0, 0.0, 1.0, 1.0 / u0
    lo, hi = box
    a_in = bool(np.all(o >= lo) and np.all(o <= hi))
    a_room = bool(np.all(o >= K["lo"]) and np.all(o <= K["hi"]))
    si2 = K["si"] * K["si"]
    rc = K["r"] * (1.0 + 1e-9)
    pa = o.copy()
    for j in range(K["steps"]):
        sg = -1.0 if vprev < 0.0 else 1.0
        up = (vprev * K["co1"] - K["rho"] * s) / K["si"]
        s = abs(vprev) / K["rho"]
        f1 = -s + K["k15"] * s * s
        u2 = s + up * (K["dt"] * 0.5)
        f2 = -u2 + K["k15"] * u2 * u2
        u3 = u2 + f1 * (K["dt"] * K["dt"] / 4.0)
        f3 = -u3 + K["k15"] * u3 * u3
        v = s + up * K["dt"] + (f1 + f2 + f3) * (K["dt"] * K["dt"] / 6.0)
        if not abs(v) >= KAPPA * (s + abs(up) * K["dt"]):
            return False, -1, None, j
        a_, b_ = sg * K["co1"], sig * K["si1"]
        na, nb = a_ * ea - b_ * eb, a_ * eb + b_ * ea
        sig *= sg
        av, avp = abs(v), abs(vprev)
        r = K["rho"] / av * (1.0 + 1e-6)
        m = ETA * (max(rp, r) + K["scale"])
        rb = rc + m
        D = v * v + vprev * vprev - 2.0 * K["co1"] * avp * v
        inside = v * (K["co1"] * avp - v) < 0.0 and avp * (avp - K["co1"] * v) > 0.0
        clear = si2 > rb * rb * D if inside else K["rho"] ** 2 > rb * rb * max(v * v, vprev * vprev)
        if not clear:
            return False, -1, None, j
        pb = c + (na * K["rho"] / v) * X + (nb * K["rho"] / v) * Y
        b_in = bool(np.all(pb >= lo) and np.all(pb <= hi))
        found, q_found = None, None
        if not (a_in and b_in):
            for k in range(3):
                for f, past in ((k, not (pb[k] >= lo[k] and pa[k] >= lo[k])), (k + 3, not (pb[k] <= hi[k] and pa[k] <= hi[k]))):
                    if not past:
                        continue
                    for i, tri in enumerate(faces[f]):
                        res, q = touch(tri, pa, pb, m)
                        if res == 1:
                            return False, -1, None, j
                        if res == 2:
                            if found is not None:
                                return False, -1, None, j
                            found, q_found = (f, i), q
        if not seg_clear(pa[None], pb[None], nlo, nhi, np.array([m]))[0]:
            return False, -1, None, j
        if found is not None:
            f, i = found
            if (emit[f] >> i) & 1:
                return False, -1, None, j
            return True, faces[f][i][4], q_found, j
        b_room = bool(np.all(pb >= K["lo"]) and np.all(pb <= K["hi"]))
        if a_room and not b_room:
            return False, -1, None, j  # leaving the room without a crossing
        a_in, a_room = b_in, b_room
        pa = pb
        rp, vprev, ea, eb = r, v, na, nb
    return False, -1, None, K["steps"]
