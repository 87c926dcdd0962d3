#!/usr/bin/env python3
"""Diagnostic (CPU, numpy): march a sample of camera rays of a golden case through the reference's
geodesic stepper and BVH walk, and report per-segment work statistics -- box tests per micro
segment, where they happen, and how many a walk started below the root would save.  Used to
choose traversal optimisations; not a parity tool (the oracle is)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(ROOT, "relativistic-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rrt  # noqa: E402
from golden_cases import Case  # noqa: E402
from test_capi_host import _scene_prims  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="cfg3_bunny_1080p_s64")
    ap.add_argument("--stride", type=int, default=12)
    a = ap.parse_args()
    c = Case(a.case)
    ctx = rrt.Renderer(-1)
    ctx.set_scene(rrt.SceneFile(c.scene_path))
    boxes, nodes, prims = ctx.bvh()
    nn = len(nodes)
    first, count, left, right = nodes[:, 0], nodes[:, 1], nodes[:, 2], nodes[:, 3]
    skip = np.full(nn, -1, np.int64)
    for i in range(nn):
        if count[i] == 0:
            skip[left[i]] = right[i]
            skip[right[i]] = skip[i]
    depth = np.zeros(nn, np.int64)
    parent = np.full(nn, -1, np.int64)
    for i in range(nn):
        if count[i] == 0:
            for ch in (left[i], right[i]):
                depth[ch] = depth[i] + 1
                parent[ch] = i
    tris, sph = _scene_prims(c.scene_path)
    assert len(sph) == 0
    T = tris[prims.astype(np.int64)]  # leaf-slot order
    p0, e1, e2 = T[:, 0], T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]
    cam = rrt.load_camera(c.camera_path)
    pos = np.array(cam.pos)
    c2w = np.array(cam.c2w).reshape(3, 3)
    blx = -np.tan(cam.hFov * (np.pi / 180) / 2)
    bly = -np.tan(cam.vFov * (np.pi / 180) / 2)
    W, H = c.frame_w, c.frame_h
    xs, ys = np.meshgrid(np.arange(0, W, a.stride) + 0.5, np.arange(0, H, a.stride) + 0.5)
    cx, cy = xs.ravel() / W, ys.ravel() / H
    v = np.stack([(1 - cx) * blx + cx * -blx, (1 - cy) * bly + cy * -bly, -np.ones_like(cx)], 1)
    w = v @ c2w.T
    d = w / np.linalg.norm(w, axis=1, keepdims=True)
    o = np.repeat(pos[None], len(d), 0)
    bh = c.cfg["bh"]
    C0, rs, dt = np.array(bh[:3]), bh[3], bh[4]
    steps = int(np.ceil(2 * np.pi / dt - 1e-12))
    n = len(d)
    mt = np.zeros(n)
    alive = np.ones(n, bool)
    seg_tests, seg_len, seg_o, seg_ray, seg_minleafdepth, seg_lca_tests = [], [], [], [], [], []
    for j in range(steps):
        idx = np.nonzero(alive)[0]
        if len(idx) == 0:
            break
        oo, dd, mm = o[idx], d[idx], mt[idx]
        no = oo + dd * mm[:, None]
        x = no - C0
        dist = np.linalg.norm(x, axis=1)
        x = x / dist[:, None]
        u = 1 / dist
        dx = (dd * x).sum(1)
        y = dd - dx[:, None] * x
        dy = np.linalg.norm(y, axis=1)
        y = y / dy[:, None]
        up = -u * dx / dy
        k = 3 * rs
        f1 = -u + k * u * u / 2
        u2 = u + up * dt / 2
        f2 = -u2 + k * u2 * u2 / 2
        u3 = u + up * dt / 2 + f1 * dt * dt / 4
        f3 = -u3 + k * u3 * u3 / 2
        u = u + up * dt + (f1 + f2 + f3) * dt * dt / 6
        ddn = 1 / u
        nd = (C0 + (ddn * np.cos(dt))[:, None] * x + (ddn * np.sin(dt))[:, None] * y) - no
        mt2 = np.linalg.norm(nd, axis=1)
        d2 = nd / mt2[:, None]
        o[idx], d[idx], mt[idx] = no, d2, mt2
        # capture
        tmp = no - C0
        b = 2 * (tmp * d2).sum(1)
        cc = (tmp * tmp).sum(1) - rs * rs
        disc = b * b - 4 * cc
        sq = np.sqrt(np.maximum(disc, 0))
        t1, t2 = (-b - sq) / 2, (-b + sq) / 2
        cap = (disc >= 0) & (((t1 >= 0) & (t1 <= mt2)) | ((t2 >= 0) & (t2 <= mt2)))
        alive[idx[cap]] = False
        idx2 = idx[~cap]
        # walk (vectorised SIMT over segments)
        so, sd, st = o[idx2], d[idx2], mt[idx2].copy()
        node = np.zeros(len(idx2), np.int64)
        tests = np.zeros(len(idx2), np.int64)
        hit = np.zeros(len(idx2), bool)
        minleaf = np.full(len(idx2), 99, np.int64)
        passed_leaves = [[] for _ in range(len(idx2))]
        with np.errstate(divide="ignore", invalid="ignore"):
            while True:
                act = np.nonzero(node >= 0)[0]
                if len(act) == 0:
                    break
                nd_ = node[act]
                bx = boxes[nd_]
                t0 = (bx[:, :3] - so[act]) / sd[act]
                t1_ = (bx[:, 3:] - so[act]) / sd[act]
                tmin = np.minimum(t0, t1_).max(1)
                tmax = np.maximum(t0, t1_).min(1)
                ok = (tmin <= tmax) & (tmin <= st[act]) & (tmax >= 0)
                tests[act] += 1
                leaf = count[nd_] > 0
                nxt = np.where(ok & ~leaf, nd_ + 1, skip[nd_])
                for q in np.nonzero(ok & leaf)[0]:
                    r = act[q]
                    passed_leaves[r].append(nd_[q])
                    minleaf[r] = min(minleaf[r], depth[nd_[q]])
                    for s in range(first[nd_[q]], first[nd_[q]] + count[nd_[q]]):
                        s1 = np.cross(sd[r], e2[s])
                        s0 = so[r] - p0[s]
                        s2 = np.cross(s0, e1[s])
                        den = s1 @ e1[s]
                        if den == 0:
                            continue
                        inv = 1.0 / den
                        tt, bb1, bb2 = (s2 @ e2[s]) * inv, (s1 @ s0) * inv, (s2 @ sd[r]) * inv
                        if 0 <= tt <= st[r] and bb1 >= 0 and bb2 >= 0 and 1 - bb1 - bb2 >= 0:
                            st[r] = tt
                            hit[r] = True
                node[act] = nxt
        # LCA of passing leaves: tests of a walk over that subtree only
        for r in range(len(idx2)):
            L = passed_leaves[r]
            if not L:
                seg_lca_tests.append(0)
                continue
            anc = set()
            a0 = L[0]
            while a0 >= 0:
                anc.add(a0)
                a0 = parent[a0]
            lca = L[0]
            for l2 in L[1:]:
                a1 = l2
                while a1 not in anc:
                    a1 = parent[a1]
                # keep the deepest common ancestor
                while lca not in _anc(a1, parent):
                    lca = parent[lca]
            seg_lca_tests.append(_subtree_tests(lca, so[r], sd[r], mt[idx2[r]], boxes, count, skip))
        alive[idx2[hit]] = False
        seg_tests.append(tests)
        seg_len.append(mt[idx2])
        seg_o.append(so)
        seg_ray.append(idx2)
        seg_minleafdepth.append(minleaf)
    tests = np.concatenate(seg_tests)
    ln = np.concatenate(seg_len)
    so = np.concatenate(seg_o)
    lca_t = np.array(seg_lca_tests)
    rb = boxes[0]
    inside = np.all((so >= rb[:3]) & (so <= rb[3:]), 1)
    print(f"rays {n}, segments {len(tests)} ({len(tests) / n:.1f}/ray), box tests {tests.sum()} "
          f"({tests.sum() / n:.1f}/ray, {tests.mean():.2f}/segment)")
    print(f"segments starting inside root box: {inside.mean():.3f}, their tests: {tests[inside].sum() / tests.sum():.3f}")
    for lo, hi in [(1, 1), (2, 4), (5, 10), (11, 20), (21, 40), (41, 1000)]:
        m = (tests >= lo) & (tests <= hi)
        print(f"  segments with {lo}-{hi} tests: {m.mean():.3f} of segments, {tests[m].sum() / tests.sum():.3f} of tests, "
              f"mean len {ln[m].mean() if m.any() else 0:.3f}")
    print(f"walk from the LCA of passing leaves: {lca_t.sum()} tests ({lca_t.sum() / tests.sum():.3f} of root walks)")
    np.savez("/tmp/segstats.npz", tests=tests, ln=ln, so=so, lca=lca_t)


_anc_cache = {}


def _anc(a, parent):
    s = set()
    while a >= 0:
        s.add(a)
        a = parent[a]
    return s


def _subtree_tests(top, o, d, mt, boxes, count, skip):
    end = skip[top]
    node, t = top, 0
    with np.errstate(divide="ignore", invalid="ignore"):
        while node >= 0 and node != end:
            bx = boxes[node]
            t0 = (bx[:3] - o) / d
            t1 = (bx[3:] - o) / d
            tmin = np.minimum(t0, t1).max()
            tmax = np.maximum(t0, t1).min()
            ok = (tmin <= tmax) & (tmin <= mt) & (tmax >= 0)
            t += 1
            node = node + 1 if (ok and count[node] == 0) else skip[node]
    return t


if __name__ == "__main__":
    main()
