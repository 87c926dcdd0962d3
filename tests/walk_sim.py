"""Scalar Python restatement of the two BVH walks, for host-side tests and diagnostics.

reference_walk: BVHAccel::intersect_micro (bvh.cpp:115-138) over the reference tree -- left-first,
every accepted primitive shrinks max_t (t <= max_t: a later equal t wins).
clean_walk: rrt_device.h traverse_clean over the clean tree plus the oversized-leaf list.
search: rrt_device.h traverse_free -- the SAH search tree's walk at the full max_t, then the ordered
replay of the accepted primitives in windows of `window` slots.
Both use IEEE double arithmetic with the reference's operation order (Python floats), and
std::min/max semantics, so their answers can be compared exactly."""
import numpy as np


def _mn(a, b):
    return b if b < a else a


def _mx(a, b):
    return b if a < b else a


def slab(box, o, d, max_t):
    t = []
    for k in range(3):
        try:
            t0 = (box[k] - o[k]) / d[k]
            t1 = (box[3 + k] - o[k]) / d[k]
        except ZeroDivisionError:  # IEEE: x / 0 -> +-inf or nan
            a, b = box[k] - o[k], box[3 + k] - o[k]
            s = np.copysign(1.0, d[k])
            t0 = float("nan") if a == 0 else s * np.copysign(np.inf, a)
            t1 = float("nan") if b == 0 else s * np.copysign(np.inf, b)
        t.append((t0, t1))
    tmin = _mx(_mx(_mn(*t[0]), _mn(*t[1])), _mn(*t[2]))
    tmax = _mn(_mn(_mx(*t[0]), _mx(*t[1])), _mx(*t[2]))
    return tmin <= tmax and tmin <= max_t and tmax >= 0.0


def tri(p0, e1, e2, o, d, max_t):
    """Triangle::intersect (triangle.cpp:25-55): (t, b1, b2) or None."""
    s = [o[k] - p0[k] for k in range(3)]
    s1 = (d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0])
    s2 = (s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0])
    den = s1[0] * e1[0] + s1[1] * e1[1] + s1[2] * e1[2]
    if den == 0:
        return None
    inv = 1.0 / den
    t = (s2[0] * e2[0] + s2[1] * e2[1] + s2[2] * e2[2]) * inv
    b1 = (s1[0] * s[0] + s1[1] * s[1] + s1[2] * s[2]) * inv
    b2 = (s2[0] * d[0] + s2[1] * d[1] + s2[2] * d[2]) * inv
    b0 = 1 - b1 - b2
    if 0.0 <= t <= max_t and b0 >= 0 and b1 >= 0 and b2 >= 0:
        return t, b1, b2
    return None


class Walker:
    def __init__(self, boxes, nodes, geo, clean=None):
        """boxes/nodes: rrt.Renderer.bvh() (nodes = first, count, left, right); geo: [slots, 9]
        (p0, e1, e2 per leaf slot, triangles only); clean: rrt.Renderer.clean_tree()."""
        self.boxes = [tuple(b) for b in boxes]
        self.first, self.count = nodes[:, 0].tolist(), nodes[:, 1].tolist()
        n = len(nodes)
        self.skip = [-1] * n
        for i in range(n):
            if self.count[i] == 0:
                self.skip[nodes[i, 2]] = int(nodes[i, 3])
                self.skip[nodes[i, 3]] = self.skip[i]
        self.geo = [tuple(g) for g in geo]
        if clean is not None:
            cb, cn, bb, bg = clean
            self.cboxes = [tuple(b) for b in cb]
            self.cnodes = [tuple(int(v) for v in r) for r in cn]
            self.big = [(tuple(bb[i]), int(bg[i, 0]), int(bg[i, 1]), int(bg[i, 2])) for i in range(len(bg))]

    def set_search_tree(self, st):
        """st: rrt.Renderer.search_tree() -> (boxes, nodes (skip, first, count, ordinal))."""
        boxes, nodes = st
        self.sboxes = [tuple(b) for b in boxes]
        self.snodes = [tuple(int(v) for v in r) for r in nodes]
        # the oversized leaves that joined the search tree (rrt_host.cpp build_free_tree: the local
        # ones) leave the walk's list
        inside = {(f, c) for _, f, c, _ in self.snodes if c > 0}
        self.big_all = self.big
        self.big = [b for b in self.big if (b[1], b[2]) not in inside]

    def _tri_or_sphere(self, s, o, d, max_t):
        g = self.geo[s]
        return tri(g[0:3], g[3:6], g[6:9], o, d, max_t)

    def search(self, o, d, max_t, window=4, any_hit=False):
        """traverse_free: (slot, t) of the closest hit (or (-1, max_t)), and the box tests."""
        tests = 1
        if not slab(self.boxes[0], o, d, max_t):
            return -1, max_t, tests
        L = max_t
        e = tuple(o[k] + d[k] * L for k in range(3))
        m, hit, after, cut, cut_pass = L, -1, -1, None, False
        self.windows = 0
        while True:
            self.windows += 1
            acc = []  # (slot, leaf ref) accepted at L with slot > after

            def take(first, count, ref):
                for s in range(first, first + count):
                    if s <= after or not self._may(s, o, e):
                        continue
                    if self._tri_or_sphere(s, o, d, L) is not None:
                        acc.append((s, ref))

            for bi, (box, first, count, _) in enumerate(self.big):
                if any(self._may(s, o, e) for s in range(first, first + count)):
                    tests += 1
                    if slab(box, o, d, L):
                        take(first, count, ("big", bi))
            node = 0
            while node >= 0:
                tests += 1
                skip, first, count, _ = self.snodes[node]
                if not slab(self.sboxes[node], o, d, L):
                    node = skip
                    continue
                if count == 0:
                    node += 1
                    continue
                take(first, count, ("tree", node))
                node = skip
            if any_hit:
                return (acc[0][0] if acc else -1), L, tests
            if not acc:
                break
            acc.sort()
            more = len(acc) > window
            acc = acc[:window]
            cur, passed = None, False
            for s, ref in acc:
                if ref != cur:
                    cur = ref
                    if ref == cut and after >= 0:
                        passed = cut_pass
                    else:
                        box = self.big[ref[1]][0] if ref[0] == "big" else self.sboxes[ref[1]]
                        passed = slab(box, o, d, m)
                if not passed:
                    continue
                r = self._tri_or_sphere(s, o, d, m)
                if r is not None:
                    m, hit = r[0], s
            if not more:
                break
            after, cut, cut_pass = acc[-1][0], acc[-1][1], passed
        return hit, m, tests

    def planes(self, eps):
        """Supporting planes for the cull of rrt_device.h plane_may_hit (rrt_host.cpp)."""
        self.eps = eps
        self.pl = []
        for g in self.geo:
            e1, e2 = g[3:6], g[6:9]
            nn = (e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0])
            nl = (nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]) ** 0.5
            l1 = (e1[0] ** 2 + e1[1] ** 2 + e1[2] ** 2) ** 0.5
            l2 = (e2[0] ** 2 + e2[1] ** 2 + e2[2] ** 2) ** 0.5
            if nl >= 1e-6 * l1 * l2:
                n = (nn[0] / nl, nn[1] / nl, nn[2] / nl)
                self.pl.append((n, n[0] * g[0] + n[1] * g[1] + n[2] * g[2]))
            else:
                self.pl.append(((0.0, 0.0, 0.0), 0.0))

    def _may(self, s, o, e):
        n, c = self.pl[s]
        a = (n[0] * o[0] + n[1] * o[1] + n[2] * o[2]) - c
        b = (n[0] * e[0] + n[1] * e[1] + n[2] * e[2]) - c
        return not ((a > self.eps and b > self.eps) or (a < -self.eps and b < -self.eps))

    culled = 0

    def _leaf(self, first, count, o, d, st, e=None):
        for s in range(first, first + count):
            if e is not None and not self._may(s, o, e):
                self.culled += 1
                continue
            g = self.geo[s]
            r = tri(g[0:3], g[3:6], g[6:9], o, d, st[0])
            if r is not None:
                st[0] = r[0]
                st[1] = s

    def reference(self, o, d, max_t):
        st = [max_t, -1]
        node, tests = 0, 0
        while node >= 0:
            tests += 1
            if not slab(self.boxes[node], o, d, st[0]):
                node = self.skip[node]
                continue
            if self.count[node] == 0:
                node += 1
                continue
            self._leaf(self.first[node], self.count[node], o, d, st)
            node = self.skip[node]
        return st[1], st[0], tests

    def clean(self, o, d, max_t, cull=False):
        st = [max_t, -1]
        tests = 1
        self.culled = 0
        if not slab(self.boxes[0], o, d, st[0]):
            return -1, max_t, tests
        e = tuple(o[k] + d[k] * max_t for k in range(3)) if cull else None
        bi, node = 0, 0
        while True:
            lim = self.cnodes[node][3] if node >= 0 else 1 << 62
            while bi < len(self.big) and self.big[bi][3] < lim:
                box, first, count, _ = self.big[bi]
                if e is None or any(self._may(s, o, e) for s in range(first, first + count)):
                    tests += 1
                    if slab(box, o, d, st[0]):
                        self._leaf(first, count, o, d, st, e)
                bi += 1
            if node < 0:
                break
            skip, first, count, _ = self.cnodes[node]
            tests += 1
            if not slab(self.cboxes[node], o, d, st[0]):
                node = skip
                continue
            if count == 0:
                node += 1
                continue
            self._leaf(first, count, o, d, st, e)
            node = skip
        return st[1], st[0], tests
