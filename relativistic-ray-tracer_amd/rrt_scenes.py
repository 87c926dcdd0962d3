"""Synthetic scene assets for the BASELINE configs the reference's own assets cannot cover.

cfg4 (BASELINE.json configs[3]) names CBdragon.dae, which the reference does not ship
(`.MISSING_LARGE_BLOBS`).  SURVEY.md 8(d) substitutes a committed, deterministic mesh of the
same size: a (2,3) torus knot tube, 1000 segments x 50 sides = 100,000 triangles, Lambertian
0.6, fitted inside [-0.6,0.6] x [0.05,0.8] x [-0.6,0.6] (clear of the hole at y = 1 +- 0.1) and
inserted into CBempty.dae's Cornell box.  The result is an ordinary COLLADA file, so the
reference's own loader (oracle harness) and the native ingest (rrt_collada_load) read the SAME
bytes; tests pin its SHA-256 so a different libm or numpy cannot silently change the scene.
No randomness.
"""
import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CBEMPTY = os.path.join(HERE, "..", "tests", "golden", "dae", "CBempty.dae")


def _fmt(v):
    # shortest decimal that reads back (strtof) to the same float32
    return np.format_float_positional(np.float32(v), unique=True, trim="-")


def torus_knot_mesh(segments=1000, sides=50, p=2, q=3, tube=0.35):
    """Vertices (segments*sides, 3) float64 in WORLD coordinates and triangles (2*segments*sides, 3),
    consistently oriented (closed manifold tube)."""
    t = np.arange(segments, dtype=np.float64) * (2.0 * np.pi / segments)
    rr = 2.0 + np.cos(q * t)
    c = np.stack([rr * np.cos(p * t), rr * np.sin(p * t), np.sin(q * t)], 1)
    # derivatives (closed form) for a Frenet frame
    drr = -q * np.sin(q * t)
    d1 = np.stack([drr * np.cos(p * t) - rr * p * np.sin(p * t),
                   drr * np.sin(p * t) + rr * p * np.cos(p * t),
                   q * np.cos(q * t)], 1)
    d2rr = -q * q * np.cos(q * t)
    d2 = np.stack([d2rr * np.cos(p * t) - 2 * drr * p * np.sin(p * t) - rr * p * p * np.cos(p * t),
                   d2rr * np.sin(p * t) + 2 * drr * p * np.cos(p * t) - rr * p * p * np.sin(p * t),
                   -q * q * np.sin(q * t)], 1)
    T = d1 / np.linalg.norm(d1, axis=1, keepdims=True)
    N = d2 - (d2 * T).sum(1, keepdims=True) * T
    N /= np.linalg.norm(N, axis=1, keepdims=True)
    B = np.cross(T, N)
    th = np.arange(sides, dtype=np.float64) * (2.0 * np.pi / sides)
    ring = (np.cos(th)[None, :, None] * N[:, None, :] + np.sin(th)[None, :, None] * B[:, None, :])
    v = (c[:, None, :] + tube * ring).reshape(-1, 3)
    # fit: curve x,y in [-3-tube, 3+tube] -> world X,Z in [-0.6, 0.6]; curve z -> world Y around 0.425
    s = 0.6 / (3.0 + tube)
    world = np.stack([v[:, 0] * s, 0.425 + v[:, 2] * s, v[:, 1] * s], 1)
    i = np.arange(segments)[:, None]
    j = np.arange(sides)[None, :]
    a = i * sides + j
    b = ((i + 1) % segments) * sides + j
    cc = ((i + 1) % segments) * sides + (j + 1) % sides
    d = i * sides + (j + 1) % sides
    tri = np.concatenate([np.stack([a, b, cc], -1).reshape(-1, 3), np.stack([a, cc, d], -1).reshape(-1, 3)], 0)
    # interleave the two triangles of each quad (stable, deterministic order)
    n = segments * sides
    tri = np.stack([tri[:n], tri[n:]], 1).reshape(-1, 3)
    return world, tri


def cfg4_dae_text(segments=1000, sides=50):
    """CBempty.dae with the torus knot added as one more mesh node (Lambertian 0.6)."""
    base = open(CBEMPTY).read()
    world, tri = torus_knot_mesh(segments, sides)
    # CBempty is Z_UP: the parser pre-multiplies (x,y,z) -> (-x, z, y); store the inverse so the
    # world coordinates come out exactly (the identity node matrix and the +-1 swap are exact).
    local = np.stack([-world[:, 0], world[:, 2], world[:, 1]], 1)
    pos = " ".join(_fmt(x) for x in local.reshape(-1))
    idx = " ".join(str(int(k)) for k in tri.reshape(-1))
    nt = len(tri)
    geom = (f'    <geometry id="knot-mesh" name="knot">\n      <mesh>\n'
            f'        <source id="knot-mesh-positions">\n'
            f'          <float_array id="knot-mesh-positions-array" count="{local.size}">{pos}</float_array>\n'
            f'        </source>\n'
            f'        <vertices id="knot-mesh-vertices">\n'
            f'          <input semantic="POSITION" source="#knot-mesh-positions"/>\n        </vertices>\n'
            f'        <polylist material="knot-material" count="{nt}">\n'
            f'          <input semantic="VERTEX" source="#knot-mesh-vertices" offset="0"/>\n'
            f'          <vcount>{" ".join(["3"] * nt)}</vcount>\n          <p>{idx}</p>\n'
            f'        </polylist>\n      </mesh>\n    </geometry>\n')
    effect = ('    <effect id="knot-effect">\n      <profile_COMMON>\n        <technique sid="common">\n'
              '          <phong>\n            <diffuse>\n              <color sid="diffuse">0.6 0.6 0.6 1</color>\n'
              '            </diffuse>\n          </phong>\n        </technique>\n      </profile_COMMON>\n'
              '    </effect>\n')
    material = ('    <material id="knot-material" name="knot">\n'
                '      <instance_effect url="#knot-effect"/>\n    </material>\n')
    node = ('      <node id="knot" name="knot" type="NODE">\n'
            '        <matrix sid="transform">1 0 0 0 0 1 0 0 0 0 1 0 0 0 0 1</matrix>\n'
            '        <instance_geometry url="#knot-mesh">\n          <bind_material>\n'
            '            <technique_common>\n'
            '              <instance_material symbol="knot-material" target="#knot-material"/>\n'
            '            </technique_common>\n          </bind_material>\n        </instance_geometry>\n'
            '      </node>\n')
    for tag, add in (("  </library_effects>", effect), ("  </library_materials>", material),
                     ("  </library_geometries>", geom)):
        assert base.count(tag) == 1, tag
        base = base.replace(tag, add + tag)
    end_vs = "    </visual_scene>"
    assert base.count(end_vs) == 1
    return base.replace(end_vs, node + end_vs)


def write_cfg4_dae(path, segments=1000, sides=50):
    """Write the cfg4 scene; returns its SHA-256 (tests pin it)."""
    text = cfg4_dae_text(segments, sides).encode()
    with open(path, "wb") as f:
        f.write(text)
    return hashlib.sha256(text).hexdigest()
