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


# ------------------------------------------------------------------------------------------
# cfg5 (BASELINE.json configs[4]): HDR environment map.  SURVEY.md 8(d): a synthetic 1024x512
# equirectangular f32 RGB map -- analytic sky gradient plus a sun disc, no randomness -- passed
# with `-e`.  Texel (x, y) covers the direction EnvironmentLight::theta_phi_to_dir gives for
# theta = (y + 0.5) / h * pi, phi = (x + 0.5) / w * 2 pi (environment_light.cpp:96-106).
SUN_DIR = np.array([0.45, 0.62, -0.64]) / np.linalg.norm([0.45, 0.62, -0.64])


def sky_texels(w=1024, h=512):
    """[h][w][3] float32 radiance: zenith-to-horizon blue gradient, a warm horizon band, a dark
    ground below the horizon and a 3-degree sun disc of radiance 60."""
    theta = (np.arange(h, dtype=np.float64) + 0.5) / h * np.pi
    phi = (np.arange(w, dtype=np.float64) + 0.5) / w * 2 * np.pi
    T, P = np.meshgrid(theta, phi, indexing="ij")
    d = np.stack([np.cos(P - np.pi) * np.sin(T), np.cos(T), -np.sin(P - np.pi) * np.sin(T)], -1)
    up = d[..., 1]
    zen = np.array([0.25, 0.45, 1.10])
    hor = np.array([1.00, 0.85, 0.70])
    ground = np.array([0.12, 0.10, 0.08])
    a = np.clip(up, 0.0, 1.0)[..., None]
    sky = hor * (1 - a) ** 3 + zen * (1 - (1 - a) ** 3)
    img = np.where(up[..., None] >= 0, sky, ground * (0.6 + 0.4 * np.exp(up[..., None] * 4)))
    cosang = d @ SUN_DIR
    sun = cosang > np.cos(np.radians(3.0))
    img = np.where(sun[..., None], np.array([60.0, 55.0, 45.0]), img)
    return np.ascontiguousarray(img.astype(np.float32))


def write_exr(path, rgb):
    """Single-part scanline OpenEXR, no compression, FLOAT channels B, G, R (what the reference's
    tinyexr and rrt_exr_load both read).  Returns the file's SHA-256."""
    import struct
    h, w, _ = rgb.shape

    def attr(name, typ, val):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(val)) + val
    ch = b"".join(n + b"\0" + struct.pack("<iB3xii", 2, 0, 1, 1) for n in (b"B", b"G", b"R")) + b"\0"
    box = struct.pack("<4i", 0, 0, w - 1, h - 1)
    hdr = (struct.pack("<II", 20000630, 2) + attr("channels", "chlist", ch) + attr("compression", "compression", b"\0")
           + attr("dataWindow", "box2i", box) + attr("displayWindow", "box2i", box)
           + attr("lineOrder", "lineOrder", b"\0") + attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
           + attr("screenWindowCenter", "v2f", b"\0" * 8) + attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
           + b"\0")
    row_bytes = w * 12
    base = len(hdr) + 8 * h
    table = b"".join(struct.pack("<Q", base + y * (8 + row_bytes)) for y in range(h))
    rows = []
    for y in range(h):
        rows.append(struct.pack("<ii", y, row_bytes) + rgb[y, :, 2].tobytes() + rgb[y, :, 1].tobytes()
                    + rgb[y, :, 0].tobytes())
    data = hdr + table + b"".join(rows)
    with open(path, "wb") as f:
        f.write(data)
    return hashlib.sha256(data).hexdigest()


def write_cfg5_envmap(path, w=1024, h=512):
    return write_exr(path, sky_texels(w, h))
