"""ctypes binding of the CPU restatement (oracle/restate/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB_DIR = os.path.join(ROOT, "oracle", "restate")
LIB_PATH = os.path.join(LIB_DIR, "liboracle.so")

_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")


class Camera(C.Structure):
    _fields_ = [("hFov", C.c_double), ("vFov", C.c_double), ("nClip", C.c_double), ("fClip", C.c_double),
                ("pos", C.c_double * 3), ("c2w", C.c_double * 9), ("lensRadius", C.c_double),
                ("focalDistance", C.c_double)]


class Params(C.Structure):
    _fields_ = [("ns_aa", C.c_uint32), ("max_ray_depth", C.c_uint32), ("ns_area_light", C.c_uint32),
                ("samples_per_batch", C.c_uint32), ("max_tolerance", C.c_float),
                ("direct_hemisphere", C.c_uint32), ("seed", C.c_uint64), ("frame_w", C.c_uint32),
                ("frame_h", C.c_uint32), ("bh_center", C.c_double * 3), ("bh_radius", C.c_double),
                ("bh_dtheta", C.c_double), ("bh_kind", C.c_uint32), ("pad_", C.c_uint32), ("bh_spin", C.c_double),
                ("bh_axis", C.c_double * 3), ("illum", C.c_uint32), ("adaptive", C.c_uint32),
                ("thin_lens", C.c_uint32), ("env_hemi", C.c_uint32), ("microfacet_hemi", C.c_uint32),
                ("pad2_", C.c_uint32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", LIB_DIR], check=True, stdout=subprocess.DEVNULL)
        L = C.CDLL(LIB_PATH)
        L.ro_scene_load.restype = C.c_void_p
        L.ro_scene_load.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.ro_scene_free.argtypes = [C.c_void_p]
        L.ro_scene_num_prims.argtypes = [C.c_void_p]
        L.ro_scene_num_nodes.argtypes = [C.c_void_p]
        L.ro_scene_bvh.argtypes = [C.c_void_p, _f64p, _i32p, _u32p]
        L.ro_camera_load.argtypes = [C.c_char_p, C.POINTER(Camera), C.c_char_p, C.c_int]
        L.ro_params_default.argtypes = [C.POINTER(Params)]
        L.ro_render.argtypes = [C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint32, _f32p, _i32p, C.c_void_p, C.c_void_p, C.c_int]
        L.ro_pixel_key.restype = C.c_uint64
        L.ro_pixel_key.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.ro_keyed_rand.argtypes = [C.c_uint64, C.c_uint32]
        L.ro_micro_chain.argtypes = [_f64p, _f64p, _f64p, _f64p, C.c_int]
        L.ro_kerr_chain.argtypes = [_f64p, _f64p, _f64p, _f64p, C.c_int, _f64p]
        L.ro_kerr_chain_st.argtypes = [_f64p, _f64p, _f64p, _f64p, C.c_int, _f64p, C.c_double, _f64p]
        L.ro_shadow_query.argtypes = [C.c_void_p, C.POINTER(Params), _f64p, _f64p]
        L.ro_query.argtypes = [C.c_void_p, C.POINTER(Params), _f64p, _f64p, _f64p]
        L.ro_bbox_intersect.argtypes = [_f64p, _f64p, _f64p, _f64p, C.c_double, C.c_double,
                                        C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.ro_tri_intersect.argtypes = [_f64p, _f64p, _f64p, _f64p, C.POINTER(C.c_double), _f64p, _f64p]
        L.ro_sphere_intersect.argtypes = [_f64p, C.c_double, _f64p, _f64p, C.POINTER(C.c_double), _f64p,
                                          _f64p, C.c_int]
        L.ro_coord_space.argtypes = [_f64p, _f64p, _f64p, _f64p, _f64p]
        L.ro_sampler.argtypes = [C.c_int, _i32p, _f64p, C.POINTER(C.c_float), C.POINTER(C.c_int)]
        L.ro_bsdf_sample.argtypes = [C.c_int, _f64p, _f64p, _i32p, _f32p, _f64p, C.POINTER(C.c_float),
                                     C.POINTER(C.c_int), _f32p]
        L.ro_area_sample.argtypes = [_f32p, _f64p, _f64p, _i32p, _f32p, _f64p, C.POINTER(C.c_float),
                                     C.POINTER(C.c_float)]
        L.ro_light_sample.argtypes = [C.c_int, _f32p, _f64p, _f64p, _i32p, _f32p, _f64p, C.POINTER(C.c_float),
                                      C.POINTER(C.c_float), C.POINTER(C.c_int)]
        L.ro_camera_ray.argtypes = [C.c_double, C.c_double, _f64p, _f64p, C.c_double, C.c_double, C.c_double,
                                    C.c_double, _f64p, _f64p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.ro_scene_set_envmap.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
        L.ro_libm_eval.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long]
        _lib = L
    return _lib


class Scene:
    def __init__(self, path):
        err = C.create_string_buffer(256)
        self.h = lib().ro_scene_load(path.encode(), err, 256)
        if not self.h:
            raise RuntimeError(err.value.decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().ro_scene_free(self.h)
            self.h = None

    def set_envmap(self, texels):
        """texels: [h][w][3] float32 (HDRImageBuffer layout)."""
        t = np.ascontiguousarray(texels, np.float32)
        self._env = t
        rc = lib().ro_scene_set_envmap(self.h, t.shape[1], t.shape[0], t.ctypes.data)
        if rc != 0:
            raise RuntimeError("ro_scene_set_envmap failed")

    def bvh(self):
        n = lib().ro_scene_num_nodes(self.h)
        p = lib().ro_scene_num_prims(self.h)
        boxes = np.zeros((n, 6), np.float64)
        nodes = np.zeros((n, 4), np.int32)
        prims = np.zeros(p, np.uint32)
        lib().ro_scene_bvh(self.h, boxes, nodes, prims)
        return boxes, nodes, prims


def load_camera(path):
    cam = Camera()
    err = C.create_string_buffer(256)
    if lib().ro_camera_load(path.encode(), C.byref(cam), err, 256) != 0:
        raise RuntimeError(err.value.decode())
    return cam


def make_params(frame_w, frame_h, ns_aa=1, max_ray_depth=1, ns_area_light=1, samples_per_batch=32,
                max_tolerance=0.05, direct_hemisphere=False, seed=0, bh=(0.0, 1.0, 0.0, 0.1, 0.1), kerr=None,
                illum=2, adaptive=True, thin_lens=False, env_hemi=False, microfacet_hemi=False):
    """kerr: None (Schwarzschild) or (spin a/M, (ax, ay, az)) for the build-defined Kerr integrator.
    illum / adaptive / thin_lens / env_hemi / microfacet_hemi: the reference's compile-time switches
    (ILLUM, ADAPTIVE, THIN_LENS pathtracer.h:4-6, ENV_HEMI environment_light.h:4, MICROFACET_HEMI
    bsdf.h:4), defaults as the reference build."""
    p = Params()
    lib().ro_params_default(C.byref(p))
    p.ns_aa, p.max_ray_depth, p.ns_area_light = ns_aa, max_ray_depth, ns_area_light
    p.samples_per_batch, p.max_tolerance = samples_per_batch, max_tolerance
    p.direct_hemisphere, p.seed, p.frame_w, p.frame_h = int(direct_hemisphere), seed, frame_w, frame_h
    p.bh_center[0], p.bh_center[1], p.bh_center[2] = bh[0], bh[1], bh[2]
    p.bh_radius, p.bh_dtheta = bh[3], bh[4]
    if kerr is not None:
        p.bh_kind, p.bh_spin = 1, kerr[0]
        p.bh_axis[0], p.bh_axis[1], p.bh_axis[2] = kerr[1]
    p.illum, p.adaptive, p.thin_lens = illum, int(adaptive), int(thin_lens)
    p.env_hemi, p.microfacet_hemi = int(env_hemi), int(microfacet_hemi)
    return p


def kerr_chain(bh, spin, axis, o, d, max_rows=64):
    """The Kerr march of one ray: rows of (o3, d3, max_t, captured, q3, p3), and the frame (ex, ey, ez)."""
    b = np.array(list(bh) + [spin] + list(axis), np.float64)
    out = np.zeros((max_rows, 14), np.float64)
    frame = np.zeros(9, np.float64)
    n = lib().ro_kerr_chain(b, np.asarray(o, np.float64), np.asarray(d, np.float64), out, max_rows, frame)
    return out[:n], frame.reshape(3, 3)


def kerr_chain_st(bh, spin, axis, o, d, st, max_rows=64):
    """kerr_chain with steps st times longer (the Kerr occlusion proof's coarse march): rows as
    kerr_chain's and extra [n, 4] = (swept polar angle after the step, segment end point)."""
    b = np.array(list(bh) + [spin] + list(axis), np.float64)
    out = np.zeros((max_rows, 14), np.float64)
    extra = np.zeros((max_rows, 4), np.float64)
    frame = np.zeros(9, np.float64)
    n = lib().ro_kerr_chain_st(b, np.asarray(o, np.float64), np.asarray(d, np.float64), out, max_rows, frame, st,
                               extra)
    return out[:n], extra[:n]


def shadow_query(scene, params, o, d):
    """BVHAccel::intersect's boolean for the ray (o, d) under params' spacetime (restatement)."""
    return bool(lib().ro_shadow_query(scene.h, C.byref(params), np.asarray(o, np.float64), np.asarray(d, np.float64)))


def query(scene, params, o, d):
    """The reference's closest-hit query of one ray: (hit, hit_p [3], n [3], bsdf)."""
    out = np.zeros(7)
    h = lib().ro_query(scene.h, C.byref(params), np.ascontiguousarray(o, np.float64),
                       np.ascontiguousarray(d, np.float64), out)
    return bool(h), out[:3].copy(), out[3:6].copy(), int(out[6])


def render(scene, cam, params, x0, y0, w, h, threads=None, counters=False):
    threads = threads or os.cpu_count() or 1
    rgb = np.zeros((h, w, 3), np.float32)
    cnt = np.zeros((h, w), np.int32)
    draws = np.zeros((h, w), np.uint32)
    ctr = np.zeros((h, w, 4), np.uint32) if counters else None
    rc = lib().ro_render(scene.h, C.byref(cam), C.byref(params), x0, y0, w, h, rgb, cnt,
                         draws.ctypes.data, ctr.ctypes.data if counters else None, threads)
    if rc != 0:
        raise RuntimeError("ro_render failed")
    return rgb, cnt, draws, ctr


LIBM_FN = {"sin": 0, "cos": 1, "acos": 2, "atan2": 3, "sinf": 4, "cosf": 5, "exp": 6, "log": 7, "erf": 8, "atan": 9,
           "tan": 10}


def libm_eval(fn, a, b=None):
    """The host C library's `fn` (what the reference calls) on float64 arrays a (, b)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty_like(a)
    lib().ro_libm_eval(LIBM_FN[fn], a.ctypes.data, None if b is None else b.ctypes.data, out.ctypes.data, a.size)
    return out
