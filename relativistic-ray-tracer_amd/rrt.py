"""ctypes binding of librrt.so (include/rrt.h) -- the host-side mirror of the reference's
PathTracer hot-path interface for Python callers (tests, bench, smoke).

The product path is native: librrt.so (HIP kernels + C ABI).  This module only marshals
arguments; it never computes radiance itself and raises if the library is missing.

Reference correspondence (pathtracer.h / pathtracer.cpp):
    Renderer(device)                  PathTracer ctor (pathtracer.cpp:32-85)
    .set_scene(SceneFile)             PathTracer::set_scene + build_accel (:95-117, :304-328)
    .set_camera(camera)               PathTracer::set_camera (:119-134)
    .set_black_hole(c, r_s, dtheta)   the `-B` override of global_black_hole (main.cpp:139-145)
    .render(params, x0, y0, w, h)     raytrace_tile / raytrace_cell over a region (:549-609)
    RenderParams(...)                 AppConfig fields (application.h:41-85)
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RRT_LIB") or os.path.join(HERE, "librrt.so")  # RRT_LIB: A/B of builds

RRT_OK, RRT_E_INVALID, RRT_E_HIP, RRT_E_CANCELLED, RRT_E_NO_DEVICE, RRT_E_IO = 0, -1, -2, -3, -4, -5
RRT_RENDER_COUNTERS, RRT_RENDER_DRAWS, RRT_RENDER_WAVEFRONT, RRT_RENDER_EXACT_DIV = 1, 2, 4, 8
RRT_RENDER_PIXEL_LOOP, RRT_RENDER_NO_SKIP, RRT_RENDER_NO_CLEAN, RRT_RENDER_PER_PIXEL = 16, 32, 64, 128
RRT_RENDER_COUNT_EXECUTED, RRT_RENDER_ORDERED, RRT_RENDER_NO_FIRST = 256, 512, 1024
RRT_RENDER_ONE_QUEUE, RRT_RENDER_XCD_QUEUES, RRT_RENDER_NO_MISS_PROOF, RRT_RENDER_PREPASS = 2048, 4096, 8192, 16384
RRT_RENDER_STRIPED_QUEUES, RRT_RENDER_NO_SHADOW_PROOF, RRT_RENDER_NO_PIXEL_PROOF = 1 << 15, 1 << 16, 1 << 17
RRT_RENDER_NO_SEARCH_TREE, RRT_RENDER_DEEP_SAMPLE, RRT_RENDER_NO_HEAVY, RRT_RENDER_HEAVY = 1 << 18, 1 << 19, 1 << 20, 1 << 21
RRT_RENDER_DIAG_NO_TRAVERSE, RRT_RENDER_DIAG_CLEAR_STATS = 1 << 30, 1 << 31
# the reference's compile-time switches (pathtracer.h:4-6, environment_light.h:4, bsdf.h:4) as flags
RRT_RENDER_THIN_LENS, RRT_RENDER_NO_ADAPTIVE, RRT_RENDER_ENV_HEMI, RRT_RENDER_MICROFACET_HEMI = 1 << 22, 1 << 23, 1 << 24, 1 << 25


def RRT_RENDER_ILLUM(n):
    """ILLUM n (pathtracer.h:4) as flag bits 26..27 (ILLUM 2, the default: 0)."""
    return ((n ^ 2) & 3) << 26


class RRTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rrt error {code}: {msg}")
        self.code = code


class DeviceCfg(C.Structure):
    _fields_ = [("device", C.c_int), ("free_grid_res", C.c_uint32), ("reserved", C.c_uint32 * 6)]


class CameraDesc(C.Structure):
    _fields_ = [("hFov", C.c_double), ("vFov", C.c_double), ("nClip", C.c_double), ("fClip", C.c_double),
                ("pos", C.c_double * 3), ("c2w", C.c_double * 9), ("lensRadius", C.c_double),
                ("focalDistance", C.c_double)]


class CameraState(C.Structure):
    """The full CGL::Camera record (Camera::dump_settings order; the .rrtc payload)."""
    _fields_ = [("hFov", C.c_double), ("vFov", C.c_double), ("ar", C.c_double), ("nClip", C.c_double),
                ("fClip", C.c_double), ("pos", C.c_double * 3), ("targetPos", C.c_double * 3), ("phi", C.c_double),
                ("theta", C.c_double), ("r", C.c_double), ("minR", C.c_double), ("maxR", C.c_double),
                ("c2w", C.c_double * 9), ("screenW", C.c_double), ("screenH", C.c_double),
                ("screenDist", C.c_double), ("focalDistance", C.c_double), ("lensRadius", C.c_double)]

    def to_array(self):
        return np.frombuffer(bytes(self), np.float64).copy()


class ColladaOptions(C.Structure):
    _fields_ = [("screen_w", C.c_uint32), ("screen_h", C.c_uint32), ("lens_radius", C.c_double),
                ("focal_distance", C.c_double), ("reserved", C.c_uint32 * 4)]


class EnvmapDesc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("texels", C.c_void_p)]


RRT_METRIC_SCHWARZSCHILD, RRT_METRIC_KERR = 0, 1


class SpacetimeDesc(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("reserved", C.c_uint32), ("center", C.c_double * 3), ("r_s", C.c_double),
                ("delta_theta", C.c_double), ("spin", C.c_double), ("axis", C.c_double * 3)]


class RenderParams(C.Structure):
    _fields_ = [("ns_aa", C.c_uint32), ("max_ray_depth", C.c_uint32), ("ns_area_light", C.c_uint32),
                ("samples_per_batch", C.c_uint32), ("max_tolerance", C.c_float),
                ("direct_hemisphere", C.c_uint32), ("seed", C.c_uint64), ("frame_w", C.c_uint32),
                ("frame_h", C.c_uint32), ("flags", C.c_uint32), ("variant", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("n_prims", C.c_uint32), ("n_nodes", C.c_uint32), ("n_leaf_refs", C.c_uint32),
                ("max_depth", C.c_uint32), ("device_bytes", C.c_uint64), ("grid_n", C.c_uint32 * 3),
                ("n_clean", C.c_uint32), ("n_big", C.c_uint32),
                ("grid_free_frac", C.c_float), ("last_kernel_ms", C.c_float), ("grid_blocks", C.c_uint32),
                ("block_threads", C.c_uint32), ("kernel", C.c_char * 64), ("last_main_kernel_ms", C.c_float),
                ("last_heavy_pixels", C.c_uint32), ("last_cont_pixels", C.c_uint32)]


# every symbol include/rrt.h declares (checked by tests/test_capi_host.py)
EXPORTS = ["rrt_abi_version", "rrt_create", "rrt_destroy", "rrt_last_error", "rrt_set_scene", "rrt_set_camera",
           "rrt_set_spacetime", "rrt_render_params_default", "rrt_render", "rrt_render_tiles_device",
           "rrt_unpack_tiles_device", "rrt_tonemap_device", "rrt_partition_tiles", "rrt_region_tiles", "rrt_get_stats", "rrt_get_launch_times", "rrt_get_bvh", "rrt_get_free_grid", "rrt_get_clean_tree", "rrt_get_search_tree", "rrt_proof_envelope",
           "rrt_scene_file_load", "rrt_scene_file_desc", "rrt_scene_file_free", "rrt_camera_file_load",
           "rrt_scene_file_save", "rrt_collada_options_default", "rrt_collada_load", "rrt_camera_settings_load",
           "rrt_camera_settings_save", "rrt_camera_state_file_load", "rrt_camera_state_file_save",
           "rrt_camera_state_desc", "rrt_set_envmap", "rrt_tonemap_pixel", "rrt_write_png",
           "rrt_exr_load", "rrt_exr_free", "rrt_exr_save", "rrt_kerr_frame", "rrt_get_big_masks",
           "rrt_get_occluders", "rrt_group_create", "rrt_group_render", "rrt_group_destroy", "rrt_libm_eval",
           "rrt_set_proof_audit", "rrt_get_proof_audit", "rrt_get_search_tree4"]
AUDIT_KINDS = ("camera", "shadow", "pixel", "strip", "kerr", "zero")  # include/rrt.h RRT_AUDIT_*

_lib = None


def build_id():
    """First 16 hex digits of the sha256 of the librrt.so this process loads (ties measured
    profiles -- PMC counters, traffic -- to the exact kernel build they were taken on)."""
    import hashlib
    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def lib():
    """Load librrt.so (fails loudly if it was not built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RRTError(RRT_E_IO, f"{LIB_PATH} not built (run `make -C relativistic-ray-tracer_amd`)")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.rrt_create.argtypes = [C.POINTER(vp), C.POINTER(DeviceCfg)]
        L.rrt_destroy.argtypes = [vp]
        L.rrt_last_error.restype = C.c_char_p
        L.rrt_last_error.argtypes = [vp]
        L.rrt_set_scene.argtypes = [vp, vp]
        L.rrt_set_camera.argtypes = [vp, C.POINTER(CameraDesc)]
        L.rrt_set_spacetime.argtypes = [vp, C.POINTER(SpacetimeDesc)]
        if hasattr(L, "rrt_kerr_frame"):
            L.rrt_kerr_frame.argtypes = [vp, vp, vp, vp]
            L.rrt_kerr_frame.restype = None
        if hasattr(L, "rrt_set_envmap"):
            L.rrt_set_envmap.argtypes = [vp, C.POINTER(EnvmapDesc)]
            L.rrt_exr_load.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_uint32)]
            L.rrt_exr_free.argtypes = [vp]
        L.rrt_render_params_default.argtypes = [C.POINTER(RenderParams)]
        L.rrt_render.argtypes = [vp, C.POINTER(RenderParams), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp,
                                 vp, vp, vp]
        L.rrt_render_tiles_device.argtypes = [vp, C.POINTER(RenderParams), vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp]
        L.rrt_unpack_tiles_device.argtypes = [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp,
                                              vp]
        L.rrt_tonemap_device.argtypes = [vp, C.c_uint32, vp, vp, vp]
        L.rrt_partition_tiles.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, C.c_uint32]
        if hasattr(L, "rrt_region_tiles"):  # absent from older builds loaded through RRT_LIB
            L.rrt_region_tiles.argtypes = [C.c_uint32] * 7 + [vp, C.c_uint32]
        L.rrt_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.rrt_get_launch_times.argtypes = [vp, C.c_uint32, vp, vp]
        L.rrt_libm_eval.argtypes = [vp, C.c_int, vp, vp, vp, C.c_uint64]
        if hasattr(L, "rrt_set_proof_audit"):  # absent from older builds loaded through RRT_LIB
            L.rrt_set_proof_audit.argtypes = [vp, C.c_int]
            L.rrt_get_proof_audit.argtypes = [vp, vp]
        L.rrt_proof_envelope.argtypes = [vp]
        L.rrt_get_bvh.argtypes = [vp, vp, vp, vp]
        for name, n_args in (("rrt_get_free_grid", 4), ("rrt_get_clean_tree", 5), ("rrt_get_search_tree", 3),
                             ("rrt_get_search_tree4", 3),
                             ("rrt_get_big_masks", 3),
                             ("rrt_get_occluders", 3)):
            if hasattr(L, name):  # absent from older builds loaded through RRT_LIB
                getattr(L, name).argtypes = [vp] * n_args
        L.rrt_scene_file_load.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.rrt_scene_file_desc.restype = vp
        L.rrt_scene_file_desc.argtypes = [vp]
        L.rrt_scene_file_free.argtypes = [vp]
        L.rrt_camera_file_load.argtypes = [C.c_char_p, C.POINTER(CameraDesc)]
        if hasattr(L, "rrt_collada_load"):  # absent from older builds loaded through RRT_LIB
            L.rrt_scene_file_save.argtypes = [C.c_char_p, vp]
            L.rrt_collada_options_default.argtypes = [C.POINTER(ColladaOptions)]
            L.rrt_collada_load.argtypes = [C.c_char_p, C.POINTER(ColladaOptions), C.POINTER(vp),
                                           C.POINTER(CameraState), C.c_char_p, C.c_size_t]
            for name in ("rrt_camera_settings_load", "rrt_camera_state_file_load"):
                getattr(L, name).argtypes = [C.c_char_p, C.POINTER(CameraState)]
            for name in ("rrt_camera_settings_save", "rrt_camera_state_file_save"):
                getattr(L, name).argtypes = [C.c_char_p, C.POINTER(CameraState)]
            L.rrt_camera_state_desc.argtypes = [C.POINTER(CameraState), C.POINTER(CameraDesc)]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class ObjectDesc(C.Structure):  # rrt_object_desc
    _fields_ = [("kind", C.c_uint32), ("bsdf", C.c_uint32), ("n_vertices", C.c_uint32), ("n_triangles", C.c_uint32),
                ("positions", C.POINTER(C.c_double)), ("normals", C.POINTER(C.c_double)),
                ("indices", C.POINTER(C.c_uint32)), ("center", C.c_double * 3), ("radius", C.c_double)]


class LightDesc(C.Structure):  # rrt_light_desc
    _fields_ = [("type", C.c_uint32), ("is_delta", C.c_uint32), ("radiance", C.c_float * 3), ("area", C.c_float),
                ("v", (C.c_double * 3) * 4)]


class SceneDesc(C.Structure):  # rrt_scene_desc
    _fields_ = [("n_objects", C.c_uint32), ("n_bsdfs", C.c_uint32), ("n_lights", C.c_uint32), ("reserved", C.c_uint32),
                ("objects", C.POINTER(ObjectDesc)), ("bsdfs", C.c_void_p), ("lights", C.POINTER(LightDesc))]


class SceneFile:
    """A flattened static scene (.rrts, include/rrt_scene_format.h) loaded by librrt."""

    def __init__(self, path=None, handle=None):
        if handle is None:
            h = C.c_void_p()
            rc = lib().rrt_scene_file_load(path.encode(), C.byref(h))
            if rc != RRT_OK:
                raise RRTError(rc, f"cannot load scene {path}")
            handle = h
        self.h = handle

    def desc(self):
        return lib().rrt_scene_file_desc(self.h)

    def triangles(self):
        """[n, 3, 3] vertex positions of every mesh triangle, in object / BVH build order."""
        d = SceneDesc.from_address(self.desc())
        out = []
        for i in range(d.n_objects):
            o = d.objects[i]
            if o.kind != 0 or o.n_triangles == 0:
                continue
            P = np.ctypeslib.as_array(o.positions, shape=(o.n_vertices * 3,)).reshape(-1, 3)
            idx = np.ctypeslib.as_array(o.indices, shape=(o.n_triangles * 3,)).reshape(-1, 3)
            out.append(P[idx])
        return np.concatenate(out) if out else np.zeros((0, 3, 3))

    def lights(self):
        """[(type, is_delta, v [4][3])] of the scene's lights."""
        d = SceneDesc.from_address(self.desc())
        return [(d.lights[i].type, d.lights[i].is_delta, np.array(d.lights[i].v, np.float64))
                for i in range(d.n_lights)]

    def save(self, path):
        rc = lib().rrt_scene_file_save(path.encode(), self.desc())
        if rc != RRT_OK:
            raise RRTError(rc, f"cannot write {path}")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.rrt_scene_file_free(self.h)
            self.h = None


def load_collada(path, screen_w=800, screen_h=600, lens_radius=0.25, focal_distance=4.7):
    """Native COLLADA ingest: (SceneFile, CameraState) as the reference's loader + Application::load
    produce them for a `-r screen_w screen_h` render (include/rrt.h rrt_collada_load)."""
    o = ColladaOptions()
    lib().rrt_collada_options_default(C.byref(o))
    o.screen_w, o.screen_h, o.lens_radius, o.focal_distance = screen_w, screen_h, lens_radius, focal_distance
    h = C.c_void_p()
    cam = CameraState()
    err = C.create_string_buffer(512)
    rc = lib().rrt_collada_load(path.encode(), C.byref(o), C.byref(h), C.byref(cam), err, len(err))
    if rc != RRT_OK:
        raise RRTError(rc, err.value.decode(errors="replace"))
    return SceneFile(handle=h), cam


def camera_desc(state):
    """The rrt_set_camera subset of a CameraState."""
    cam = CameraDesc()
    rc = lib().rrt_camera_state_desc(C.byref(state), C.byref(cam))
    if rc != RRT_OK:
        raise RRTError(rc, "bad camera state")
    return cam


def load_camera_settings(path):
    """Camera::load_settings text file (the `-c` flag)."""
    st = CameraState()
    rc = lib().rrt_camera_settings_load(path.encode(), C.byref(st))
    if rc != RRT_OK:
        raise RRTError(rc, f"cannot read camera settings {path}")
    return st


def load_camera_state(path):
    """.rrtc record as a CameraState."""
    st = CameraState()
    rc = lib().rrt_camera_state_file_load(path.encode(), C.byref(st))
    if rc != RRT_OK:
        raise RRTError(rc, f"cannot load camera {path}")
    return st


def load_camera(path):
    cam = CameraDesc()
    rc = lib().rrt_camera_file_load(path.encode(), C.byref(cam))
    if rc != RRT_OK:
        raise RRTError(rc, f"cannot load camera {path}")
    return cam


def kerr_frame(axis=(0.0, 1.0, 0.0)):
    """(ex, ey, ez) of the Kerr local frame the library uses for this spin axis."""
    a = np.ascontiguousarray(axis, np.float64)
    out = np.zeros((3, 3), np.float64)
    lib().rrt_kerr_frame(a.ctypes.data, out[0].ctypes.data, out[1].ctypes.data, out[2].ctypes.data)
    return out


def load_exr(path):
    """Environment map texels [h][w][3] float32 (rrt_exr_load: main.cpp's load_exr)."""
    t = C.POINTER(C.c_float)()
    w, h = C.c_uint32(), C.c_uint32()
    rc = lib().rrt_exr_load(path.encode(), C.byref(t), C.byref(w), C.byref(h))
    if rc != RRT_OK:
        raise RRTError(rc, f"cannot load {path}")
    arr = np.ctypeslib.as_array(t, shape=(h.value, w.value, 3)).copy()
    lib().rrt_exr_free(t)
    return arr


def render_params(frame_w, frame_h, ns_aa=1, max_ray_depth=1, ns_area_light=1, samples_per_batch=32,
                  max_tolerance=0.05, direct_hemisphere=False, seed=0, flags=0, variant=0):
    p = RenderParams()
    lib().rrt_render_params_default(C.byref(p))
    p.ns_aa, p.max_ray_depth, p.ns_area_light = ns_aa, max_ray_depth, ns_area_light
    p.samples_per_batch, p.max_tolerance, p.direct_hemisphere = samples_per_batch, max_tolerance, int(direct_hemisphere)
    p.seed, p.frame_w, p.frame_h, p.flags, p.variant = seed, frame_w, frame_h, flags, variant
    return p


def partition_tiles(frame_w, frame_h, tile_size, rank, world):
    n = lib().rrt_partition_tiles(frame_w, frame_h, tile_size, rank, world, None, 0)
    if n < 0:
        raise RRTError(n, "bad partition arguments")
    out = np.zeros((max(n, 1), 2), np.uint32)
    lib().rrt_partition_tiles(frame_w, frame_h, tile_size, rank, world, out.ctypes.data, n)
    return out[:n]


def region_tiles(x0, y0, w, h, tile_size, rank, world):
    """rrt_region_tiles: rank's tiles of the region's lattice deal (rrt_group_render's split)."""
    n = lib().rrt_region_tiles(x0, y0, w, h, tile_size, rank, world, None, 0)
    if n < 0:
        raise RRTError(n, "bad partition arguments")
    out = np.zeros((max(n, 1), 2), np.uint32)
    lib().rrt_region_tiles(x0, y0, w, h, tile_size, rank, world, out.ctypes.data, n)
    return out[:n]


class Renderer:
    """One rendering context on one HIP device (device=-1: host-only, for BVH/host tests)."""

    def __init__(self, device=0, free_grid_res=0):
        cfg = DeviceCfg()
        cfg.device = device
        cfg.free_grid_res = free_grid_res
        h = C.c_void_p()
        rc = lib().rrt_create(C.byref(h), C.byref(cfg))
        if rc != RRT_OK:
            raise RRTError(rc, f"rrt_create(device={device}) failed")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.rrt_destroy(self.h)
            self.h = None

    __del__ = close

    def _chk(self, rc):
        if rc != RRT_OK:
            raise RRTError(rc, lib().rrt_last_error(self.h).decode())

    def set_scene(self, scene_file):
        self._scene = scene_file
        self._chk(lib().rrt_set_scene(self.h, scene_file.desc()))

    def set_camera(self, cam):
        self._chk(lib().rrt_set_camera(self.h, C.byref(cam)))

    def set_black_hole(self, center=(0.0, 1.0, 0.0), r_s=0.1, delta_theta=0.1, spin=None, axis=(0.0, 1.0, 0.0)):
        """The global black hole (-B).  spin=None: Schwarzschild (the reference's stepper);
        spin=a/M in [0, 1): the Kerr integrator (build-defined) about `axis`."""
        st = SpacetimeDesc()
        st.kind = RRT_METRIC_SCHWARZSCHILD if spin is None else RRT_METRIC_KERR
        st.center[0], st.center[1], st.center[2] = center
        st.r_s, st.delta_theta = r_s, delta_theta
        if spin is not None:
            st.spin = spin
            st.axis[0], st.axis[1], st.axis[2] = axis
        self._chk(lib().rrt_set_spacetime(self.h, C.byref(st)))

    def set_envmap(self, texels):
        """Environment map ([h][w][3] float32) or None (the PathTracer ctor's envmap argument)."""
        if texels is None:
            self._chk(lib().rrt_set_envmap(self.h, None))
            return
        t = np.ascontiguousarray(texels, np.float32)
        d = EnvmapDesc()
        d.width, d.height, d.texels = t.shape[1], t.shape[0], t.ctypes.data
        self._chk(lib().rrt_set_envmap(self.h, C.byref(d)))

    LIBM_FN = {"sin": 0, "cos": 1, "acos": 2, "atan2": 3, "sinf": 4, "cosf": 5, "exp": 6, "log": 7, "erf": 8,
               "atan": 9, "tan": 10}

    def libm_eval(self, fn, a, b=None):
        """The device's restated host-libm function `fn` (rrt_glibm.h) on float64 arrays a (, b)."""
        a = np.ascontiguousarray(a, dtype=np.float64)
        b = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
        out = np.empty_like(a)
        self._chk(lib().rrt_libm_eval(self.h, self.LIBM_FN[fn], _p(a), _p(b), _p(out), a.size))
        return out

    def render(self, params, x0, y0, w, h, draws=False, counters=False):
        rgb = np.zeros((h, w, 3), np.float32)
        cnt = np.zeros((h, w), np.int32)
        dr = np.zeros((h, w), np.uint32) if draws else None
        ct = np.zeros((h, w, 4), np.uint32) if counters else None
        self._chk(lib().rrt_render(self.h, C.byref(params), x0, y0, w, h, _p(rgb), _p(cnt), _p(dr), _p(ct), None))
        return rgb, cnt, dr, ct

    def render_tiles_device(self, params, tiles, tile_size, d_rgb, d_count, d_counters=None, stream=None):
        tiles = np.ascontiguousarray(tiles, dtype=np.uint32)
        self._chk(lib().rrt_render_tiles_device(self.h, C.byref(params), _p(tiles), len(tiles), tile_size, d_rgb,
                                                d_count, d_counters, stream))

    def unpack_tiles_device(self, tiles, tile_size, frame_w, frame_h, rgb_p, cnt_p, rgb, cnt, stream=None):
        tiles = np.ascontiguousarray(tiles, dtype=np.uint32)
        self._chk(lib().rrt_unpack_tiles_device(self.h, _p(tiles), len(tiles), tile_size, frame_w, frame_h, rgb_p,
                                                cnt_p, rgb, cnt, stream))

    def tonemap_device(self, n, d_rgb, d_rgba, stream=None):
        self._chk(lib().rrt_tonemap_device(self.h, n, d_rgb, d_rgba, stream))

    def stats(self):
        s = Stats()
        self._chk(lib().rrt_get_stats(self.h, C.byref(s)))
        return s

    def set_proof_audit(self, every_log2):
        """Counting launches (RRT_RENDER_COUNTERS | RRT_RENDER_COUNT_EXECUTED) re-march every
        2^every_log2-th proven ray exactly (rrt_set_proof_audit); every_log2 < 0 turns it off."""
        self._chk(lib().rrt_set_proof_audit(self.h, every_log2))

    def proof_audit(self):
        """{proof: {"checked": n, "violations": m}} since the last call (rrt_get_proof_audit; resets)."""
        out = np.zeros(2 * len(AUDIT_KINDS), np.uint64)
        self._chk(lib().rrt_get_proof_audit(self.h, _p(out)))
        return {k: {"checked": int(out[2 * i]), "violations": int(out[2 * i + 1])} for i, k in enumerate(AUDIT_KINDS)}

    def launch_times(self, n):
        """HIP-event ms of the last n (<= 32) launches, oldest first: (whole launch, main kernel)."""
        tot, main = np.zeros(n, np.float32), np.zeros(n, np.float32)
        k = lib().rrt_get_launch_times(self.h, n, _p(tot), _p(main))
        if k < 0:
            self._chk(k)
        return tot[:k], main[:k]

    def search_tree4(self):
        """(boxes [n, 4, 6] f32, kids [n, 4, 3] = child, first, count) of the 4-wide walk's nodes."""
        n = lib().rrt_get_search_tree4(self.h, None, None)
        if n < 0:
            self._chk(n)
        b = np.zeros((max(n, 1), 4, 6), np.float32)
        k = np.zeros((max(n, 1), 4, 3), np.int32)
        lib().rrt_get_search_tree4(self.h, _p(b), _p(k))
        return b[:n], k[:n]

    def free_grid(self):
        """(k [nz][ny][nx] uint8, g0 (3,), inv_h, h_free) of the empty-space grid, or None."""
        n = np.zeros(3, np.int32)
        cells = lib().rrt_get_free_grid(self.h, None, None, _p(n))
        if cells < 0:
            raise RRTError(cells, "no scene")
        if cells == 0:
            return None
        k = np.zeros((n[2], n[1], n[0]), np.uint8)
        geom = np.zeros(5, np.float64)
        self._chk(0 if lib().rrt_get_free_grid(self.h, _p(k), _p(geom), _p(n)) > 0 else RRT_E_INVALID)
        return k, geom[:3].copy(), float(geom[3]), float(geom[4])

    def big_masks(self):
        """(mask [nz][ny][nx] uint32 over the free grid's cells, reach) of the oversized-leaf masks, or None."""
        cells = lib().rrt_get_big_masks(self.h, None, None)
        if cells < 0:
            raise RRTError(cells, "no scene")
        if cells == 0:
            return None
        g = self.free_grid()
        m = np.zeros(g[0].shape, np.uint32)
        reach = np.zeros(1, np.float64)
        lib().rrt_get_big_masks(self.h, _p(m), _p(reach))
        return m, float(reach[0])

    def occluders(self):
        """(tris [6][4][16] = plane n (3), d, in-plane edge normals en [3][3], offsets eo [3];
        counts [6]) of the shadow-ray occlusion proof's root-box face triangles (include/rrt.h
        rrt_get_occluders)."""
        tris = np.zeros((6, 4, 16), np.float64)
        counts = np.zeros(6, np.uint32)
        n = lib().rrt_get_occluders(self.h, _p(tris), _p(counts))
        if n < 0:
            raise RRTError(n, "no scene")
        return tris, counts

    def clean_tree(self):
        """(boxes [n,6], nodes [n,4] (skip, first, count, ordinal), big_boxes [nb,6], big [nb,3]
        (first, count, ordinal)) of the clean tree, or None."""
        s = self.stats()
        if s.n_clean == 0:
            return None
        boxes = np.zeros((s.n_clean, 6), np.float64)
        nodes = np.zeros((s.n_clean, 4), np.int32)
        bb = np.zeros((max(s.n_big, 1), 6), np.float64)
        big = np.zeros((max(s.n_big, 1), 3), np.int32)
        self._chk(0 if lib().rrt_get_clean_tree(self.h, _p(boxes), _p(nodes), _p(bb), _p(big)) > 0 else RRT_E_INVALID)
        return boxes, nodes, bb[:s.n_big], big[:s.n_big]

    def proof_envelope(self):
        """True if the scene and hole lie in the proofs' validated envelope (rrt_proof_envelope)."""
        return lib().rrt_proof_envelope(self.h) == 1

    def search_tree(self):
        """(boxes [n,6], nodes [n,4] (skip, first, count, ordinal)) of the search tree, or None."""
        n = lib().rrt_get_search_tree(self.h, None, None)
        if n <= 0:
            return None
        boxes = np.zeros((n, 6), np.float64)
        nodes = np.zeros((n, 4), np.int32)
        lib().rrt_get_search_tree(self.h, _p(boxes), _p(nodes))
        return boxes, nodes

    def bvh(self):
        s = self.stats()
        boxes = np.zeros((s.n_nodes, 6), np.float64)
        nodes = np.zeros((s.n_nodes, 4), np.int32)
        prims = np.zeros(s.n_leaf_refs, np.uint32)
        self._chk(lib().rrt_get_bvh(self.h, _p(boxes), _p(nodes), _p(prims)))
        return boxes, nodes, prims
