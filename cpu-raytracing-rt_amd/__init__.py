"""MI355X-native path-tracing hot path of uncerso/cpu-raytracing-rt — host side.

Python mirror of the reference's frame-level interface over the C ABI in
``include/rt_api.h`` (``build/librt_amd.so``, HIP kernels for gfx950):

=====================================  ==========================================
reference (Rust, /root/reference/src)  here
=====================================  ==========================================
scene_parser::parse_scene (:5-43)      :func:`parse_scene` (text -> ParsedScene)
gltf::parse + gltf::build_scene        :func:`load_gltf`
Scene::new / make_scenes (scene.rs)    :class:`Scene` (device-resident, BVHs built)
generate_image (main.rs:85-114)        :meth:`Scene.generate_image` (mean radiance),
                                       :func:`generate_image` (tonemapped like main.rs:104)
intersect (intersections.rs:42-62)     :meth:`Scene.intersect`
Light::pdf (ray_sampler.rs:132-139)    :meth:`Scene.light_pdf`
aces_tonemap/correct_gamma             :func:`tonemap_gamma`
ppm::save_to_ppm (ppm.rs:4-11)         :func:`save_to_ppm`
=====================================  ==========================================

There is no CPU fallback: loading fails loudly if the shared library is
missing, and every render call fails with ``RtError`` when no HIP device is
visible.  The package directory name contains dashes, so import it with
``importlib`` (see ``tests/conftest.py``) or ``__graft_entry__``.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_AMD_LIB: alternate build of the same library (tuning experiments only)
LIB_PATH = os.environ.get("RT_AMD_LIB") or os.path.join(_HERE, "build", "librt_amd.so")

# ----------------------------------------------------------------- ABI ----
RT_MAT_DIFFUSE, RT_MAT_METALLIC, RT_MAT_DIELECTRIC = 0, 1, 2
RT_SHAPE_PLANE, RT_SHAPE_BOX, RT_SHAPE_ELLIPSOID = 0, 1, 2
RT_TRI_CUSTOM, RT_TRI_GLTF = 0, 1
RT_FOV_X, RT_FOV_Y = 0, 1
RT_FLAG_STATS, RT_FLAG_HIT_IDS = 0x1, 0x2
RT_HIT_MISS, RT_HIT_NONE = -1, -2
RT_TILE = 16
ERRORS = {0: "OK", -1: "INVALID", -2: "DEVICE", -3: "NOMEM", -4: "PARSE", -5: "IO", -6: "UNSUPPORTED"}
(RT_OK, RT_ERR_INVALID, RT_ERR_DEVICE, RT_ERR_NOMEM, RT_ERR_PARSE, RT_ERR_IO,
 RT_ERR_UNSUPPORTED) = 0, -1, -2, -3, -4, -5, -6


class rt_material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("_pad", C.c_uint32), ("ior", C.c_double),
                ("color", C.c_double * 3), ("emission", C.c_double * 3)]


class rt_shape(C.Structure):
    _fields_ = [("type", C.c_uint32), ("material", C.c_uint32), ("shape", C.c_double * 3),
                ("position", C.c_double * 3), ("rotation", C.c_double * 4)]


class rt_scene_desc(C.Structure):
    _fields_ = [("n_materials", C.c_uint32), ("n_shapes", C.c_uint32), ("n_triangles", C.c_uint64),
                ("materials", C.POINTER(rt_material)), ("shapes", C.POINTER(rt_shape)),
                ("tri_mode", C.c_uint32), ("_pad", C.c_uint32),
                ("tri_vertices", C.POINTER(C.c_double)), ("tri_normals", C.POINTER(C.c_double)),
                ("tri_position", C.POINTER(C.c_double)), ("tri_rotation", C.POINTER(C.c_double)),
                ("tri_material", C.POINTER(C.c_uint32))]


class rt_render_params(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32), ("ray_depth", C.c_uint32),
                ("bg_color", C.c_double * 3), ("cam_position", C.c_double * 3), ("cam_right", C.c_double * 3),
                ("cam_up", C.c_double * 3), ("cam_forward", C.c_double * 3), ("fov_axis", C.c_uint32),
                ("flags", C.c_uint32), ("fov", C.c_double), ("seed", C.c_uint64)]


class rt_stats(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("segments", C.c_uint64), ("aabb_tests", C.c_uint64),
                ("tri_tests", C.c_uint64), ("shape_tests", C.c_uint64), ("shaded_hits", C.c_uint64),
                ("light_queries", C.c_uint64), ("light_hits", C.c_uint64), ("kernel_ms", C.c_double),
                ("total_ms", C.c_double), ("lane_steps", C.c_uint64), ("wave_steps", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class rt_hit(C.Structure):
    _fields_ = [("t", C.c_double), ("geometry_normal", C.c_double * 3), ("shading_normal", C.c_double * 3),
                ("inside", C.c_int32), ("prim", C.c_int32)]


HIT_DTYPE = np.dtype([("t", "<f8"), ("geometry_normal", "<f8", 3), ("shading_normal", "<f8", 3),
                      ("inside", "<i4"), ("prim", "<i4")])
assert HIT_DTYPE.itemsize == C.sizeof(rt_hit)


class rt_scene_info(C.Structure):
    _fields_ = [("n_planes", C.c_uint32), ("n_boxes", C.c_uint32), ("n_ellipsoids", C.c_uint32),
                ("n_triangles", C.c_uint64), ("n_light_boxes", C.c_uint32), ("n_light_ellipsoids", C.c_uint32),
                ("n_light_triangles", C.c_uint64), ("bvh_nodes", C.c_uint64 * 6), ("bvh_depth", C.c_uint32 * 6),
                ("build_ms", C.c_double), ("upload_ms", C.c_double), ("device_bytes", C.c_uint64),
                ("shared_light_mask", C.c_uint32), ("layout_flags", C.c_uint32)]


class rt_tuning(C.Structure):
    _fields_ = [("waves", C.c_uint32), ("resume", C.c_int32), ("kinds", C.c_uint32),
                ("suspend_lanes", C.c_uint32), ("leaf_lanes", C.c_uint32), ("chunk_spp", C.c_uint32),
                ("compact", C.c_int32), ("tail_split", C.c_uint32)]


TUNING_AUTO = dict(waves=0, resume=-1, kinds=0, suspend_lanes=0, leaf_lanes=0, chunk_spp=0, compact=-1, tail_split=0)
RT_LAYOUT_COMPACT_TRIS = 0x1
RT_LAYOUT_PAIR_NODES = 0x4


# every symbol include/rt_api.h declares (checked by tests/test_abi.py)
EXPORTS = {
    "rt_scene_create": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(C.c_void_p)]),
    "rt_scene_destroy": (None, [C.c_void_p]),
    "rt_scene_get_info": (C.c_int, [C.c_void_p, C.POINTER(rt_scene_info)]),
    "rt_scene_checksum": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "rt_scene_set_tuning": (C.c_int, [C.c_void_p, C.POINTER(rt_tuning)]),
    "rt_scene_get_tuning": (C.c_int, [C.c_void_p, C.POINTER(rt_tuning)]),
    "rt_scene_sample_chunks": (C.c_int, [C.c_void_p, C.POINTER(rt_render_params), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32)]),
    "rt_render": (C.c_int, [C.c_void_p, C.POINTER(rt_render_params), C.c_void_p, C.c_void_p, C.POINTER(rt_stats)]),
    "rt_tiles_per_rank": (C.c_int, [C.POINTER(rt_render_params), C.c_uint32, C.POINTER(C.c_uint32)]),
    "rt_sample_chunks": (C.c_int, [C.POINTER(rt_render_params), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "rt_render_tiles_async": (C.c_int, [C.c_void_p, C.POINTER(rt_render_params), C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.c_void_p]),
    "rt_read_stats": (C.c_int, [C.c_void_p, C.POINTER(rt_stats), C.c_int]),
    "rt_read_raw_stats": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "rt_unpack_tiles_async": (C.c_int, [C.POINTER(rt_render_params), C.c_uint32, C.c_void_p, C.c_void_p,
                                        C.c_void_p]),
    "rt_unpack_tiles_bytes_async": (C.c_int, [C.POINTER(rt_render_params), C.c_uint32, C.c_void_p, C.c_void_p,
                                              C.c_void_p]),
    "rt_tonemap_bytes_async": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "rt_intersect_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "rt_intersect_rays_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]),
    "rt_light_pdf_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "rt_intersect_lights_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    "rt_parse_custom_scene": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    "rt_load_gltf": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p)]),
    "rt_parsed_scene_get": (C.c_int, [C.c_void_p, C.POINTER(rt_scene_desc), C.POINTER(rt_render_params)]),
    "rt_parsed_scene_free": (None, [C.c_void_p]),
    "rt_tonemap_gamma": (None, [C.c_void_p, C.c_uint64, C.c_void_p]),
    "rt_save_ppm": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, C.c_void_p]),
    "rt_byte_thresholds": (C.c_int, [C.c_void_p]),
    "rt_last_error": (C.c_char_p, []),
    "rt_api_version": (C.c_int, []),
    "rt_device_count": (C.c_int, []),
    "rt_probe_fp64": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "rt_bvh_build": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p, C.c_void_p, C.c_void_p,
                               C.POINTER(C.c_uint32)]),
    "rt_multi_create": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(C.c_int), C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_void_p)]),
    "rt_multi_render": (C.c_int, [C.c_void_p, C.POINTER(rt_render_params), C.c_void_p, C.c_void_p,
                                  C.POINTER(rt_stats)]),
    "rt_multi_scene": (C.c_void_p, [C.c_void_p, C.c_uint32]),
    "rt_multi_destroy": (None, [C.c_void_p]),
}
RT_MULTI_PEER = 0x1

_lib = None


def lib() -> C.CDLL:
    """Load ``build/librt_amd.so`` (raises if it was not built — no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
        # One HIP runtime per process: torch ships its own libamdhip64.so with
        # the same SONAME (libamdhip64.so.7) as /opt/rocm's.  Importing torch
        # first makes our DT_NEEDED bind to torch's copy, so device pointers
        # and streams from torch (tile buffers, RCCL gather) are valid here;
        # loading ours first would leave torch unable to initialise HIP.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rt error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


def _check(rc: int):
    if rc != 0:
        raise RtError(rc, lib().rt_last_error().decode(errors="replace"))


def _ptr(a: Optional[np.ndarray], ctype=C.c_double):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


def device_count() -> int:
    return lib().rt_device_count()


# --------------------------------------------------------- scene model ----
@dataclass
class RenderParams:
    """Scene-level settings of the reference's Scene (scene.rs:81-90) + RNG seed."""
    width: int
    height: int
    spp: int = 64
    ray_depth: int = 16
    bg_color: tuple = (0.0, 0.0, 0.0)
    cam_position: tuple = (0.0, 0.0, 0.0)
    cam_right: tuple = (1.0, 0.0, 0.0)
    cam_up: tuple = (0.0, 1.0, 0.0)
    cam_forward: tuple = (0.0, 0.0, 1.0)
    fov_axis: int = RT_FOV_X
    fov: float = np.pi / 2
    seed: int = 0x5EED
    flags: int = 0

    def to_c(self) -> rt_render_params:
        p = rt_render_params()
        p.width, p.height, p.spp, p.ray_depth = self.width, self.height, self.spp, self.ray_depth
        p.bg_color[:] = self.bg_color
        p.cam_position[:] = self.cam_position
        p.cam_right[:] = self.cam_right
        p.cam_up[:] = self.cam_up
        p.cam_forward[:] = self.cam_forward
        p.fov_axis, p.fov, p.seed, p.flags = self.fov_axis, self.fov, self.seed, self.flags
        return p

    @staticmethod
    def from_c(p: rt_render_params) -> "RenderParams":
        return RenderParams(p.width, p.height, p.spp, p.ray_depth, tuple(p.bg_color), tuple(p.cam_position),
                            tuple(p.cam_right), tuple(p.cam_up), tuple(p.cam_forward), p.fov_axis, p.fov,
                            p.seed, p.flags)

    def replace(self, **kw) -> "RenderParams":
        d = dict(self.__dict__)
        d.update(kw)
        return RenderParams(**d)


@dataclass
class SceneDesc:
    """The parsed scene (parsed_scene.rs) as numpy arrays; see rt_scene_desc."""
    materials: np.ndarray                  # structured, rt_material layout
    shapes: np.ndarray                     # structured, rt_shape layout
    tri_vertices: np.ndarray = field(default_factory=lambda: np.zeros((0, 9)))
    tri_normals: Optional[np.ndarray] = None
    tri_position: Optional[np.ndarray] = None
    tri_rotation: Optional[np.ndarray] = None
    tri_material: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    tri_mode: int = RT_TRI_CUSTOM

    def to_c(self):
        """Returns (rt_scene_desc, keepalive) — the arrays must outlive the call."""
        keep = []

        def arr(a, dt):
            if a is None or len(a) == 0:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a

        mats = arr(self.materials, MATERIAL_DTYPE)
        shapes = arr(self.shapes, SHAPE_DTYPE)
        tv = arr(self.tri_vertices, np.float64)
        tn = arr(self.tri_normals, np.float64)
        tp = arr(self.tri_position, np.float64)
        tr = arr(self.tri_rotation, np.float64)
        tm = arr(self.tri_material, np.uint32)
        d = rt_scene_desc()
        d.n_materials = 0 if mats is None else len(mats)
        d.n_shapes = 0 if shapes is None else len(shapes)
        d.n_triangles = 0 if tm is None else len(tm)
        d.materials = None if mats is None else mats.ctypes.data_as(C.POINTER(rt_material))
        d.shapes = None if shapes is None else shapes.ctypes.data_as(C.POINTER(rt_shape))
        d.tri_mode = self.tri_mode
        d.tri_vertices = _ptr(tv)
        d.tri_normals = _ptr(tn)
        d.tri_position = _ptr(tp)
        d.tri_rotation = _ptr(tr)
        d.tri_material = _ptr(tm, C.c_uint32)
        return d, keep


MATERIAL_DTYPE = np.dtype([("kind", "<u4"), ("_pad", "<u4"), ("ior", "<f8"), ("color", "<f8", 3),
                           ("emission", "<f8", 3)])
SHAPE_DTYPE = np.dtype([("type", "<u4"), ("material", "<u4"), ("shape", "<f8", 3), ("position", "<f8", 3),
                        ("rotation", "<f8", 4)])
assert MATERIAL_DTYPE.itemsize == C.sizeof(rt_material) and SHAPE_DTYPE.itemsize == C.sizeof(rt_shape)


def _desc_from_c(d: rt_scene_desc) -> SceneDesc:
    def np_from(ptr, n, dt, shape):
        if not ptr or n == 0:
            return None
        buf = C.cast(ptr, C.POINTER(C.c_char * (n * np.dtype(dt).itemsize))).contents
        return np.frombuffer(bytes(buf), dtype=dt).reshape(shape).copy()

    nt = d.n_triangles
    mats = np_from(d.materials, d.n_materials, MATERIAL_DTYPE, (d.n_materials,))
    shapes = np_from(d.shapes, d.n_shapes, SHAPE_DTYPE, (d.n_shapes,))
    return SceneDesc(
        materials=mats if mats is not None else np.zeros(0, MATERIAL_DTYPE),
        shapes=shapes if shapes is not None else np.zeros(0, SHAPE_DTYPE),
        tri_vertices=np_from(d.tri_vertices, nt * 9, np.float64, (nt, 9)) if nt else np.zeros((0, 9)),
        tri_normals=np_from(d.tri_normals, nt * 9, np.float64, (nt, 9)),
        tri_position=np_from(d.tri_position, nt * 3, np.float64, (nt, 3)),
        tri_rotation=np_from(d.tri_rotation, nt * 4, np.float64, (nt, 4)),
        tri_material=np_from(d.tri_material, nt, np.uint32, (nt,)) if nt else np.zeros(0, np.uint32),
        tri_mode=d.tri_mode)


def _take_parsed(handle: C.c_void_p):
    d, p = rt_scene_desc(), rt_render_params()
    try:
        _check(lib().rt_parsed_scene_get(handle, C.byref(d), C.byref(p)))
        return _desc_from_c(d), RenderParams.from_c(p)
    finally:
        lib().rt_parsed_scene_free(handle)


def parse_scene(text: str):
    """scene_parser::parse_scene + Scene::new defaults -> (SceneDesc, RenderParams)."""
    h = C.c_void_p()
    _check(lib().rt_parse_custom_scene(text.encode(), C.byref(h)))
    return _take_parsed(h)


def load_gltf(path: str, width: int, height: int, spp: int):
    """gltf::parse + gltf::build_scene (main.rs:47-66) -> (SceneDesc, RenderParams)."""
    h = C.c_void_p()
    _check(lib().rt_load_gltf(path.encode(), width, height, spp, C.byref(h)))
    return _take_parsed(h)


class Scene:
    """Scene::new: BVHs built on the host, flattened arrays resident on the current HIP device."""

    def __init__(self, desc: SceneDesc):
        self.desc = desc
        d, keep = desc.to_c()
        h = C.c_void_p()
        _check(lib().rt_scene_create(C.byref(d), C.byref(h)))
        self._h = h
        del keep

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def checksum(self) -> int:
        """rt_scene_checksum: content hash of the scene's device arrays."""
        h = C.c_uint64()
        _check(lib().rt_scene_checksum(self._h, C.byref(h)))
        return h.value

    def info(self) -> dict:
        i = rt_scene_info()
        _check(lib().rt_scene_get_info(self._h, C.byref(i)))
        out = {k: getattr(i, k) for k, _ in i._fields_}
        out["bvh_nodes"] = list(i.bvh_nodes)
        out["bvh_depth"] = list(i.bvh_depth)
        return out

    def set_tuning(self, **kw):
        """Force the kernel form of this scene's renders (rt_scene_set_tuning): waves (3|4|5; 5 = shape-only fused only),
        resume (0|1), kinds (3 = all-kinds instance), suspend_lanes, leaf_lanes (1..64),
        chunk_spp, compact (0 = f64 triangle-BVH layout, 1 = compact when the scene has it),
        tail_split (1 = every wave-tile whole, 2..8 = the queue's last wave-tiles in that many parts).
        Fields not given are auto (the library's per-scene pick)."""
        bad = set(kw) - set(TUNING_AUTO)
        if bad:
            raise ValueError(f"unknown tuning fields {sorted(bad)}")
        t = rt_tuning(**{**TUNING_AUTO, **{k: int(v) for k, v in kw.items()}})
        _check(lib().rt_scene_set_tuning(self._h, C.byref(t)))

    def tuning(self) -> dict:
        """The resolved kernel form the next render runs (rt_scene_get_tuning)."""
        t = rt_tuning()
        _check(lib().rt_scene_get_tuning(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in t._fields_ if not k.startswith("_")}

    def sample_chunks(self, params: RenderParams):
        """(chunks, chunk_spp) this scene's renders use (rt_scene_sample_chunks)."""
        k, cs = C.c_uint32(), C.c_uint32()
        _check(lib().rt_scene_sample_chunks(self._h, C.byref(params.to_c()), C.byref(k), C.byref(cs)))
        return k.value, cs.value

    def generate_image(self, params: RenderParams, hit_ids: bool = False, stats: bool = False):
        """Mean radiance per pixel [H, W, 3] f64 (main.rs:100-104 before tonemapping).

        Returns (image, hit_ids or None, stats dict)."""
        flags = params.flags | (RT_FLAG_HIT_IDS if hit_ids else 0) | (RT_FLAG_STATS if stats else 0)
        p = params.replace(flags=flags).to_c()
        img = np.zeros((params.height, params.width, 3), np.float64)
        hits = None
        if hit_ids:
            hits = np.zeros((params.height * params.width, params.spp, params.ray_depth), np.int32)
        st = rt_stats()
        _check(lib().rt_render(self._h, C.byref(p), img.ctypes.data_as(C.c_void_p),
                               None if hits is None else hits.ctypes.data_as(C.c_void_p), C.byref(st)))
        return img, hits, st.as_dict()

    def intersect(self, rays: np.ndarray) -> np.ndarray:
        """intersect(ray, &scene.primitives, +inf) for rays [n, 6] -> structured hits."""
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        out = np.zeros(len(rays), HIT_DTYPE)
        _check(lib().rt_intersect_rays(self._h, rays.ctypes.data_as(C.c_void_p), len(rays),
                                       out.ctypes.data_as(C.c_void_p)))
        return out

    def intersect_async(self, d_rays_ptr: int, n: int, d_hits_ptr: int, method: int = 1, stream_ptr: int = 0):
        """Device-buffer batch intersect (rt_intersect_rays_async): d_rays [n][6] f64 and
        d_hits [n] rt_hit (64 B) in HBM; method 0 = one thread per ray, 1 = persistent."""
        _check(lib().rt_intersect_rays_async(self._h, C.c_void_p(d_rays_ptr), n, C.c_void_p(d_hits_ptr), method,
                                             C.c_void_p(stream_ptr)))

    def light_pdf(self, pos_dir: np.ndarray) -> np.ndarray:
        """Light::pdf for [n, 6] (surface position, unit direction)."""
        pos_dir = np.ascontiguousarray(pos_dir, np.float64).reshape(-1, 6)
        out = np.zeros(len(pos_dir), np.float64)
        _check(lib().rt_light_pdf_rays(self._h, pos_dir.ctypes.data_as(C.c_void_p), len(pos_dir),
                                       out.ctypes.data_as(C.c_void_p)))
        return out

    def intersect_lights(self, rays: np.ndarray):
        """Raw intersect_lights accumulation -> (impact sum, callback count)."""
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        imp = np.zeros(len(rays), np.float64)
        cnt = np.zeros(len(rays), np.uint32)
        _check(lib().rt_intersect_lights_rays(self._h, rays.ctypes.data_as(C.c_void_p), len(rays),
                                              imp.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p)))
        return imp, cnt

    # ---- multi-GPU tile partition ----
    def tiles_per_rank(self, params: RenderParams, world: int) -> int:
        n = C.c_uint32()
        _check(lib().rt_tiles_per_rank(C.byref(params.to_c()), world, C.byref(n)))
        return n.value

    def render_tiles_async(self, params: RenderParams, rank: int, world: int, d_out_ptr: int, stream_ptr: int = 0,
                           stats: bool = False):
        p = params.replace(flags=params.flags | (RT_FLAG_STATS if stats else 0)).to_c()
        _check(lib().rt_render_tiles_async(self._h, C.byref(p), rank, world, C.c_void_p(d_out_ptr),
                                           C.c_void_p(stream_ptr)))

    def read_stats(self, reset: bool = True) -> dict:
        st = rt_stats()
        _check(lib().rt_read_stats(self._h, C.byref(st), 1 if reset else 0))
        return st.as_dict()

    def read_raw_stats(self, n: int = 64) -> np.ndarray:
        """Raw device counter words (diagnostics; rt_read_raw_stats)."""
        out = np.zeros(n, np.uint64)
        _check(lib().rt_read_raw_stats(self._h, out.ctypes.data_as(C.c_void_p), n))
        return out


class MultiScene:
    """generate_image over several GPUs of one process (rt_multi_*): one scene
    replica per listed device (BVHs built once, uploaded to devices[0] and
    broadcast from there: ncclBroadcast, or peer copies), the frame's tiles dealt
    round-robin, one gather to devices[0] (RCCL ncclGather, or peer copies with
    peer=True, which also allows a device listed twice)."""

    def __init__(self, desc: SceneDesc, devices, peer: bool = False):
        self.desc = desc
        self.devices = [int(d) for d in devices]
        d, keep = desc.to_c()
        devs = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        _check(lib().rt_multi_create(C.byref(d), devs, len(self.devices), RT_MULTI_PEER if peer else 0,
                                     C.byref(h)))
        self._h = h
        del keep

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def scene_checksum(self, index: int) -> int:
        """rt_scene_checksum of the replica on devices[index] (rt_multi_create already
        checked every replica against devices[0]'s)."""
        h = lib().rt_multi_scene(self._h, index)
        if not h:
            raise IndexError(index)
        v = C.c_uint64()
        _check(lib().rt_scene_checksum(C.c_void_p(h), C.byref(v)))
        return v.value

    def scene_info(self, index: int) -> dict:
        """rt_scene_get_info of the replica on devices[index] (rt_multi_scene): devices[0]'s came
        from the host, the others from devices[0] (ncclBroadcast / peer copies), whose fill time
        is part of their upload_ms."""
        h = lib().rt_multi_scene(self._h, index)
        if not h:
            raise IndexError(index)
        i = rt_scene_info()
        _check(lib().rt_scene_get_info(C.c_void_p(h), C.byref(i)))
        out = {k: getattr(i, k) for k, _ in i._fields_}
        out["bvh_nodes"] = list(i.bvh_nodes)
        out["bvh_depth"] = list(i.bvh_depth)
        return out

    def generate_image(self, params: RenderParams, ppm_bytes: bool = False, stats: bool = False):
        """(mean radiance [H, W, 3] f64, PPM payload [H, W, 3] u8 or None, stats dict)."""
        p = params.replace(flags=params.flags | (RT_FLAG_STATS if stats else 0)).to_c()
        img = np.zeros((params.height, params.width, 3), np.float64)
        byts = np.zeros((params.height, params.width, 3), np.uint8) if ppm_bytes else None
        st = rt_stats()
        _check(lib().rt_multi_render(self._h, C.byref(p), img.ctypes.data_as(C.c_void_p),
                                     None if byts is None else byts.ctypes.data_as(C.c_void_p), C.byref(st)))
        return img, byts, st.as_dict()


def tile_layout(width: int, height: int, world: int):
    """16x16 tiles, tile t owned by rank t % world at slot t // world.
    Returns (tiles_x, tiles_y, n_tiles, slots_per_rank)."""
    tx = (width + RT_TILE - 1) // RT_TILE
    ty = (height + RT_TILE - 1) // RT_TILE
    n = tx * ty
    return tx, ty, n, (n + world - 1) // world


def gather_tiles(tiles, gathered, rank: int, world: int, group=None):
    """The single framebuffer exchange: every rank's packed tiles [slots, 256, 3]
    to rank 0's [world, slots, 256, 3] (rank-major, ncclGather layout) with one
    torch.distributed gather (RCCL under the "nccl" backend, gloo on CPU)."""
    if world == 1:
        return tiles
    import torch.distributed as dist
    dist.gather(tiles, list(gathered.unbind(0)) if rank == 0 else None, dst=0, group=group)
    return gathered


def unpack_tiles_async(params: RenderParams, world: int, d_gathered_ptr: int, d_image_ptr: int, stream_ptr: int = 0):
    _check(lib().rt_unpack_tiles_async(C.byref(params.to_c()), world, C.c_void_p(d_gathered_ptr),
                                       C.c_void_p(d_image_ptr), C.c_void_p(stream_ptr)))


def unpack_tiles_bytes_async(params: RenderParams, world: int, d_gathered_ptr: int, d_bytes_ptr: int,
                             stream_ptr: int = 0):
    """Gathered tiles -> PPM payload [H][W][3] u8 on the device (unpack + tonemap + gamma + bytes)."""
    _check(lib().rt_unpack_tiles_bytes_async(C.byref(params.to_c()), world, C.c_void_p(d_gathered_ptr),
                                             C.c_void_p(d_bytes_ptr), C.c_void_p(stream_ptr)))


def tonemap_bytes_async(d_rgb_ptr: int, n_pixels: int, d_bytes_ptr: int, stream_ptr: int = 0):
    """Device correct_gamma(aces_tonemap(.)) + PPM bytes of an HBM-resident mean image."""
    _check(lib().rt_tonemap_bytes_async(C.c_void_p(d_rgb_ptr), n_pixels, C.c_void_p(d_bytes_ptr),
                                        C.c_void_p(stream_ptr)))


# ------------------------------------------------------- output surface ----
def tonemap_gamma(mean_rgb: np.ndarray) -> np.ndarray:
    """correct_gamma(aces_tonemap(x)) per channel (postprocessing.rs:5-37)."""
    a = np.ascontiguousarray(mean_rgb, np.float64)
    out = np.empty_like(a)
    lib().rt_tonemap_gamma(a.ctypes.data_as(C.c_void_p), a.size // 3, out.ctypes.data_as(C.c_void_p))
    return out


def save_to_ppm(path: str, rgb: np.ndarray):
    """ppm::save_to_ppm of an already tonemapped [H, W, 3] image (ppm.rs:4-19)."""
    rgb = np.ascontiguousarray(rgb, np.float64)
    _check(lib().rt_save_ppm(path.encode(), rgb.shape[1], rgb.shape[0], rgb.ctypes.data_as(C.c_void_p)))


def generate_image(scene: Scene, params: RenderParams) -> np.ndarray:
    """generate_image (main.rs:85-114): tonemapped + gamma-corrected pixels."""
    img, _, _ = scene.generate_image(params)
    return tonemap_gamma(img)


def build_bvh(boxes: np.ndarray):
    """BVH::new over [n, 6] (min, max) boxes on the host -> (links [m,4], bounds [m,6], order [n], depth)."""
    boxes = np.ascontiguousarray(boxes, np.float64).reshape(-1, 6)
    n = C.c_uint64(0)
    depth = C.c_uint32(0)
    _check(lib().rt_bvh_build(boxes.ctypes.data_as(C.c_void_p), len(boxes), C.byref(n), None, None, None,
                              C.byref(depth)))
    links = np.zeros((n.value, 4), np.int64)
    bounds = np.zeros((n.value, 6), np.float64)
    order = np.zeros(len(boxes), np.uint64)
    _check(lib().rt_bvh_build(boxes.ctypes.data_as(C.c_void_p), len(boxes), C.byref(n),
                              links.ctypes.data_as(C.c_void_p), bounds.ctypes.data_as(C.c_void_p),
                              order.ctypes.data_as(C.c_void_p), C.byref(depth)))
    return links, bounds, order, depth.value


def byte_thresholds() -> np.ndarray:
    """The device epilogue's 255 byte thresholds on the tonemapped value (host only)."""
    out = np.zeros(255, np.float64)
    _check(lib().rt_byte_thresholds(out.ctypes.data_as(C.c_void_p)))
    return out


def sample_chunks(params: RenderParams):
    """(chunks, chunk_spp) of the device's work units for this frame (rt_sample_chunks)."""
    k, cs = C.c_uint32(), C.c_uint32()
    _check(lib().rt_sample_chunks(C.byref(params.to_c()), C.byref(k), C.byref(cs)))
    return k.value, cs.value


def probe_fp64(op: int, a: np.ndarray, b: Optional[np.ndarray] = None) -> np.ndarray:
    a = np.ascontiguousarray(a, np.float64)
    bb = None if b is None else np.ascontiguousarray(b, np.float64)
    out = np.zeros_like(a)
    _check(lib().rt_probe_fp64(op, a.ctypes.data_as(C.c_void_p),
                               None if bb is None else bb.ctypes.data_as(C.c_void_p), len(a),
                               out.ctypes.data_as(C.c_void_p)))
    return out
