"""ctypes wrapper of the oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker / CPU baseline; never by the
product package.  See oracle.h for what the restatement covers and its parity
status ("parity pinned" by the reference's 13 KATs + Random123 Philox KATs;
the rest restates the reference operation by operation, "parity unpinned").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
# "portable": -O3 (built once, travels with the tree); "native": -O3 -march=native,
# built by `make native` on the machine that runs it (bench.py's cpu_baseline leg
# builds it on the GPU box's host)
LIB_PATHS = {"portable": LIB_PATH, "native": os.path.join(HERE, "build", "liboracle_native.so")}
_libs = {}


def build(quiet: bool = True, variant: str = "portable"):
    subprocess.run(["make", "-C", HERE, "all" if variant == "portable" else "native"], check=True,
                   capture_output=quiet)


def lib(variant: str = "portable"):
    if variant not in _libs:
        path = LIB_PATHS[variant]
        if not os.path.exists(path) or variant == "native":  # native: always for this host's CPU
            build(variant=variant)
        L = C.CDLL(path)
        vp, dp, u32, u64, i32 = C.c_void_p, C.POINTER(C.c_double), C.c_uint32, C.c_uint64, C.c_int
        sig = {
            "oracle_scene_create": (vp, [vp]),
            "oracle_scene_destroy": (None, [vp]),
            "oracle_scene_bvh_info": (None, [vp, vp, vp]),
            "oracle_scene_bvh_dump": (u64, [vp, i32, vp, vp]),
            "oracle_scene_bvh_prim": (C.c_int64, [vp, i32, u64]),
            "oracle_render": (i32, [vp, vp, i32, i32, u32, u32, vp, vp, vp]),
            "oracle_render_chunked": (i32, [vp, vp, i32, i32, u32, u32, u32, vp, vp, vp]),
            "oracle_render_moments": (i32, [vp, vp, i32, i32, u32, u32, vp, vp, vp]),
            "oracle_intersect_rays": (None, [vp, vp, u32, vp]),
            "oracle_light_pdf_rays": (None, [vp, vp, u32, vp]),
            "oracle_aabb_intersects": (i32, [dp, dp, dp, dp, dp]),
            "oracle_box_intersection": (i32, [dp, dp, dp, dp, dp, C.POINTER(i32)]),
            "oracle_ellipsoid_intersection": (i32, [dp, dp, dp, dp, dp, C.POINTER(i32)]),
            "oracle_plane_intersection": (i32, [dp, dp, dp, dp, dp]),
            "oracle_triangle_intersection": (i32, [dp, dp, dp, dp, dp, dp, dp, dp, C.POINTER(i32)]),
            "oracle_cof3": (None, [dp, dp]),
            "oracle_philox4x32_10": (None, [vp, vp, vp]),
            "oracle_rng_stream_u64": (None, [u64, u64, u32, u32, vp]),
            "oracle_sampler_draws": (None, [u64, u64, u32, i32, dp, u32, dp]),
            "oracle_tonemap_gamma": (None, [vp, u64, vp]),
            "oracle_ppm_bytes": (None, [vp, u64, vp]),
            "oracle_bvh_build": (u64, [vp, u64, vp, vp, vp, vp]),
            "oracle_intersect_lights_rays": (None, [vp, vp, u32, vp, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _libs[variant] = L
    return _libs[variant]


def _d(a):
    a = np.ascontiguousarray(a, np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


class OracleScene:
    """Scene::new restated on the CPU (oracle.c)."""

    def __init__(self, desc, variant: str = "portable"):
        self._L = lib(variant)
        d, keep = desc.to_c()
        self._h = self._L.oracle_scene_create(C.byref(d))
        del keep
        if not self._h:
            raise RuntimeError("oracle_scene_create failed")

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.oracle_scene_destroy(self._h)
            self._h = None

    def bvh_info(self):
        n = np.zeros(6, np.uint64)
        dep = np.zeros(6, np.uint32)
        self._L.oracle_scene_bvh_info(self._h, n.ctypes.data, dep.ctypes.data)
        return n, dep

    def bvh_dump(self, k: int):
        n = int(self._L.oracle_scene_bvh_dump(self._h, k, None, None))
        links = np.zeros((n, 4), np.int64)
        bounds = np.zeros((n, 6), np.float64)
        self._L.oracle_scene_bvh_dump(self._h, k, links.ctypes.data, bounds.ctypes.data)
        return links, bounds

    def bvh_prims(self, k: int):
        out = []
        i = 0
        while True:
            g = self._L.oracle_scene_bvh_prim(self._h, k, i)
            if g < 0:
                return out
            out.append(g)
            i += 1

    def render(self, params, mode: int = 1, threads: int = 0, rows=None, hit_ids: bool = False,
               chunk_spp: int = 0):
        """generate_image without tonemapping. mode 0 = recursive, 1 = iterative (device algorithm),
        2 = recursive with the reference's literal rand call sequence.
        chunk_spp > 0 sums samples in runs of chunk_spp like the device's chunked
        work units (oracle_render_chunked); 0 = the reference's sequential sum.
        Returns (image [H, W, 3], hit ids or None, stats dict)."""
        from_params = params.to_c()
        H, W = params.height, params.width
        r0, r1 = (0, H) if rows is None else rows
        img = np.zeros((H, W, 3), np.float64)
        hits = None
        if hit_ids:
            hits = np.full((H * W, params.spp, params.ray_depth), -2, np.int32)
        st = _stats_struct()
        rc = self._L.oracle_render_chunked(self._h, C.byref(from_params), mode, threads, r0, r1, chunk_spp,
                                         img.ctypes.data, None if hits is None else hits.ctypes.data, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_render failed: {rc}")
        return img, hits, {k: getattr(st, k) for k, _ in st._fields_}

    def render_moments(self, params, mode: int = 0, threads: int = 0):
        """(mean [H, W, 3], second moment [H, W, 3], stats): mode 0 = the build's stream
        layout (recursive form), 2 = the reference's literal rand call sequence."""
        H, W = params.height, params.width
        mean = np.zeros((H, W, 3), np.float64)
        sq = np.zeros((H, W, 3), np.float64)
        st = _stats_struct()
        rc = self._L.oracle_render_moments(self._h, C.byref(params.to_c()), mode, threads, 0, H, mean.ctypes.data,
                                         sq.ctypes.data, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_render_moments failed: {rc}")
        return mean, sq, {k: getattr(st, k) for k, _ in st._fields_}

    def intersect(self, rays):
        from importlib import import_module  # noqa: F401
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        out = np.zeros(len(rays), HIT_DTYPE)
        self._L.oracle_intersect_rays(self._h, rays.ctypes.data, len(rays), out.ctypes.data)
        return out

    def intersect_lights(self, rays):
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        imp = np.zeros(len(rays), np.float64)
        cnt = np.zeros(len(rays), np.uint32)
        self._L.oracle_intersect_lights_rays(self._h, rays.ctypes.data, len(rays), imp.ctypes.data, cnt.ctypes.data)
        return imp, cnt

    def light_pdf(self, pos_dir):
        pos_dir = np.ascontiguousarray(pos_dir, np.float64).reshape(-1, 6)
        out = np.zeros(len(pos_dir), np.float64)
        self._L.oracle_light_pdf_rays(self._h, pos_dir.ctypes.data, len(pos_dir), out.ctypes.data)
        return out


HIT_DTYPE = np.dtype([("t", "<f8"), ("geometry_normal", "<f8", 3), ("shading_normal", "<f8", 3),
                      ("inside", "<i4"), ("prim", "<i4")])


def _stats_struct():
    class rt_stats(C.Structure):
        _fields_ = [("paths", C.c_uint64), ("segments", C.c_uint64), ("aabb_tests", C.c_uint64),
                    ("tri_tests", C.c_uint64), ("shape_tests", C.c_uint64), ("shaded_hits", C.c_uint64),
                    ("light_queries", C.c_uint64), ("light_hits", C.c_uint64), ("kernel_ms", C.c_double),
                    ("total_ms", C.c_double), ("lane_steps", C.c_uint64), ("wave_steps", C.c_uint64)]
    return rt_stats()


def build_bvh(boxes):
    """BVH::new over [n, 6] boxes -> (links [m,4], bounds [m,6], order [n], depth)."""
    boxes = np.ascontiguousarray(boxes, np.float64).reshape(-1, 6)
    m = int(lib().oracle_bvh_build(boxes.ctypes.data, len(boxes), None, None, None, None))
    links = np.zeros((m, 4), np.int64)
    bounds = np.zeros((m, 6), np.float64)
    order = np.zeros(len(boxes), np.uint64)
    depth = np.zeros(1, np.uint32)
    lib().oracle_bvh_build(boxes.ctypes.data, len(boxes), links.ctypes.data, bounds.ctypes.data, order.ctypes.data,
                           depth.ctypes.data)
    return links, bounds, order, int(depth[0])


# ----------------------------------------------------------- KAT hooks ----
def aabb_intersects(mn, mx, o, d):
    t = C.c_double()
    args = [_d(x) for x in (mn, mx, o, d)]
    ok = lib().oracle_aabb_intersects(*[a[1] for a in args], C.byref(t))
    return t.value if ok else None


def box_intersection(sizes, o, d):
    t, n, ins = C.c_double(), np.zeros(3), C.c_int()
    args = [_d(x) for x in (sizes, o, d)]
    ok = lib().oracle_box_intersection(*[a[1] for a in args], C.byref(t), n.ctypes.data_as(C.POINTER(C.c_double)),
                                       C.byref(ins))
    return (t.value, n, bool(ins.value)) if ok else None


def ellipsoid_intersection(r, o, d):
    t, n, ins = C.c_double(), np.zeros(3), C.c_int()
    args = [_d(x) for x in (r, o, d)]
    ok = lib().oracle_ellipsoid_intersection(*[a[1] for a in args], C.byref(t),
                                             n.ctypes.data_as(C.POINTER(C.c_double)), C.byref(ins))
    return (t.value, n, bool(ins.value)) if ok else None


def plane_intersection(nrm, o, d):
    t, n = C.c_double(), np.zeros(3)
    args = [_d(x) for x in (nrm, o, d)]
    ok = lib().oracle_plane_intersection(*[a[1] for a in args], C.byref(t), n.ctypes.data_as(C.POINTER(C.c_double)))
    return (t.value, n) if ok else None


def triangle_intersection(abc, pos, rot, o, d):
    t, ng, ns, ins = C.c_double(), np.zeros(3), np.zeros(3), C.c_int()
    args = [_d(x) for x in (abc, pos, rot, o, d)]
    ok = lib().oracle_triangle_intersection(*[a[1] for a in args], C.byref(t),
                                            ng.ctypes.data_as(C.POINTER(C.c_double)),
                                            ns.ctypes.data_as(C.POINTER(C.c_double)), C.byref(ins))
    return (t.value, ng, ns, bool(ins.value)) if ok else None


def cof3(m_colmajor):
    a, p = _d(np.asarray(m_colmajor, np.float64).reshape(9))
    out = np.zeros(9)
    lib().oracle_cof3(p, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def philox(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(c.ctypes.data, k.ctypes.data, out.ctypes.data)
    return out


def rng_stream_u64(seed, pixel, sample, n):
    out = np.zeros(n, np.uint64)
    lib().oracle_rng_stream_u64(seed, pixel, sample, n, out.ctypes.data)
    return out


def sampler_draws(seed, pixel, sample, kind, arg, n):
    a, p = _d(np.asarray(arg, np.float64).reshape(3))
    out = np.zeros((n, 3))
    lib().oracle_sampler_draws(seed, pixel, sample, kind, p, n, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def tonemap_gamma(img):
    a = np.ascontiguousarray(img, np.float64)
    out = np.empty_like(a)
    lib().oracle_tonemap_gamma(a.ctypes.data, a.size // 3, out.ctypes.data)
    return out


def ppm_bytes(rgb):
    a = np.ascontiguousarray(rgb, np.float64)
    out = np.zeros(a.size, np.uint8)
    lib().oracle_ppm_bytes(a.ctypes.data, a.size // 3, out.ctypes.data)
    return out
