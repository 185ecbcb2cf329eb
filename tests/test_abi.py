"""CPU tests of the product library (no device calls): every symbol the C ABI
header declares is exported, the host-side pieces (custom-scene parser, BVH
builder, ACES/gamma/PPM output surface) match the oracle / the reference's
rules, and the hot path refuses to run without a GPU (no CPU fallback)."""
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "rt_api.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported(rt):
    import ctypes
    lib = ctypes.CDLL(rt.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(rt.EXPORTS), set(names) ^ set(rt.EXPORTS)


def test_version_and_errors(rt):
    assert rt.lib().rt_api_version() == 6
    with pytest.raises(rt.RtError) as e:
        rt.parse_scene("NEW_PRIMITIVE\nBOX 1 2\n")
    assert e.value.code == -4


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_no_cpu_fallback(rt, scene_text):
    assert rt.device_count() == 0
    desc, params = rt.parse_scene(scene_text("cornell.txt"))
    with pytest.raises(rt.RtError) as e:
        rt.Scene(desc)
    assert e.value.code == -2 and "no HIP device" in str(e.value)
    for peer in (False, True):  # the multi-GPU entry refuses the same way
        with pytest.raises(rt.RtError) as e:
            rt.MultiScene(desc, [0, 1], peer=peer)
        assert e.value.code == -2 and "no HIP device" in str(e.value)


def test_multi_argument_errors(rt, scene_text):
    """rt_multi_* reject bad arguments before touching a device."""
    import ctypes as C
    L = rt.lib()
    desc, params = rt.parse_scene(scene_text("cornell.txt"))
    d, keep = desc.to_c()
    h = C.c_void_p()
    devs = (C.c_int * 1)(0)
    assert L.rt_multi_create(C.byref(d), devs, 0, 0, C.byref(h)) == -1       # no devices
    assert L.rt_multi_create(C.byref(d), devs, 1, 0x80, C.byref(h)) == -1    # unknown flag
    assert L.rt_multi_create(None, devs, 1, 0, C.byref(h)) == -1
    p = params.to_c()
    assert L.rt_multi_render(None, C.byref(p), None, None, None) == -1
    assert L.rt_multi_scene(None, 0) is None
    L.rt_multi_destroy(None)  # no-op
    del keep


def test_tuning_argument_errors(rt):
    """rt_scene_set_tuning / get_tuning / sample_chunks refuse a NULL scene (no env knobs exist)."""
    import ctypes as C
    L = rt.lib()
    t = rt.rt_tuning(**rt.TUNING_AUTO)
    assert L.rt_scene_set_tuning(None, C.byref(t)) == -1
    assert L.rt_scene_get_tuning(None, C.byref(t)) == -1
    k, cs = C.c_uint32(), C.c_uint32()
    p = rt.RenderParams(64, 64).to_c()
    assert L.rt_scene_sample_chunks(None, C.byref(p), C.byref(k), C.byref(cs)) == -1
    src = open(os.path.join(REPO, "cpu-raytracing-rt_amd", "csrc", "api.cpp")).read()
    assert "getenv" not in src  # the kernel form is a property of the scene handle


# ------------------------------------------------------------- parser ----
def test_parse_cornell(rt, scene_text):
    desc, p = rt.parse_scene(scene_text("cornell.txt"))
    assert (p.width, p.height, p.spp, p.ray_depth) == (256, 256, 64, 16)
    assert p.fov == 0.9 and p.fov_axis == rt.RT_FOV_X
    assert list(desc.shapes["type"]) == [0, 0, 0, 0, 0, 1, 1, 2, 2]
    assert list(desc.materials["kind"]) == [0, 0, 0, 0, 0, 0, 0, 2, 1]
    assert desc.materials["ior"][7] == 1.5
    assert list(desc.materials["emission"][5]) == [10, 10, 10]
    # ROTATION x y z w -> (s, x, y, z) = (w, x, y, z) (scene_parser.rs:51-57)
    assert list(desc.shapes["rotation"][6]) == [0.984807753012208, 0, 0.17364817766693033, 0]
    assert list(desc.shapes["rotation"][0]) == [1, 0, 0, 0]


def test_parse_defaults(rt):
    """Scene::new / CameraParams::new defaults (scene.rs:167-191)."""
    desc, p = rt.parse_scene("DIMENSIONS 3 2\nCAMERA_FORWARD 0 0 2\nCAMERA_UP 0 3 0\n")
    assert (p.spp, p.ray_depth, p.bg_color) == (64, 16, (0.0, 0.0, 0.0))
    assert p.cam_forward == (0.0, 0.0, 1.0) and p.cam_up == (0.0, 1.0, 0.0)  # normalised
    assert p.fov == np.pi / 2 and p.cam_position == (0.0, 0.0, 0.0)
    assert len(desc.shapes) == 0 and len(desc.tri_material) == 0


def test_parse_ignores_unknown_and_blank(rt):
    desc, p = rt.parse_scene("garbage line\n\n  \nDIMENSIONS 4 4\nWHATEVER 1 2 3\nNEW_PRIMITIVE\nPLANE 0 1 0\n")
    assert len(desc.shapes) == 1


def test_parse_triangles_and_props(rt):
    text = ("DIMENSIONS 8 8\nNEW_PRIMITIVE\nTRIANGLE 0 0 0 1 0 0 0 1 0\nPOSITION 1 2 3\n"
            "ROTATION 0 0 0.5 0.5\nCOLOR 0.1 0.2 0.3\nMETALLIC\nRAY_DEPTH 3\nSAMPLES 5\nBG_COLOR 1 1 1\n")
    desc, p = rt.parse_scene(text)
    assert p.ray_depth == 3 and p.spp == 5 and p.bg_color == (1.0, 1.0, 1.0)
    assert list(desc.tri_vertices[0]) == [0, 0, 0, 1, 0, 0, 0, 1, 0]
    assert list(desc.tri_position[0]) == [1, 2, 3]
    assert list(desc.tri_rotation[0]) == [0.5, 0, 0, 0.5]
    assert desc.materials["kind"][0] == rt.RT_MAT_METALLIC


@pytest.mark.parametrize("text", [
    "NEW_PRIMITIVE\nPLANE 0 1 0\n",                           # no DIMENSIONS (scene.rs:188 unwrap)
    "DIMENSIONS 4 4\nPLANE 0 1 0\n",                          # property before NEW_PRIMITIVE
    "DIMENSIONS 4 4\nNEW_PRIMITIVE\nCOLOR 1 1 1\n",           # primitive without shape
    "DIMENSIONS 4 4\nNEW_PRIMITIVE\nBOX 1 1 1\nDIELECTRIC\n",  # DIELECTRIC without IOR
    "DIMENSIONS 4 4\nNEW_PRIMITIVE\nBOX 1 x 1\n",             # f64 parse error
    "DIMENSIONS 4\n",                                         # missing token
    "DIMENSIONS 4 4\nRAY_DEPTH 300\n",                        # u8 overflow
])
def test_parse_errors(rt, text):
    with pytest.raises(rt.RtError) as e:
        rt.parse_scene(text)
    assert e.value.code == -4


# --------------------------------------------------------- BVH builder ----
def _boxes(rng, n, grid=False):
    c = rng.integers(0, 4, (n, 3)).astype(float) if grid else rng.uniform(-10, 10, (n, 3))
    h = rng.uniform(0.01, 1.0, (n, 3))
    return np.concatenate([c - h, c + h], axis=1)


@pytest.mark.parametrize("n,grid", [(1, False), (4, False), (5, False), (37, False), (500, False),
                                    (300, True), (2000, True)])
def test_bvh_builder_matches_oracle(rt, orc, n, grid):
    """Product builder == oracle builder node for node (bvh.rs:75-140), incl. equal-midpoint ties."""
    boxes = _boxes(np.random.default_rng(n), n, grid)
    a = rt.build_bvh(boxes)
    b = orc.build_bvh(boxes)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3] == b[3]
    links = a[0]
    leaves = links[links[:, 0] < 0]
    assert (leaves[:, 3] - leaves[:, 2]).sum() == n  # every primitive in exactly one leaf
    assert sorted(a[2].tolist()) == list(range(n))


@pytest.mark.parametrize("case", ["random", "grid_ties", "identical", "clustered"])
def test_bvh_parallel_builder_matches_oracle(rt, orc, case):
    """Above 200k primitives the presorted builder splits subtrees off to threads; the
    tree must still equal the reference restatement's node for node (incl. leaf order)."""
    n = 210000
    rng = np.random.default_rng(11)
    if case == "random":
        boxes = _boxes(rng, n)
    elif case == "grid_ties":      # integer centres: heavy equal-midpoint ties on every axis
        boxes = _boxes(rng, n, grid=True)
    elif case == "identical":      # SAH finds no gain at the root: one 210k leaf in axis-2 order
        boxes = np.tile([0, 0, 0, 1, 1, 1.0], (n, 1))
    else:                          # a dense cluster plus far outliers (deep, unbalanced tree)
        boxes = _boxes(rng, n)
        boxes[: n // 2] *= 1e-3
    a, b = rt.build_bvh(boxes), orc.build_bvh(boxes)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3] == b[3]


def test_bvh_builders_match_above_parallel_sort(rt, orc):
    """1.2M primitives: the oracle sorts ranges >= 1M with its parallel merge sort and
    builds subtrees as OpenMP tasks (oracle.c psort, build_sub); still the product
    builder's tree node for node."""
    boxes = _boxes(np.random.default_rng(5), 1_200_000)
    a, b = rt.build_bvh(boxes), orc.build_bvh(boxes)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3] == b[3]


def test_bvh_same_boxes_is_one_leaf(rt):
    """SAH finds no gain on identical boxes -> one leaf holding all of them (bvh.rs:93-96)."""
    boxes = np.tile([0, 0, 0, 1, 1, 1.0], (9, 1))
    links, bounds, order, depth = rt.build_bvh(boxes)
    assert len(links) == 1 and links[0, 3] == 9 and depth == 1


# ---------------------------------------------------- output surface ----
def test_tonemap_gamma_matches_oracle(rt, orc):
    x = np.random.default_rng(0).uniform(-1, 30, (64, 3))
    x[0] = [0.0, np.nan, np.inf]
    a, b = rt.tonemap_gamma(x), orc.tonemap_gamma(x)
    assert np.array_equal(a, b, equal_nan=True)


def _aces(x):  # postprocessing.rs:9-28 with the host/device op order (post.cpp aces)
    v = ((2.51 * x + 0.03) * x) / ((2.43 * x + 0.59) * x + 0.14)
    return np.where(v < 0.0, 0.0, np.where(v > 1.0, 1.0, v))


def test_byte_thresholds_reproduce_host_bytes(rt, orc):
    """The device epilogue's byte = #thresholds <= aces(x) (post_dev.hip) equals the host
    path's round(clamp(pow(aces(x), 1/2.2)) * 255) (postprocessing.rs:5-7, ppm.rs:13-15)
    on random radiance and on inputs packed around every byte boundary."""
    thr = rt.byte_thresholds()
    assert thr.shape == (255,) and np.all(np.diff(thr) > 0) and thr[0] > 0 and thr[-1] <= 1.0
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(0, 40.0, 1 << 20) * rng.uniform(0, 1, 1 << 20) ** 4,
                        [0.0, -0.0, np.nan, np.inf, -np.inf, -1.0, 1e-300, 1e300, 0.18]])
    # preimages of the thresholds under aces (a quadratic), then +-64 ulps around each
    t = thr[:, None]
    A, B, Cq = 2.51 - 2.43 * t, 0.03 - 0.59 * t, -0.14 * t
    x0 = ((-B + np.sqrt(B * B - 4 * A * Cq)) / (2 * A)).ravel()
    steps = np.arange(-64, 65)
    near = (x0[:, None].view(np.int64) + steps[None, :]).view(np.float64).ravel()
    x = np.concatenate([x, near])
    with np.errstate(invalid="ignore", over="ignore"):
        a = _aces(x)
    dev_model = np.searchsorted(thr, a, side="right").astype(np.uint8)
    dev_model[np.isnan(a)] = 0
    host = orc.ppm_bytes(orc.tonemap_gamma(np.ascontiguousarray(x.reshape(-1, 1).repeat(3, 1)))).reshape(-1, 3)[:, 0]
    assert np.array_equal(dev_model, host)
    assert set(range(1, 256)) <= set(np.unique(host[len(x) - len(near):]).tolist())  # every boundary exercised


def test_ppm_writer(rt, orc, tmp_path):
    rgb = np.random.default_rng(1).uniform(-0.2, 1.2, (5, 7, 3))
    rgb[0, 0] = [0.5 / 255, 1.5 / 255, np.nan]  # round half away from zero; NaN -> 0
    path = str(tmp_path / "x.ppm")
    rt.save_to_ppm(path, rgb)
    data = open(path, "rb").read()
    head = b"P6\n7 5\n255\n"
    assert data.startswith(head)
    assert np.array_equal(np.frombuffer(data[len(head):], np.uint8), orc.ppm_bytes(rgb))
    assert list(data[len(head):len(head) + 3]) == [1, 2, 0]
