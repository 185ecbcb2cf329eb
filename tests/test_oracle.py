"""CPU tests of the oracle (oracle/oracle.c): pinned against the reference's own
known-answer tests (tests/golden/kats.json), internally consistent (recursive
raytrace_impl vs the device's throughput form), and reproducing the committed
golden fixtures."""
import json
import math
import os

import numpy as np
import pytest

from conftest import REPO

GOLD = os.path.join(REPO, "tests", "golden")
with open(os.path.join(GOLD, "kats.json")) as f:
    KATS = json.load(f)


def cg_normalize(v):
    """cgmath normalize: v * (1 / sqrt((x*x + y*y) + z*z))."""
    x, y, z = (float(c) for c in v)
    inv = 1.0 / math.sqrt((x * x + y * y) + z * z)
    return [x * inv, y * inv, z * inv]


# ---------------------------------------------------------------- KATs ----
@pytest.mark.parametrize("kat", KATS["aabb"], ids=lambda k: k["name"])
def test_kat_aabb(orc, kat):
    d = cg_normalize(kat["dir"]) if kat["normalize"] else kat["dir"]
    t = orc.aabb_intersects(kat["min"], kat["max"], kat["origin"], d)
    assert t == kat["expected_t"]  # exact, as the reference's assert_eq!


@pytest.mark.parametrize("kat", KATS["box"], ids=lambda k: k["name"])
def test_kat_box(orc, kat):
    d = cg_normalize(kat["dir"])
    r = orc.box_intersection(kat["sizes"], kat["origin"], d)
    exp = kat["expected"]
    if exp is None:
        assert r is None
    else:
        t, n, inside = r
        assert t == exp["t"] and list(n) == exp["normal"] and inside == exp["inside"]


def test_kat_triangle_bbb(orc):
    k = KATS["triangle_bbb"]
    r = orc.triangle_intersection(k["a"] + k["b"] + k["c"], [0, 0, 0], [1, 0, 0, 0], k["origin"], k["dir"])
    assert r is None  # |det| < 1e-11 (triangle.rs:51)


def triangle_aaa_scene(rt):
    k = KATS["triangle_aaa"]
    a, ba, ca = (np.array(k[x]) for x in ("a", "ba", "ca"))
    mats = np.zeros(1, rt.MATERIAL_DTYPE)
    mats[0]["emission"] = (1.0, 1.0, 1.0)
    desc = rt.SceneDesc(materials=mats, shapes=np.zeros(0, rt.SHAPE_DTYPE),
                        tri_vertices=np.concatenate([a, a + ba, a + ca])[None, :],
                        tri_position=np.array([k["position"]]), tri_rotation=np.array([[1.0, 0, 0, 0]]),
                        tri_material=np.zeros(1, np.uint32))
    # TrianglePrimitive::new with no rotation: a' = a + pos; ba', ca' recomputed from b', c'
    pos = np.array(k["position"])
    a2 = a + pos
    b2 = (ba + a) + pos
    c2 = (ca + a) + pos
    ba2, ca2 = b2 - a2, c2 - a2
    world = (ba2 * k["u"] + ca2 * k["v"]) + a2
    o = np.array(k["pos"])
    d = np.array(cg_normalize(world + o))
    return desc, np.concatenate([o, d])[None, :]


def test_kat_triangle_aaa(rt, orc):
    desc, ray = triangle_aaa_scene(rt)
    imp, cnt = orc.OracleScene(desc).intersect_lights(ray)
    assert cnt[0] >= 1  # `called` (primitives/triangle.rs:125-127)


def test_kat_cof_aaa(orc):
    """cof(M)·n ∥ (Mᵀ)⁻¹·n for M = Rx(10°)·Ry(20°)·Rz(30°)·diag(2,3,4) (gltf/scene_builder.rs:408-426)."""
    k = KATS["cof_aaa"]

    def rx(t):  # cgmath Matrix3::from_angle_x, columns
        s, c = math.sin(t), math.cos(t)
        return np.array([[1, 0, 0], [0, c, s], [0, -s, c]]).T

    def ry(t):
        s, c = math.sin(t), math.cos(t)
        return np.array([[c, 0, -s], [0, 1, 0], [s, 0, c]]).T

    def rz(t):
        s, c = math.sin(t), math.cos(t)
        return np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]]).T

    ang = [a * (math.pi / 180.0) for a in k["angles_deg"]]
    m = rx(ang[0]) @ ry(ang[1]) @ rz(ang[2]) @ np.diag(k["scales"])
    cof = orc.cof3(m.T.reshape(9)).reshape(3, 3).T  # column-major in/out
    inv_t = np.linalg.inv(m.T)
    for n in k["normals"]:
        n = np.array(cg_normalize(n))
        a = cof @ n
        b = inv_t @ n
        np.testing.assert_allclose(a / np.linalg.norm(a), b / np.linalg.norm(b), atol=1e-15)


@pytest.mark.parametrize("v", KATS["philox4x32_10"], ids=["zero", "ones", "pi"])
def test_kat_philox(orc, v):
    assert list(orc.philox(v["ctr"], v["key"])) == v["out"]


# ------------------------------------------------------ sampler sanity ----
def test_rand_transforms(orc):
    seed = 1234
    # gen_range(0..n): uniform over n values
    draws = np.concatenate([orc.sampler_draws(seed, p, 0, 3, [5, 0, 0], 200)[:, 0] for p in range(20)])
    counts = np.bincount(draws.astype(int), minlength=5)
    assert counts.sum() == 4000 and counts.min() > 700
    # exact acceptance zone: power-of-two ranges never reject, so gen_range(0..2)
    # is the top bit of each u64 of the stream, one word pair per draw
    two = orc.sampler_draws(seed, 9, 1, 3, [2, 0, 0], 300)[:, 0]
    stream = orc.rng_stream_u64(seed, 9, 1, 300)
    assert np.array_equal(two.astype(np.uint64), stream >> np.uint64(63))
    assert np.all(orc.sampler_draws(seed, 9, 1, 3, [1, 0, 0], 50)[:, 0] == 0)
    # gen_bool(0.5)
    b = np.concatenate([orc.sampler_draws(seed, p, 1, 4, [0.5, 0, 0], 200)[:, 0] for p in range(20)])
    assert 1800 < b.sum() < 2200
    assert np.all(orc.sampler_draws(seed, 0, 0, 4, [1.0, 0, 0], 50)[:, 0] == 1)  # p == 1: ALWAYS_TRUE
    assert np.all(orc.sampler_draws(seed, 0, 0, 4, [0.0, 0, 0], 50)[:, 0] == 0)
    # inclusive [-1, 1] and half-open [0, 3)
    u = orc.sampler_draws(seed, 3, 0, 5, [-1.0, 1.0, 0], 2000)[:, 0]
    assert u.min() >= -1.0 and u.max() <= 1.0 and abs(u.mean()) < 0.08
    h = orc.sampler_draws(seed, 4, 0, 6, [0.0, 3.0, 0], 2000)[:, 0]
    assert h.min() >= 0.0 and h.max() < 3.0


def test_samplers_geometry(orc):
    s = np.array([0.25, 0.01, 0.5])
    pts = orc.sampler_draws(7, 0, 0, 1, s, 3000)
    on_face = np.isclose(np.abs(pts) / s, 1.0, rtol=0, atol=1e-15).any(axis=1)
    assert on_face.all() and (np.abs(pts) <= s + 1e-15).all()
    # faces chosen proportional to (sy*sz, sx*sz, sx*sy)
    face = np.argmax(np.isclose(np.abs(pts) / s, 1.0, rtol=0, atol=1e-15), axis=1)
    w = np.array([s[1] * s[2], s[0] * s[2], s[0] * s[1]])
    np.testing.assert_allclose(np.bincount(face, minlength=3) / len(face), w / w.sum(), atol=0.03)
    # the face's sign (the lowest bit of the choice draw): +-1 equally likely on each face
    sign = np.sign(pts[np.arange(len(pts)), face])
    assert set(np.unique(sign)) == {-1.0, 1.0}
    for f in range(3):
        on = sign[face == f]
        assert abs(on.mean()) < 4.0 / np.sqrt(max(len(on), 1)) + 1e-9, (f, len(on), on.mean())
    sph = orc.sampler_draws(7, 1, 0, 2, [0, 0, 0], 2000)
    np.testing.assert_allclose(np.linalg.norm(sph, axis=1), 1.0, atol=1e-15)
    n = np.array([0.0, 1.0, 0.0])
    cos = orc.sampler_draws(7, 2, 0, 0, n, 4000)
    np.testing.assert_allclose(np.linalg.norm(cos, axis=1), 1.0, atol=1e-15)
    assert (cos @ n > 0).mean() > 0.99


# -------------------------------------------- recursive vs device form ----
# Kitchen sink, pixel 33 (x 1, y 1), sample 213: the path hits the back wall, then the
# rotated emissive box twice; the second box bounce's Light::pdf query starts inside
# that box by rounding and its exit crossing gives t^2/|d.n| = NaN, as the reference
# computes it.  With ray_depth 3 that bounce is the last one: raytrace_impl's
# dot * col (x) 0 / pi / pdf is then NaN (raytrace.rs:32-33) and so is the pixel.
NAN_LAST_BOUNCE = dict(width=32, height=24, spp=214, ray_depth=3)


@pytest.mark.parametrize("scene,over", [
    ("cornell.txt", dict(width=32, height=24, spp=4)),
    ("kitchen_sink.txt", {}),
    ("kitchen_sink.txt", dict(width=16, height=12, spp=3, ray_depth=30, seed=5)),
    ("box_lights.txt", dict(width=16, height=12, spp=3)),
    ("kitchen_sink.txt", NAN_LAST_BOUNCE),
    ("kitchen_sink.txt", dict(NAN_LAST_BOUNCE, ray_depth=6)),
])
def test_recursive_vs_iterative(rt, orc, scene_text, scene, over):
    desc, params = rt.parse_scene(scene_text(scene))
    params = params.replace(**over)
    o = orc.OracleScene(desc)
    a, ha, sa = o.render(params, mode=0, hit_ids=True)
    b, hb, sb = o.render(params, mode=1, hit_ids=True)
    assert np.array_equal(ha, hb)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-300)  # NaNs in the same places
    if params.spp == 214:
        assert np.isnan(a[1, 1]).all() and np.isnan(a).sum() == 3
    for k in ("paths", "segments", "aabb_tests", "tri_tests", "shape_tests", "shaded_hits",
              "light_queries", "light_hits"):
        assert sa[k] == sb[k]


@pytest.mark.parametrize("seed", range(24))
def test_recursive_vs_iterative_fuzz(rt, orc, seed):
    """The two oracle forms on seeded random scenes (tests/fuzz_scenes.py): the same hit
    ids and counters, radiance within reassociation."""
    from fuzz_scenes import random_scene
    desc, params = rt.parse_scene(random_scene(seed, spp=3))
    o = orc.OracleScene(desc)
    a, ha, sa = o.render(params, mode=0, hit_ids=True)
    b, hb, sb = o.render(params, mode=1, hit_ids=True)
    assert np.array_equal(ha, hb)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-300)
    for k in ("paths", "segments", "aabb_tests", "tri_tests", "shape_tests", "shaded_hits",
              "light_queries", "light_hits"):
        assert sa[k] == sb[k]


def _layout_z(o, params):
    """Per-pixel z of (the build's stream layout) - (the reference's literal rand call
    order): two independent estimates of each pixel's mean, sigma from the per-sample
    variances.  Returns z over the pixels/channels with nonzero variance."""
    m0, s0, st0 = o.render_moments(params, mode=0)
    m2, s2, st2 = o.render_moments(params, mode=2)
    n = params.spp
    fin = np.isfinite(m0) & np.isfinite(m2)
    var = (np.maximum(s0 - m0 * m0, 0.0) + np.maximum(s2 - m2 * m2, 0.0)) / n
    ok = fin & (var > 0)
    assert np.array_equal(m0[fin & ~ok], m2[fin & ~ok])  # zero-variance pixels: identical constants
    return (m0[ok] - m2[ok]) / np.sqrt(var[ok]), st0, st2


@pytest.mark.parametrize("scene", ["cornell.txt", "kitchen_sink.txt", "box_lights.txt", "atrium"])
def test_layout_matches_literal_draw_order(rt, orc, scene_text, tmp_path, scene):
    """The build's RNG stream layout (block-aligned draws at each hit, one u32 Mix coin,
    shared A/B/C draws for both Mix branches, no index draw for one light, exact
    UniformInt zones) is the same ESTIMATOR as the reference's literal rand 0.8.5 call
    sequence (oracle mode 2: gen_bool(0.5) coin, per-branch draws, an index draw even for
    one light, gen_range(0..=1) for the box sign with rand's conservative zones;
    ray_sampler.rs:87-157, raytrace.rs:46): at 4096 spp per pixel both converged images
    agree within the per-pixel standard error (|z| <= 5 everywhere, mean z^2 ~ 1,
    few |z| > 3).  Box lights (rotated and axis-aligned), ellipsoid, triangle (custom
    and glTF) lights and dielectrics are covered."""
    if scene == "atrium":
        import subprocess
        import sys
        subprocess.run([sys.executable, os.path.join(REPO, "scenes", "gen_sponza_like.py"), str(tmp_path), "--scale",
                        "0.1", "--name", "atrium"], check=True, capture_output=True)
        desc, params = rt.load_gltf(str(tmp_path / "atrium.gltf"), 32, 24, 4096)
    else:
        desc, params = rt.parse_scene(scene_text(scene))
        params = params.replace(width=32, height=24, spp=4096)
    z, st0, st2 = _layout_z(orc.OracleScene(desc), params)
    assert z.size > 2000
    assert np.abs(z).max() <= 5.0, np.abs(z).max()
    assert 0.8 <= float(np.mean(z * z)) <= 1.25, float(np.mean(z * z))
    assert (np.abs(z) > 3).mean() <= 0.01
    # the same work per path in expectation: segment counts within 1%
    assert abs(st0["segments"] / st2["segments"] - 1.0) < 0.01


def test_chunked_sum_is_reassociation_only(rt, orc, scene_text):
    """Chunked sample runs (the device's work units) change only the f64 summation order."""
    desc, params = rt.parse_scene(scene_text("kitchen_sink.txt"))
    params = params.replace(width=12, height=10, spp=7)
    o = orc.OracleScene(desc)
    seq, hs, ss = o.render(params, mode=1, hit_ids=True)
    same, _, _ = o.render(params, mode=1, chunk_spp=7)
    assert np.array_equal(seq, same)
    for cs in (1, 2, 3, 5):
        ch, hc, sc = o.render(params, mode=1, hit_ids=True, chunk_spp=cs)
        assert np.array_equal(hs, hc) and ss == sc
        np.testing.assert_allclose(ch, seq, rtol=1e-13, atol=1e-300)


@pytest.mark.parametrize("w,h,spp,want", [
    (1920, 1080, 256, (32, 8)),     # C2/C3: 8-spp chunks (66M work units: short wave-tiles trim the 8-GPU tail)
    (3840, 2160, 1024, (16, 64)),   # C4: capped by the 4-GiB partial-sum budget (64 chunks: 12.7 GB)
    (1920, 1080, 64, (16, 4)),      # C5
    (256, 256, 64, (64, 1)),        # C1: capped at kMaxChunks
    (48, 32, 4, (4, 1)),
    (20, 12, 5, (3, 2)),            # 4 runs of 2 would leave one empty: trimmed to 3
    (4000, 4000, 9, (2, 5)),        # 16M pixels: two runs reach 32M work units
    (7, 3, 1, (1, 1)),
])
def test_sample_chunk_rule(rt, w, h, spp, want):
    k, cs = rt.sample_chunks(rt.RenderParams(w, h, spp))
    assert (k, cs) == want
    assert (k - 1) * cs < spp <= k * cs   # no empty run, all samples covered
    assert ((w + 15) // 16) * ((h + 15) // 16) * 256 * 3 * 8 * k <= 4 << 30  # partial sums within budget


def test_thread_count_independent(rt, orc, scene_text):
    desc, params = rt.parse_scene(scene_text("kitchen_sink.txt"))
    o = orc.OracleScene(desc)
    a, ha, _ = o.render(params, threads=1, hit_ids=True)
    b, hb, _ = o.render(params, threads=7, hit_ids=True)
    assert np.array_equal(a, b) and np.array_equal(ha, hb)


def test_row_window_matches_full(rt, orc, scene_text):
    desc, params = rt.parse_scene(scene_text("kitchen_sink.txt"))
    o = orc.OracleScene(desc)
    full, _, _ = o.render(params)
    part, _, st = o.render(params, rows=(10, 17))
    assert np.array_equal(full[10:17], part[10:17]) and st["paths"] == 7 * params.width * params.spp


@pytest.mark.parametrize("name", ["cornell_24x16_4spp", "kitchen_sink", "kitchen_sink_deep"])
def test_golden_fixtures(orc, name):
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import render_case
    g = np.load(os.path.join(GOLD, name + ".npz"))
    params, img, hits, stats = render_case(name)
    assert np.array_equal(img, g["image"])
    assert np.array_equal(hits, g["hit_ids"])
    assert np.array_equal(stats, g["stats"])


def test_light_scene_bvhs(rt, orc, scene_text):
    desc, params = rt.parse_scene(scene_text("kitchen_sink.txt"))
    o = orc.OracleScene(desc)
    nodes, depth = o.bvh_info()
    # 5 boxes and 6 ellipsoids need a split; the 4 triangles fit one leaf (bvh.rs:77)
    assert nodes[0] > 1 and nodes[1] > 1 and nodes[2] == 1
    # lights are copies in their own BVHs (scene.rs:209-213): 1 box, 1 ellipsoid, 1 triangle
    assert list(nodes[3:]) == [1, 1, 1]
    assert sorted(o.bvh_prims(3) + o.bvh_prims(4) + o.bvh_prims(5)) == [2, 3, 13]
