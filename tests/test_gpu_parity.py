"""GPU parity: the HIP path (through the C ABI) against the oracle.

Bar:
  * hit ids (pixel, sample, bounce) -> global primitive id: bit-exact vs the
    oracle (both the device-form and the recursive form of raytrace_impl);
  * mean radiance: bit-exact vs the oracle's iterative form (the device
    algorithm), and within REL_TOL per channel of the recursive restatement of
    raytrace_impl (raytrace.rs:12-60), whose summation order differs;
  * work counters (segments, AABB/triangle/shape tests, light queries) equal.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# recursive (e + f*(e + f*(...))) vs throughput (sum T*e) association: f64
# rounding only, a handful of ulps per bounce.
REL_TOL = 1e-12


@pytest.fixture(scope="module")
def cornell(rt, orc, scene_text):
    desc, params = rt.parse_scene(scene_text("cornell.txt"))
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


@pytest.fixture(scope="module")
def sink(rt, orc, scene_text):
    desc, params = rt.parse_scene(scene_text("kitchen_sink.txt"))
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


# the kernel form the current test runs (segment_form), applied by _compare
FORM = {}


@pytest.fixture(autouse=True, params=["fused", "resume", "resume_eager", "resume_f64", "resume_c64", "general"])
def segment_form(request):
    """Every test runs both path-kernel segment forms: fused (whole closest-hit
    query, then shading) and resumable (triangle traversal suspended while few
    lanes are live); the host picks one per scene (rt_tuning.resume).
    "resume_eager" suspends whenever any lane waits and tests every leaf at once
    (suspend_lanes=64, leaf_lanes=1: the far ends of the per-scene knobs the
    host picks, api.cpp path_suspend / path_leaf_batch).
    "general" is the fused form in its all-kinds instance (kinds=3) where the
    host would pick a shape-only or triangle-only one (api.cpp path_kinds).
    The resumable forms read a glTF scene's triangle BVH in its compact layout
    (f32 child boxes and vertices, exact copies: api.cpp path_compact);
    "resume_f64" forces the f64 layout in the same kernel; the auto forms read the compact
    layout's pair lines (two BVH levels per line, RT_LAYOUT_PAIR_NODES) where the scene has
    them, and "resume_c64" forces the compact layout's 64-B nodes (rt_tuning.compact = 1)."""
    FORM.clear()
    FORM["resume"] = 1 if request.param.startswith("resume") else 0
    if request.param == "resume_eager":
        FORM.update(suspend_lanes=64, leaf_lanes=1)
    if request.param == "resume_f64":
        FORM["compact"] = 0
    if request.param == "resume_c64":
        FORM["compact"] = 1
    if request.param == "general":
        FORM["kinds"] = 3
    yield request.param
    FORM.clear()


def form(scene, **extra):
    """Apply the current test's kernel form (+ extra fields) to a device scene."""
    t = {**FORM, **extra}
    if t.get("compact") == 1 and not scene.info()["layout_flags"] & 0x1:
        t.pop("compact")  # no compact triangle BVH: the scene's own form
    scene.set_tuning(**t)
    return scene


def _compare(gpu_scene, ora_scene, params, **tuning):
    form(gpu_scene, **tuning)
    _, chunk_spp = gpu_scene.sample_chunks(params)
    g_img, g_hits, g_st = gpu_scene.generate_image(params, hit_ids=True, stats=True)
    o_img, o_hits, o_st = ora_scene.render(params, mode=1, hit_ids=True, chunk_spp=chunk_spp)
    r_img, r_hits, _ = ora_scene.render(params, mode=0, hit_ids=True)
    assert np.array_equal(g_hits, o_hits), f"hit ids differ at {np.argwhere(g_hits != o_hits)[:5]}"
    assert np.array_equal(g_hits, r_hits)
    # NaN pixels (a NaN light pdf is reachable, test_last_bounce_nan) must sit in the same places
    assert np.array_equal(g_img, o_img, equal_nan=True), f"max |d| {np.nanmax(np.abs(g_img - o_img))}"
    # the product instances (no stats: the timed kernel, and hit ids without stats)
    p_img, p_hits, _ = gpu_scene.generate_image(params, hit_ids=True)
    assert np.array_equal(p_hits, o_hits) and np.array_equal(p_img, o_img, equal_nan=True)
    p_img, _, _ = gpu_scene.generate_image(params)
    assert np.array_equal(p_img, o_img, equal_nan=True), f"product kernel: max |d| {np.nanmax(np.abs(p_img - o_img))}"
    np.testing.assert_allclose(g_img, r_img, rtol=REL_TOL, atol=1e-300)  # equal_nan: the recursive form's NaNs
    for k in ("paths", "segments", "aabb_tests", "tri_tests", "shape_tests", "shaded_hits",
              "light_queries", "light_hits"):
        assert g_st[k] == o_st[k], (k, g_st[k], o_st[k])
    return g_img, g_hits, g_st


def test_fp64_rounding_matches_host(rt):
    """sqrt and division must round exactly like the host (the premise of bit-exactness)."""
    rng = np.random.default_rng(1)
    a = np.concatenate([rng.random(20000) * 10.0 ** rng.integers(-30, 30, 20000), [0.0, 1.0, 2.0, 1e-310, np.inf]])
    b = np.concatenate([rng.standard_normal(20000) * 10.0 ** rng.integers(-30, 30, 20000), [1.0, 3.0, 7.0, 3.0, 2.0]])
    assert np.array_equal(rt.probe_fp64(0, a), np.sqrt(a))
    assert np.array_equal(rt.probe_fp64(1, a, b), a / b)


def _split_division_pairs(n, seed):
    """Dividend/divisor pairs of dev_quot's range (rt_device.h): |x| in [2^-500, 2^402],
    |y| in [2^-360, 2^360], random signs; random mantissas plus the adversarial ones
    (all-ones, 1 + ulp, powers of two) and quotients near rounding ties."""
    rng = np.random.default_rng(seed)

    def dbl(mant, exp, sign):
        return np.ldexp(1.0 + mant * 2.0 ** -52, exp) * sign

    sx = rng.choice([-1.0, 1.0], n)
    sy = rng.choice([-1.0, 1.0], n)
    ex = rng.integers(-500, 402, n)
    ey = rng.integers(-360, 360, n)
    mx = rng.integers(0, 2 ** 52, n, dtype=np.uint64).astype(np.float64)
    my = rng.integers(0, 2 ** 52, n, dtype=np.uint64).astype(np.float64)
    special = np.array([0.0, 1.0, 2.0 ** 52 - 1, 2.0 ** 52 - 2, 2.0 ** 51, 2.0 ** 51 - 1, 1.0 + 2.0 ** 51])
    k = n // 4
    my[:k] = special[rng.integers(0, len(special), k)]
    mx[k:2 * k] = special[rng.integers(0, len(special), k)]
    x, y = dbl(mx, ex, sx), dbl(my, ey, sy)
    # x = y * q (rounded) for short q: exact or near-tie quotients
    q = rng.integers(1, 2 ** 20, k).astype(np.float64) * 2.0 ** rng.integers(-30, 30, k)
    x[2 * k:3 * k] = y[2 * k:3 * k] * q
    x[3 * k:] = np.nextafter(y[3 * k:] * q[: n - 3 * k], np.inf)
    ok = (np.abs(x) >= 2.0 ** -500) & (np.abs(x) <= 2.0 ** 402)
    return x[ok], y[ok]


def test_dev_quot_matches_host(rt):
    """The kernels' split division (dev_rcp once per divisor, dev_quot per dividend) is
    the device's own division without its rescaling steps: inside its range it must give
    the host's correctly rounded x / y bit for bit (rt_device.h)."""
    for seed in range(4):
        x, y = _split_division_pairs(1 << 20, seed)
        got = rt.probe_fp64(2, x, y)
        bad = np.flatnonzero(got.view(np.uint64) != (x / y).view(np.uint64))
        assert bad.size == 0, [(x[i], y[i], got[i], x[i] / y[i]) for i in bad[:5]]
        assert np.array_equal(rt.probe_fp64(1, x, y), x / y)
        # dev_quotf: the same pairs plus signed-zero dividends (the triangle and box
        # quotients' form, rt_device.h)
        z = np.resize(np.array([0.0, -0.0]), 4096)
        xz, yz = np.concatenate([x, z]), np.concatenate([y, y[:z.size]])
        got = rt.probe_fp64(5, xz, yz)
        bad = np.flatnonzero(got.view(np.uint64) != (xz / yz).view(np.uint64))
        assert bad.size == 0, [(xz[i], yz[i], got[i], xz[i] / yz[i]) for i in bad[:5]]


def test_dev_sqrt_matches_host(rt):
    """The kernels' sqrt core (rsq + Newton steps without the compiler's range
    scaling) and normalize's 1 / sqrt(d.d) give the host's bits on and off their
    fast ranges (rt_device.h dev_sqrt, dev_inv_len)."""
    rng = np.random.default_rng(3)
    x = np.ldexp(1.0 + rng.random(1 << 20), rng.integers(-1074, 1024, 1 << 20))
    x = np.concatenate([x, rng.random(1 << 18), 1.0 + rng.random(1 << 18) * 2.0,
                        [0.0, -0.0, np.inf, -1.0, np.nan, 5e-324, 2.0 ** -767, np.nextafter(2.0 ** -767, 0),
                         2.0 ** -700, 2.0 ** 700, np.nextafter(2.0 ** 700, np.inf), 1.0, 4.0]])
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        want_s, want_i = np.sqrt(x), 1.0 / np.sqrt(x)
    got_s, got_i = rt.probe_fp64(3, x), rt.probe_fp64(4, x)
    ok = ~np.isnan(want_s)
    assert np.array_equal(got_s[ok].view(np.uint64), want_s[ok].view(np.uint64))
    assert np.isnan(got_s[~ok]).all()
    ok = ~np.isnan(want_i)
    assert np.array_equal(got_i[ok].view(np.uint64), want_i[ok].view(np.uint64))
    assert np.isnan(got_i[~ok]).all()


def test_cornell_small(cornell, segment_form):
    desc, params, g, o = cornell
    _compare(g, o, params.replace(width=48, height=40, spp=4))
    # a shape-only scene has no compact triangle layout
    assert g.tuning()["compact"] == 0


def test_wide_frame(cornell, segment_form):
    """A frame with many wave-tiles per wave and long paths, in every form."""
    desc, params, g, o = cornell
    _compare(g, o, params.replace(width=96, height=64, spp=9, ray_depth=20, seed=5))


@pytest.mark.parametrize("waves", [3, 4, 5])
def test_both_register_budgets(cornell, waves):
    """Every register budget of the shape-only scene's fused kernel (3 waves/SIMD: the
    general instance; 4 and 5: the shape-only instance with T/L in LDS) is bit-exact
    (the host picks per scene)."""
    desc, params, g, o = cornell
    _compare(g, o, params.replace(width=40, height=24, spp=3, seed=3), waves=waves)
    # 5 exists for the shape-only fused form only: the resumable and the all-kinds
    # forms run (and report) 4
    t = g.tuning()
    assert t["waves"] == (4 if waves == 5 and not (t["kinds"] == 1 and t["resume"] == 0) else waves)


@pytest.mark.parametrize("chunk_spp", [37, 1])
def test_sample_ring_wraps(sink, chunk_spp):
    """Long sample runs: the 8-row commit ring wraps many times (37 + 3 rows per
    wave-tile); run length 1: one row per wave-tile, 40 partials per pixel."""
    desc, params, g, o = sink
    p = params.replace(width=20, height=12, spp=40, ray_depth=8, seed=17)
    _compare(g, o, p, chunk_spp=chunk_spp)
    assert g.sample_chunks(p) == ((40 + chunk_spp - 1) // chunk_spp, chunk_spp)


def test_cornell_seed_changes_image(cornell):
    desc, params, g, o = cornell
    p = params.replace(width=32, height=32, spp=2)
    a, _, _ = g.generate_image(p)
    b, _, _ = g.generate_image(p.replace(seed=7))
    assert not np.array_equal(a, b)
    a2, _, _ = g.generate_image(p)
    assert np.array_equal(a, a2), "render must be deterministic for a fixed seed"


def test_kitchen_sink(sink):
    desc, params, g, o = sink
    _compare(g, o, params)


@pytest.fixture(scope="module")
def box_lights(rt, orc, scene_text):
    desc, params = rt.parse_scene(scene_text("box_lights.txt"))
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


def test_shared_light_tests_cornell(cornell):
    """Cornell's only light is a box in the single-leaf box BVH: its light pdf
    comes from the next segment's box tests (boxes_slt), still bit-exact."""
    desc, params, g, o = cornell
    assert g.info()["shared_light_mask"] == 0b01  # the light box precedes the rotated box
    _compare(g, o, params.replace(width=32, height=24, spp=4, ray_depth=12))


@pytest.mark.parametrize("over", [dict(), dict(width=20, height=16, spp=3, ray_depth=30, seed=7),
                                  dict(width=9, height=7, spp=5, ray_depth=2, seed=11)])
def test_shared_light_tests_box_lights(box_lights, over):
    """Two box lights (one rotated, one also diffuse) mixed with non-light boxes:
    light pdfs from shared tests, several lights (index draws), rotated light
    normals, deep and shallow paths — hit ids, radiance and counters exact."""
    desc, params, g, o = box_lights
    assert g.info()["shared_light_mask"] == 0b101
    _compare(g, o, params.replace(**over))


def test_no_shared_light_tests_with_other_lights(sink):
    desc, params, g, o = sink
    assert g.info()["shared_light_mask"] == 0  # ellipsoid and triangle lights: separate queries


@pytest.mark.parametrize("depth", [3, 6])
def test_last_bounce_nan(sink, depth):
    """Pixel 33, sample 213 of the kitchen sink: the second bounce on the rotated light
    box has a NaN Light::pdf (its query ray starts inside the box by rounding; t^2/|d.n|
    = NaN, as the reference computes it).  At depth 3 that bounce is the LAST one:
    raytrace_impl's dot * col (x) 0 / pi / pdf is still NaN (raytrace.rs:32-33), so the
    pixel is NaN — the timed kernel shades the last segment like every other and applies
    that rule (render.hip segment_shade), bit-exact with the oracle incl. NaN places."""
    desc, params, g, o = sink
    p = params.replace(width=32, height=24, spp=214, ray_depth=depth)
    img, _, _ = _compare(g, o, p)
    assert np.isnan(img[1, 1]).all() and np.isnan(img).sum() == 3


@pytest.fixture(scope="module")
def sink_boxlight(rt, orc, scene_text):
    """The kitchen sink with only its rotated box emissive: every light is a box, so
    the timed kernel may skip last-bounce light queries (DevScene::lq_boxes)."""
    lines, seen = [], 0
    for line in scene_text("kitchen_sink.txt").split("\n"):
        if line.startswith("EMISSION"):
            seen += 1
            if seen > 1:
                continue
        lines.append(line)
    desc, params = rt.parse_scene("\n".join(lines))
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


def test_last_bounce_nan_box_light(sink_boxlight):
    """Pixel (21, 12), sample 406 (seed 10) of the box-light kitchen sink: the last
    bounce's light query starts on the rotated light box and its pdf is NaN, so the
    pixel is NaN (found with the oracle).  The timed kernel skips the last-bounce
    queries whose origin lies outside every light's grown world box — they cannot be
    NaN (render.hip lq_skippable) — and runs this one: the same NaN
    places, bit-exact elsewhere, in every kernel form; and skips do happen here
    (raw stats word 10, counted by the stats instance)."""
    desc, params, g, o = sink_boxlight
    p = params.replace(width=32, height=24, spp=407, ray_depth=3, seed=10)
    img, _, _ = _compare(g, o, p)
    assert np.isnan(img[12, 21]).all() and np.isnan(img).sum() == 3
    g.generate_image(p.replace(spp=4), stats=True)
    assert g.read_raw_stats(11)[10] > 0


def _sink_light_rotation(rt, orc, scene_text, rotation):
    """The box-light kitchen sink with its light box's ROTATION line replaced."""
    text = scene_text("kitchen_sink.txt")
    lines, seen = [], 0
    for line in text.split("\n"):
        if line.startswith("EMISSION"):
            seen += 1
            if seen > 1:
                continue
        lines.append(line)
    text = "\n".join(lines).replace("ROTATION 0.1 0.2 0 0.97467943448089633\nEMISSION",
                                     f"ROTATION {rotation}\nEMISSION", 1)
    assert f"ROTATION {rotation}" in text
    desc, params = rt.parse_scene(text)
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


@pytest.mark.parametrize("rotation,skips", [("0.1 0.2 0 0.9747", True), ("0.3 0.6 0 1.1", False)])
def test_last_bounce_skip_nonunit_light_rotation(rt, orc, scene_text, rotation, skips):
    """A light box whose ROTATION is not a unit quaternion (printed to 4 digits: |q|^2 =
    1.00004; or far from unit: 1.66).  cgmath's rotate_vector is then n R + (1 - n) I,
    not a rotation, and the light's true world box is pos + M^-1(+-h) (api.cpp lq_boxes
    inverts the model-space map instead of assuming R).  Near-unit: the skip stays on
    and the frame is bit-exact with the oracle, NaN places included; far from unit:
    the host turns the skip off (RT_LAYOUT_LQ_SKIP clear, no query skipped)."""
    desc, params, g, o = _sink_light_rotation(rt, orc, scene_text, rotation)
    assert bool(g.info()["layout_flags"] & 2) == skips
    for depth in (2, 3):
        _compare(g, o, params.replace(width=32, height=24, spp=48, ray_depth=depth, seed=10))
    g.generate_image(params.replace(width=32, height=24, spp=4, ray_depth=3), stats=True)
    assert (g.read_raw_stats(11)[10] > 0) == skips


def test_kitchen_sink_deep(sink):
    desc, params, g, o = sink
    _compare(g, o, params.replace(width=24, height=20, spp=3, ray_depth=24, seed=99))


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_shallow_depths(cornell, depth):
    desc, params, g, o = cornell
    _compare(g, o, params.replace(width=17, height=9, spp=2, ray_depth=depth))


def test_one_pixel_odd_sizes(cornell):
    desc, params, g, o = cornell
    _compare(g, o, params.replace(width=1, height=1, spp=5))
    _compare(g, o, params.replace(width=33, height=1, spp=1))
    _compare(g, o, params.replace(width=1, height=31, spp=1))


def test_fov_y_camera(cornell, rt):
    desc, params, g, o = cornell
    _compare(g, o, params.replace(width=20, height=30, spp=2, fov_axis=rt.RT_FOV_Y, fov=0.7))


def test_intersect_rays_random(sink, rt):
    desc, params, g, o = sink
    rng = np.random.default_rng(3)
    n = 20000
    orig = rng.uniform(-1.2, 1.2, (n, 3))
    d = rng.standard_normal((n, 3))
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh["prim"], oh["prim"])
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))


def intersect_device(rt, scene, rays, method):
    """rt_intersect_rays_async on HBM-resident rays -> host structured hits."""
    import torch
    d_rays = torch.from_numpy(np.ascontiguousarray(rays, np.float64)).cuda()
    d_hits = torch.zeros(len(rays) * rt.HIT_DTYPE.itemsize // 8, dtype=torch.float64, device="cuda")
    scene.intersect_async(d_rays.data_ptr(), len(rays), d_hits.data_ptr(), method,
                          torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_hits.cpu().numpy().view(rt.HIT_DTYPE)


@pytest.mark.parametrize("method", [0, 1])
def test_intersect_rays_device(sink, rt, method):
    """Device-buffer batch intersect, per-ray and persistent (lanes refilled from a
    queue) kernels: the oracle's hits bit for bit, incl. ragged batch sizes."""
    desc, params, g, o = sink
    rng = np.random.default_rng(13)
    for n in (1, 63, 65, 20011):
        rays = np.concatenate([rng.uniform(-1.2, 1.2, (n, 3)), rng.standard_normal((n, 3))], axis=1)
        gh, oh = intersect_device(rt, g, rays, method), o.intersect(rays)
        assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8)), n


def _tri_soup(rt, scale, n=400, seed=0):
    """Smooth-normal triangle soup (tri_mode GLTF) scaled by `scale`; every 7th is emissive."""
    rng = np.random.default_rng(seed)
    v = rng.uniform(-1, 1, (n, 1, 3)) + 0.25 * rng.standard_normal((n, 3, 3))
    nrm = rng.standard_normal((n, 3, 3))
    nrm /= np.linalg.norm(nrm, axis=2, keepdims=True)
    mats = np.zeros(2, rt.MATERIAL_DTYPE)
    mats[0]["color"] = [0.6, 0.6, 0.6]
    mats[1]["color"] = [1.0, 1.0, 1.0]
    mats[1]["emission"] = [2.0, 2.0, 2.0]
    return rt.SceneDesc(materials=mats, shapes=np.zeros(0, rt.SHAPE_DTYPE),
                        tri_vertices=(v * scale).reshape(n, 9), tri_normals=nrm.reshape(n, 9),
                        tri_material=(np.arange(n) % 7 == 0).astype(np.uint32), tri_mode=rt.RT_TRI_GLTF)


@pytest.mark.parametrize("scale", [1.0, 2.0 ** 420, 2.0 ** -420])
def test_slab_division_paths(rt, orc, scale):
    """Boxes inside the fdiv_fast range (scale 1) and outside it (2^+-420: guarded
    division everywhere) give the oracle's hits and light pdfs bit for bit."""
    desc = _tri_soup(rt, scale)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    rng = np.random.default_rng(8)
    n = 30000
    orig = rng.uniform(-1.5, 1.5, (n, 3)) * scale
    d = rng.standard_normal((n, 3))
    d[:50, 1] = 0.0          # axis-parallel rays: d == 0 slabs
    d[50:60] = [1e-200, 1.0, 0.5]  # a direction component below the fast range
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))
    if scale >= 1.0:  # at 2^-420 the determinant epsilon rejects every triangle, as in the reference
        assert (gh["prim"] >= 0).sum() > 1000
    dn = d / np.linalg.norm(d, axis=1, keepdims=True)
    pd = np.concatenate([orig, dn], axis=1)
    # at 2^420 the light areas overflow and Light::pdf is NaN, as in the
    # reference: NaNs must sit in the same places, everything else bit-equal
    assert np.array_equal(g.light_pdf(pd), o.light_pdf(pd), equal_nan=True)


def test_light_pdf_random(sink):
    desc, params, g, o = sink
    rng = np.random.default_rng(4)
    n = 20000
    pos = rng.uniform(-1.0, 1.0, (n, 3))
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pd = np.concatenate([pos, d], axis=1)
    gp, op = g.light_pdf(pd), o.light_pdf(pd)
    assert np.array_equal(gp, op)
    assert (gp > 0).sum() > 100


def test_tile_partition_matches_single(cornell, rt):
    """rt_render_tiles_async for world=3 ranks + unpack == rt_render."""
    torch = pytest.importorskip("torch")
    desc, params, g, o = cornell
    p = params.replace(width=70, height=45, spp=2)
    ref, _, _ = g.generate_image(p)
    world = 3
    per = g.tiles_per_rank(p, world)
    gathered = torch.zeros((world, per, 256, 3), dtype=torch.float64, device="cuda")
    for r in range(world):
        g.render_tiles_async(p, r, world, gathered[r].data_ptr())
    img = torch.zeros((p.height, p.width, 3), dtype=torch.float64, device="cuda")
    rt.unpack_tiles_async(p, world, gathered.data_ptr(), img.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy(), ref)


def test_workspace_ordered_across_streams(cornell, rt):
    """Calls on one scene issued on different streams share its workspace
    (queue, ring, partials): the library orders them with an event, so
    back-to-back launches on two streams with no host sync still give the
    single-stream result, rank after rank (rt_api.h Conventions: Streams)."""
    torch = pytest.importorskip("torch")
    desc, params, g, o = cornell
    p = params.replace(width=96, height=64, spp=8)
    ref, _, _ = g.generate_image(p)
    world = 4
    per = g.tiles_per_rank(p, world)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    gathered = torch.zeros((world, per, 256, 3), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for r in range(world):
        g.render_tiles_async(p, r, world, gathered[r].data_ptr(), streams[r % 2].cuda_stream)
    torch.cuda.synchronize()
    img = torch.zeros((p.height, p.width, 3), dtype=torch.float64, device="cuda")
    rt.unpack_tiles_async(p, world, gathered.data_ptr(), img.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy(), ref)
    assert torch.cuda.current_device() == 0  # the device guard restores the caller's device


def test_no_lights_scene(rt, orc):
    text = """DIMENSIONS 20 16
SAMPLES 3
BG_COLOR 0.5 0.6 0.7
CAMERA_POSITION 0 0 -3
NEW_PRIMITIVE
PLANE 0 1 0
POSITION 0 -1 0
COLOR 0.8 0.8 0.8
NEW_PRIMITIVE
ELLIPSOID 0.5 0.5 0.5
COLOR 0.9 0.2 0.2
"""
    desc, params = rt.parse_scene(text)
    _compare(rt.Scene(desc), orc.OracleScene(desc), params)


def test_empty_scene_is_background(rt, orc):
    desc, params = rt.parse_scene("DIMENSIONS 8 8\nSAMPLES 2\nBG_COLOR 0.25 0.5 1\n")
    g = rt.Scene(desc)
    img, hits, st = g.generate_image(params, hit_ids=True, stats=True)
    assert np.all(img == np.array([0.25, 0.5, 1.0]))
    assert np.all(hits[:, :, 0] == rt.RT_HIT_MISS) and np.all(hits[:, :, 1:] == rt.RT_HIT_NONE)
    _compare(g, orc.OracleScene(desc), params)


def _deep_chain(rt, n=200, cluster=149, g=1.3):
    """Coplanar triangles (y = 0) at geometrically growing z steps plus a cluster
    of identical ones: the reference builder makes a 21-level tree with a
    149-triangle leaf.  Rays lying in the plane hit every box and no triangle
    (det == 0), so the traversal stack grows to the tree depth — past the LDS
    short stack (spill) — and the big leaf takes the unpacked stack word
    (render.hip child_word).  A wall at the far end gives the rays a hit."""
    tris, z = [], 0.0
    for i in range(n):
        w = 0.01 * g ** i
        tris.append([(-1, 0, z), (1, 0, z), (0, 0, z + 0.5 * w)])
        if i == n // 2:
            tris += [[(-0.5, 0, z + 0.1 * w), (0.5, 0, z + 0.1 * w), (0, 0, z + 0.2 * w)]] * cluster
        z += w
    tris.append([(-3, -3, 1.5 * z), (3, -3, 1.5 * z), (0, 3, 1.5 * z)])
    v = np.array(tris, float)
    m = len(v)
    nrm = np.tile([0.0, 1.0, 0.0], (m, 3, 1))
    mats = np.zeros(2, rt.MATERIAL_DTYPE)
    mats[0]["color"] = [0.6, 0.6, 0.6]
    mats[1]["emission"] = [1.0, 1.0, 1.0]
    return rt.SceneDesc(materials=mats, shapes=np.zeros(0, rt.SHAPE_DTYPE), tri_vertices=v.reshape(m, 9),
                        tri_normals=nrm.reshape(m, 9), tri_material=(np.arange(m) % 2).astype(np.uint32),
                        tri_mode=rt.RT_TRI_GLTF)


def test_deep_stack_and_big_leaf(rt, orc):
    desc = _deep_chain(rt)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    info = g.info()
    assert info["bvh_depth"][2] > 12 + 6, info["bvh_depth"]   # the stack spills past the LDS part
    links, _, _, _ = rt.build_bvh(_tri_boxes(desc))
    assert (links[:, 3] - links[:, 2]).max() >= 128             # a leaf that does not pack
    rng = np.random.default_rng(12)
    n = 4096
    orig = np.stack([rng.uniform(-0.9, 0.9, n), np.zeros(n), np.full(n, -1.0)], axis=1)
    d = np.stack([rng.uniform(-1e-6, 1e-6, n), np.zeros(n), np.ones(n)], axis=1)
    d[: n // 2, 0] = 0.0
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))
    assert (gh["prim"][: n // 2] == len(desc.tri_material) - 1).all()   # straight rays reach the far wall
    pd = rays.copy()
    pd[:, 3:] /= np.linalg.norm(pd[:, 3:], axis=1, keepdims=True)
    assert np.array_equal(g.light_pdf(pd), o.light_pdf(pd))


def test_deep_stack_and_big_leaf_render(rt, orc):
    """The same 21-level chain with f32-exact coordinates, so the triangle BVH also has
    its compact layout (rt_layout.h DevNodeC): whole paths through the LDS + spill
    stack and the 149-triangle leaf (a kLeafRef child word) in every kernel form,
    the 4-wave instance forced so the resumable forms read the compact layout."""
    desc = _deep_chain(rt)
    desc.tri_vertices = desc.tri_vertices.astype(np.float32).astype(np.float64)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    info = g.info()
    assert info["layout_flags"] & 1 and info["bvh_depth"][2] > 12 + 6
    f = np.array([0.0, -0.4, 1.0]) / np.sqrt(1.16)
    u = np.array([0.0, 1.0, 0.4]) / np.sqrt(1.16)
    p = rt.RenderParams(width=24, height=16, spp=2, ray_depth=4, cam_position=(0.0, 0.5, -1.0),
                        cam_forward=tuple(f), cam_up=tuple(u), fov=0.9)
    img, _, st = _compare(g, o, p, waves=4)
    assert st["tri_tests"] > 0 and st["shaded_hits"] > 0


def test_progress_guard_single_row_tiles(rt, orc, segment_form):
    """the stats instance's progress guard (render.h kStatStall) on the
    regime of the round-5 livelock — one-row wave-tiles (chunk_spp 1), the queue's tail
    in 8 parts, a deep BVH with a spilling stack, the resumable forms: every wave must
    finish (a stalled wave makes rt_render fail, api.cpp copy_stats), and the frame is the
    oracle's bit for bit."""
    if not segment_form.startswith("resume"):
        pytest.skip("the guard's regime is the resumable kernel's suspend test")
    desc = _deep_chain(rt)
    desc.tri_vertices = desc.tri_vertices.astype(np.float32).astype(np.float64)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    f = np.array([0.0, -0.4, 1.0]) / np.sqrt(1.16)
    u = np.array([0.0, 1.0, 0.4]) / np.sqrt(1.16)
    p = rt.RenderParams(width=96, height=64, spp=48, ray_depth=3, cam_position=(0.0, 0.5, -1.0),
                        cam_forward=tuple(f), cam_up=tuple(u), fov=0.9, seed=21)
    _, _, st = _compare(g, o, p, waves=4, chunk_spp=1, tail_split=8)
    assert g.sample_chunks(p) == (48, 1) and g.tuning()["tail_split"] == 8
    assert g.read_raw_stats(15)[14] == 0 and st["paths"] == 96 * 64 * 48


def test_deep_stack_and_big_leaf_compact_trace(rt, orc):
    """The persistent batch trace kernel on the compact layout (rt_intersect_rays_async
    method 1): in-plane rays along the f32-exact chain push past the LDS stack into the
    spill area and reach the 149-triangle leaf through its kLeafRef child word."""
    desc = _deep_chain(rt)
    desc.tri_vertices = desc.tri_vertices.astype(np.float32).astype(np.float64)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    rng = np.random.default_rng(12)
    n = 4096
    orig = np.stack([rng.uniform(-0.9, 0.9, n), np.zeros(n), np.full(n, -1.0)], axis=1)
    d = np.stack([rng.uniform(-1e-6, 1e-6, n), np.zeros(n), np.ones(n)], axis=1)
    d[: n // 2, 0] = 0.0
    rays = np.concatenate([orig, d], axis=1)
    oh = o.intersect(rays)
    for compact in (-1, 0):
        g.set_tuning(compact=compact)
        gh = intersect_device(rt, g, rays, 1)
        assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8)), compact
    assert (oh["prim"][: n // 2] == len(desc.tri_material) - 1).all()


def _tri_boxes(desc):
    v = desc.tri_vertices.reshape(-1, 3, 3)
    return np.concatenate([v.min(1), v.max(1)], axis=1)


AXIS_SCENE = """DIMENSIONS 24 20
SAMPLES 3
RAY_DEPTH 8
BG_COLOR 0.1 0.1 0.1
CAMERA_POSITION 0 0 -2
NEW_PRIMITIVE
PLANE 0 1 0
POSITION 0 -1 0
COLOR 0.7 0.7 0.7
NEW_PRIMITIVE
PLANE 0 0 -1
POSITION 0 0 1
COLOR 0.6 0.6 0.6
NEW_PRIMITIVE
PLANE -1 0 0
POSITION 1 0 0
COLOR 0.2 0.8 0.2
NEW_PRIMITIVE
PLANE 1 0 0
POSITION -1 0 0
COLOR 0.8 0.2 0.2
NEW_PRIMITIVE
PLANE 0 -2 0
POSITION 0 1 0
COLOR 0.5 0.5 0.5
NEW_PRIMITIVE
BOX 0.25 0.5 0.25
POSITION 0.25 -0.5 0.5
COLOR 0.8 0.8 0.8
NEW_PRIMITIVE
BOX 0.25 0.125 0.25
POSITION 0 0.875 0
EMISSION 5 5 5
NEW_PRIMITIVE
ELLIPSOID 0.25 0.5 0.375
POSITION -0.5 0 0.25
EMISSION 2 3 4
COLOR 0.3 0.3 0.3
NEW_PRIMITIVE
ELLIPSOID 0.25 0.25 0.25
POSITION 0.5 0.25 -0.25
COLOR 1 1 1
DIELECTRIC
IOR 1.5
"""


ROTBOX_SCENE = """DIMENSIONS 20 16
SAMPLES 3
RAY_DEPTH 8
BG_COLOR 0.1 0.1 0.1
CAMERA_POSITION 0 0 -2
NEW_PRIMITIVE
PLANE 0 1 0
POSITION 0 -1 0
COLOR 0.7 0.7 0.7
NEW_PRIMITIVE
BOX 0.25 0.5 0.25
POSITION 0.25 -0.5 0.5
ROTATION 0 0.7071067811865476 0 0.7071067811865476
COLOR 0.8 0.8 0.8
NEW_PRIMITIVE
BOX 0.3 0.1 0.2
POSITION -0.5 0.25 0
ROTATION 0.2 0.3 0.1 0.9273618495495704
EMISSION 4 4 4
NEW_PRIMITIVE
BOX 0.125 0.25 0.5
POSITION 0 0.5 0.25
ROTATION 0 0 0.3826834323650898 0.9238795325112867
COLOR 0.5 0.6 0.7
METALLIC
"""


def test_rotated_box_edges(rt, orc):
    """Rotated boxes take the split division on their model-space ray when every lane
    of the wave has md dir_ok and |mo| <= 2^400 (render.hip box_model), the plain
    quotients otherwise.  Axis and diagonal directions give zero md components (the
    plain form), dyadic origins exact zeros in mo; hits, light sums and pdfs must equal
    the oracle's bit for bit."""
    desc, params = rt.parse_scene(ROTBOX_SCENE)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    rng = np.random.default_rng(5)
    n = 40000
    orig = rng.integers(-8, 9, (n, 3)) / 8.0
    orig[n // 2:] += rng.uniform(-1e-3, 1e-3, (n - n // 2, 3))
    d = rng.standard_normal((n, 3))
    d[:4000] = rng.integers(-2, 3, (4000, 3)) / 2.0
    d[:4000][np.all(d[:4000] == 0, axis=1)] = [1.0, 0.0, 0.0]
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))
    assert (gh["prim"] >= 1).sum() > n // 10  # boxes hit
    gi, gc = g.intersect_lights(rays)
    oi, oc = o.intersect_lights(rays)
    assert np.array_equal(gc, oc) and gc.sum() > 1000
    assert np.array_equal(gi.view(np.uint64), oi.view(np.uint64))
    dn = d / np.linalg.norm(d, axis=1, keepdims=True)
    pd = np.concatenate([orig, dn], axis=1)
    assert np.array_equal(g.light_pdf(pd).view(np.uint64), o.light_pdf(pd).view(np.uint64))
    _compare(g, o, params)


# Shapes rotated about one coordinate axis: every axis, both signs, a half turn
# (s = 0), a tiny angle, plus an emitting rotated box and ellipsoid (the light-pdf
# walk) and a two-axis rotation.
AXIS_ROT_SCENE = """DIMENSIONS 24 20
SAMPLES 3
RAY_DEPTH 8
BG_COLOR 0.1 0.1 0.1
CAMERA_POSITION 0 0 -2
NEW_PRIMITIVE
PLANE 0 1 0
POSITION 0 -1 0
COLOR 0.7 0.7 0.7
NEW_PRIMITIVE
BOX 0.25 0.5 0.125
POSITION 0.25 -0.5 0.5
ROTATION 0 0.17364817766693033 0 0.984807753012208
COLOR 0.8 0.8 0.8
NEW_PRIMITIVE
BOX 0.2 0.1 0.3
POSITION -0.5 0.5 0.25
ROTATION -0.3826834323650898 0 0 0.9238795325112867
COLOR 0.6 0.7 0.8
NEW_PRIMITIVE
BOX 0.125 0.25 0.2
POSITION 0.5 0.5 -0.25
ROTATION 0 0 1 0
COLOR 0.5 0.5 0.5
NEW_PRIMITIVE
BOX 0.3 0.05 0.3
POSITION 0 0.9 0
ROTATION 0 0 0.25881904510252074 0.9659258262890683
EMISSION 5 5 5
NEW_PRIMITIVE
BOX 0.2 0.2 0.2
POSITION -0.25 -0.5 -0.5
ROTATION 0 1e-20 0 1
COLOR 0.9 0.4 0.4
NEW_PRIMITIVE
ELLIPSOID 0.25 0.5 0.375
POSITION -0.5 -0.25 0.5
ROTATION 0 0 -0.7071067811865476 0.7071067811865476
EMISSION 2 3 4
COLOR 0.3 0.3 0.3
NEW_PRIMITIVE
ELLIPSOID 0.2 0.3 0.1
POSITION 0.5 0 0
ROTATION 0.5 0.5 0 0.7071067811865476
COLOR 0.9 0.9 0.9
METALLIC
"""


def test_axis_rotation_edges(rt, orc):
    """Rotated boxes and ellipsoids (model_space_ray through the quaternion rotation;
    round 4 measured an 11-operation single-axis form against it).  Rays
    from the shapes' centres and dyadic points (zero o - pos components), with zero,
    tiny (below and above 2^-400) and huge direction components: hits, light sums and
    pdfs must equal the oracle's bit for bit."""
    desc, params = rt.parse_scene(AXIS_ROT_SCENE)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    rng = np.random.default_rng(33)
    n = 40000
    orig = rng.uniform(-0.9, 0.9, (n, 3))
    orig[:4000] = rng.integers(-8, 9, (4000, 3)) / 8.0
    orig[4000:6000] = [[0.25, -0.5, 0.5], [-0.5, 0.5, 0.25], [0.5, 0.5, -0.25], [0.0, 0.9, 0.0]][0]
    d = rng.standard_normal((n, 3))
    d[6000:8000, 1] = 0.0
    d[8000:10000] *= np.array([1.0, 1e-125, 1.0])  # tiny components
    d[10000:12000] *= np.array([1e-110, 1.0, 1.0])  # tiny but in range
    d[12000:14000] *= 1e300                          # above range
    d[14000:16000] = rng.integers(-2, 3, (2000, 3)) / 2.0
    d[14000:16000][np.all(d[14000:16000] == 0, axis=1)] = [0.0, 0.0, 1.0]
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))
    assert (gh["prim"] >= 0).sum() > n // 2
    gi, gc = g.intersect_lights(rays)
    oi, oc = o.intersect_lights(rays)
    assert np.array_equal(gc, oc) and gc.sum() > 1000
    assert np.array_equal(gi.view(np.uint64), oi.view(np.uint64))
    fin = np.isfinite(np.linalg.norm(d, axis=1))
    dn = d[fin] / np.linalg.norm(d[fin], axis=1, keepdims=True)
    pd = np.concatenate([orig[fin], dn], axis=1)
    assert np.array_equal(g.light_pdf(pd).view(np.uint64), o.light_pdf(pd).view(np.uint64))
    _compare(g, o, params)


def test_fast_shape_edges(rt, orc):
    """Identity-rotation shapes and signed-axis planes take the exact unguarded
    division for ray_fast rays (rt_device.h shape_fast, plane_axis_t).  Dyadic
    origins put o - pos on exact zeros (generic fallback lanes), origins on box
    faces (signed-zero quotients), zero direction components (no fast ray) and
    a non-unit axis normal (generic plane): hits, raw light sums and pdfs must
    equal the oracle's bit for bit, incl. the signs of zeros."""
    desc, params = rt.parse_scene(AXIS_SCENE)
    g, o = rt.Scene(desc), orc.OracleScene(desc)
    rng = np.random.default_rng(21)
    n = 40000
    orig = rng.integers(-8, 9, (n, 3)) / 8.0             # on the shapes' dyadic grid
    orig[n // 2:] += rng.uniform(-1e-3, 1e-3, (n - n // 2, 3)) * (rng.random((n - n // 2, 3)) < 0.5)
    d = rng.standard_normal((n, 3))
    d[:2000, 0] = 0.0
    d[2000:4000] = rng.integers(-2, 3, (2000, 3)) / 2.0  # axis and diagonal directions, some zero
    d[2000:4000][np.all(d[2000:4000] == 0, axis=1)] = [0.0, 1.0, 0.0]
    rays = np.concatenate([orig, d], axis=1)
    gh, oh = g.intersect(rays), o.intersect(rays)
    assert np.array_equal(gh.view(np.uint8), oh.view(np.uint8))
    assert (gh["prim"] >= 0).sum() > n // 2
    gi, gc = g.intersect_lights(rays)
    oi, oc = o.intersect_lights(rays)
    assert np.array_equal(gc, oc) and gc.sum() > 1000
    assert np.array_equal(gi.view(np.uint64), oi.view(np.uint64))
    dn = d / np.linalg.norm(d, axis=1, keepdims=True)
    pd = np.concatenate([orig, dn], axis=1)
    assert np.array_equal(g.light_pdf(pd).view(np.uint64), o.light_pdf(pd).view(np.uint64))
    _compare(g, o, params)


def deep_shape_scene_text(n_side=14, layers=10, seed=7):
    """A shape-only scene with a few thousand rotated boxes and ellipsoids: shape BVHs
    deep enough that closest-hit and light walks push many levels (advisor round 4: the
    5-wave shape-only instance keeps no LDS stack, every push goes to the spill stack)."""
    rng = np.random.default_rng(seed)
    out = ["DIMENSIONS 64 48", "SAMPLES 3", "RAY_DEPTH 6", "BG_COLOR 0.1 0.12 0.15",
           "CAMERA_POSITION 0.05 0.4 -4.2", "CAMERA_RIGHT 1 0 0", "CAMERA_UP 0 1 0", "CAMERA_FORWARD 0 -0.08 1",
           "CAMERA_FOV_X 1.1", "", "NEW_PRIMITIVE", "PLANE 0 1 0", "POSITION 0 -1.2 0", "COLOR 0.6 0.6 0.6"]
    for i in range(n_side):
        for j in range(layers):
            for k in range(n_side):
                p = (np.array([i, j, k]) - np.array([n_side, layers, n_side]) / 2.0) * np.array([0.16, 0.18, 0.16])
                p = p + rng.uniform(-0.03, 0.03, 3)
                q = rng.standard_normal(4)
                q /= np.linalg.norm(q)
                kind = "BOX" if (i + j + k) % 2 == 0 else "ELLIPSOID"
                s = rng.uniform(0.02, 0.06, 3)
                out += ["", "NEW_PRIMITIVE", f"{kind} {float(s[0])!r} {float(s[1])!r} {float(s[2])!r}", f"POSITION {float(p[0])!r} {float(p[1])!r} {float(p[2])!r}",
                        f"ROTATION {float(q[1])!r} {float(q[2])!r} {float(q[3])!r} {float(q[0])!r}"]
                m = rng.integers(0, 10)
                if m == 0:
                    out.append("METALLIC")
                elif m == 1:
                    out.append("DIELECTRIC")
                    out.append("IOR 1.4")
                c = rng.uniform(0.2, 0.9, 3)
                out.append(f"COLOR {float(c[0])!r} {float(c[1])!r} {float(c[2])!r}")
    for x in (-0.7, 0.7):
        out += ["", "NEW_PRIMITIVE", "BOX 0.3 0.02 0.3", f"POSITION {x} 1.4 0.2", "EMISSION 5 5 4"]
    return "\n".join(out)


@pytest.fixture(scope="module")
def deep_shapes(rt, orc):
    desc, params = rt.parse_scene(deep_shape_scene_text())
    return desc, params, rt.Scene(desc), orc.OracleScene(desc)


@pytest.mark.parametrize("waves", [3, 4, 5])
def test_deep_shape_scene(deep_shapes, waves):
    """Every register budget of the shape-only fused kernel on deep shape BVHs (the 4/5-wave
    instances push every entry to the global spill stack, the 3-wave one keeps 12 in LDS) is
    bit-exact; the host picks 3 waves for shape BVHs this large (api.cpp path_waves)."""
    desc, params, g, o = deep_shapes
    info = g.info()
    assert max(info["bvh_depth"]) >= 10 and sum(info["bvh_nodes"]) > 64
    g.set_tuning()
    assert g.tuning()["waves"] == 3 and g.tuning()["kinds"] == 1 and g.tuning()["resume"] == 0
    _, _, st = _compare(g, o, params, waves=waves, resume=0)
    assert st["shape_tests"] > 0 and st["light_hits"] > 0


@pytest.mark.parametrize("chunk_spp", [0, 1, 3])
def test_tail_split_same_image(cornell, sink, chunk_spp):
    """The queue's last wave-tiles handed out in parts (rt_tuning.tail_split, render.hip
    queue_entry) and summed in sample order after the launch (tail_combine_kernel): the
    image is bit-identical for every split, and the oracle's.  Small frames have fewer
    wave-tiles than resident waves, so every wave-tile is a tail one here."""
    for desc, params, g, o in (cornell, sink):
        p = params.replace(width=40, height=24, spp=7, seed=9)
        ref = None
        for split in (1, 2, 3, 4, 8):
            g.set_tuning(tail_split=split, chunk_spp=chunk_spp)
            assert g.tuning()["tail_split"] == split
            img, _, st = g.generate_image(p, stats=True)
            if ref is None:
                ref = img
                _, cs = g.sample_chunks(p)
                o_img, _, o_st = o.render(p, mode=1, chunk_spp=cs)
                assert np.array_equal(img, o_img, equal_nan=True)
            assert np.array_equal(img, ref, equal_nan=True), split
        g.set_tuning()
