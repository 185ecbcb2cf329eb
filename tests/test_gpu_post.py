"""GPU output surface: device tonemap + gamma + PPM
bytes, standalone and fused into the tile unpack, against the host/oracle
path (postprocessing.rs:5-37, ppm.rs:13-19).

Bar: bytes equal to the oracle's everywhere, bit for bit.  The device computes
aces_tonemap with the host's IEEE operations and turns the tonemapped value
into a byte by a search over the 255 thresholds the host derives from its own
pow (post.cpp byte_thresholds, proven exact), so no device libm rounding can
move a byte; the inputs include values packed around every byte boundary."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _host_bytes(orc, rgb):
    return orc.ppm_bytes(orc.tonemap_gamma(rgb.reshape(-1, 3))).reshape(-1)


def _check(dev, host, n):
    assert dev.shape == host.shape and dev.size == n
    bad = np.flatnonzero(dev != host)
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}: {dev[bad[:5]]} vs {host[bad[:5]]}"


def _boundary_inputs(rt):
    """Radiance values whose tonemapped value sits within +-64 ulps of every byte threshold."""
    thr = rt.byte_thresholds()[:, None]
    A, B, C = 2.51 - 2.43 * thr, 0.03 - 0.59 * thr, -0.14 * thr
    x0 = ((-B + np.sqrt(B * B - 4 * A * C)) / (2 * A)).ravel()   # aces^-1(threshold)
    return (x0[:, None].view(np.int64) + np.arange(-64, 65)[None, :]).view(np.float64).ravel()


def test_tonemap_bytes_random(rt, orc):
    rng = np.random.default_rng(2)
    near = _boundary_inputs(rt)
    n = (1 << 20) + len(near) // 3 + 1
    m = 3 * n - 12 - len(near)
    x = np.concatenate([rng.uniform(-0.5, 40.0, m) * rng.uniform(0, 1, m) ** 3, near,
                        [0.0, -0.0, np.nan, np.inf, -np.inf, 1e-300, 1e300, 0.18, 1.0, 2.0, 5.0, 1e-3]])
    dx = torch.from_numpy(x).cuda()
    out = torch.empty(3 * n, dtype=torch.uint8, device="cuda")
    rt.tonemap_bytes_async(dx.data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize()
    _check(out.cpu().numpy(), _host_bytes(orc, x), 3 * n)


def test_unpack_bytes_matches_host_ppm(rt, orc, scene_text):
    """Render tiles for 2 ranks, gather, fused unpack -> bytes == host tonemap of the mean image."""
    desc, params = rt.parse_scene(scene_text("cornell.txt"))
    p = params.replace(width=70, height=45, spp=3)
    g = rt.Scene(desc)
    world = 2
    per = g.tiles_per_rank(p, world)
    gathered = torch.zeros((world, per, 256, 3), dtype=torch.float64, device="cuda")
    for r in range(world):
        g.render_tiles_async(p, r, world, gathered[r].data_ptr())
    b = torch.empty((p.height, p.width, 3), dtype=torch.uint8, device="cuda")
    rt.unpack_tiles_bytes_async(p, world, gathered.data_ptr(), b.data_ptr())
    torch.cuda.synchronize()
    mean, _, _ = g.generate_image(p)
    _check(b.cpu().numpy().reshape(-1), _host_bytes(orc, mean), mean.size)
