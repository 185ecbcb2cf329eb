"""GPU output surface: device tonemap + gamma + PPM
bytes, standalone and fused into the tile unpack, against the host/oracle
path (postprocessing.rs:5-37, ppm.rs:13-19).

Bar: bytes equal to the oracle's everywhere except where the device and host
`pow` round differently AND 255*v lands within that ulp of a .5 boundary; such
bytes may differ by exactly 1.  The count of those is asserted tiny (it is
zero on the sets below as measured; the bound documents the tolerance)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _host_bytes(orc, rgb):
    return orc.ppm_bytes(orc.tonemap_gamma(rgb.reshape(-1, 3))).reshape(-1)


def _check(dev, host, n):
    d = dev.astype(np.int16) - host.astype(np.int16)
    assert np.abs(d).max() <= 1
    assert (d != 0).sum() <= max(1, n // 1_000_000), f"{(d != 0).sum()} bytes differ"


def test_tonemap_bytes_random(rt, orc):
    rng = np.random.default_rng(2)
    n = 1 << 20
    x = np.concatenate([rng.uniform(-0.5, 40.0, 3 * n - 12) * rng.uniform(0, 1, 3 * n - 12) ** 3,
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
