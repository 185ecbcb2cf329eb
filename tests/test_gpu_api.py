"""The tuning API's contract (rt_scene_set_tuning / rt_scene_get_tuning /
rt_scene_sample_chunks, include/rt_api.h) on the device: what get_tuning reports
can be set back, impossible forms are refused, and a forced sample run length is
held to the frame rule's limits (at most 64 runs, partial sums within 4 GiB)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cornell(rt, scene_text):
    desc, params = rt.parse_scene(scene_text("cornell.txt"))
    return desc, params, rt.Scene(desc)


def test_tuning_roundtrip_one_kind_scene(cornell, rt):
    """Cornell is shape-only: get_tuning reports kinds 1, and set_tuning accepts it back."""
    desc, params, s = cornell
    t = s.tuning()
    assert t["kinds"] == 1 and t["compact"] == 0
    s.set_tuning(**t)
    assert s.tuning() == t
    p = params.replace(width=24, height=16, spp=2)
    a, _, _ = s.generate_image(p)
    s.set_tuning()
    b, _, _ = s.generate_image(p)
    assert np.array_equal(a, b)


def test_tuning_refuses_impossible_forms(cornell, rt):
    desc, params, s = cornell
    with pytest.raises(rt.RtError) as e:
        s.set_tuning(kinds=2)  # triangle-only instance for a shape-only scene
    assert e.value.code == rt.RT_ERR_INVALID
    with pytest.raises(rt.RtError) as e:
        s.set_tuning(compact=1)  # no triangle BVH, so no compact layout
    assert e.value.code == rt.RT_ERR_UNSUPPORTED
    s.set_tuning()


def test_forced_chunk_spp_is_bounded(cornell, rt):
    """chunk_spp = 1 would ask for spp runs; the library raises the run length to keep
    <= 64 runs and the 4-GiB partial-sum budget, and reports the length it uses."""
    desc, params, s = cornell
    s.set_tuning(chunk_spp=1)
    try:
        p = params.replace(width=3840, height=2160, spp=1024)
        k, cs = s.sample_chunks(p)
        assert k <= 64 and k * cs >= 1024
        assert k * 240 * 135 * 256 * 3 * 8 <= 4 << 30
        small = params.replace(width=16, height=16, spp=8)
        assert s.sample_chunks(small) == (8, 1)  # within the limits: the forced length stands
        img, _, st = s.generate_image(small, stats=True)
        assert st["paths"] == 16 * 16 * 8 and np.isfinite(img).all()
    finally:
        s.set_tuning()


def test_tail_split_reports_the_resolved_form(cornell, rt):
    """get_tuning reports the split the last frame resolved to — 1 when the
    split cannot apply (one sample run of >= 65536 rows) — and the setting before any
    render since set_tuning."""
    desc, params, s = cornell
    try:
        s.set_tuning(tail_split=8, chunk_spp=65536)
        assert s.tuning()["tail_split"] == 8
        p = params.replace(width=16, height=16, spp=65536, ray_depth=1)
        assert s.sample_chunks(p) == (1, 65536)
        img, _, st = s.generate_image(p, stats=True)
        assert st["paths"] == 16 * 16 * 65536 and np.isfinite(img).all()
        assert s.tuning()["tail_split"] == 1
        s.set_tuning(tail_split=8)
        s.generate_image(params.replace(width=16, height=16, spp=8), stats=True)
        assert s.tuning()["tail_split"] == 8  # resolved: a small frame is all tail wave-tiles
    finally:
        s.set_tuning()
