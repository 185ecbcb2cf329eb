"""One process, several GPUs (rt_multi_*, include/rt_api.h): the N-way tile
partition with its single gather, driven from one host thread as the Rust
`main` would call it (main.rs:73, generate_image main.rs:85-114).

Bar: the mean image is bit-identical to rt_render's (one device, the oracle-
checked path) for any device count — the RNG is keyed by the global pixel and
sample and the chunking by the frame alone — and the work
counters summed over the devices equal the single-device frame's.  On a
one-GPU machine the N-way partition runs as N replicas on device 0 with the
peer-copy gather (RT_MULTI_PEER); the RCCL gather runs on the devices present
(one rank on a one-GPU machine, every GPU otherwise)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

STAT_KEYS = ("paths", "segments", "aabb_tests", "tri_tests", "shape_tests", "shaded_hits", "light_queries",
             "light_hits")


@pytest.fixture(scope="module")
def cornell(rt, scene_text):
    desc, params = rt.parse_scene(scene_text("cornell.txt"))
    params = params.replace(width=72, height=40, spp=6)
    img, _, st = rt.Scene(desc).generate_image(params, stats=True)
    return desc, params, img, st


@pytest.fixture(scope="module")
def atrium(rt, tmp_path_factory):
    d = tmp_path_factory.mktemp("atrium_multi")
    subprocess.run([sys.executable, os.path.join(REPO, "scenes", "gen_sponza_like.py"), str(d), "--scale", "0.05",
                    "--name", "atrium"], check=True, capture_output=True)
    desc, params = rt.load_gltf(str(d / "atrium.gltf"), 50, 34, 3)
    img, _, st = rt.Scene(desc).generate_image(params, stats=True)
    return desc, params, img, st


@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_peer_partition_matches_single(rt, cornell, n):
    desc, params, ref, ref_st = cornell
    m = rt.MultiScene(desc, [0] * n, peer=True)
    img, _, st = m.generate_image(params, stats=True)
    assert np.array_equal(img, ref)
    for k in STAT_KEYS:
        assert st[k] == ref_st[k], k
    assert st["kernel_ms"] > 0.0 and st["total_ms"] >= st["kernel_ms"]
    img2, _, _ = m.generate_image(params)  # a second frame on the same handle
    assert np.array_equal(img2, ref)
    m.close()


def test_replicas_filled_from_device0(rt, cornell, atrium):
    """devices[0] gets the scene from the host; every other replica is filled from it
    device to device (rt_multi_create: ncclBroadcast, here peer copies), ellipsoid
    reciprocals (written by devices[0]'s kernel) included: same layout, same bytes, and
    the frames above are bit-identical; the fill is timed in the replica's upload_ms."""
    for desc, params, ref, _ in (cornell, atrium):
        m = rt.MultiScene(desc, [0, 0, 0], peer=True)
        infos = [m.scene_info(i) for i in range(3)]
        for i in (1, 2):
            assert infos[i]["device_bytes"] == infos[0]["device_bytes"] > 0
            assert infos[i]["bvh_nodes"] == infos[0]["bvh_nodes"]
            assert infos[i]["upload_ms"] > 0.0
        # the content hashes rt_multi_create compared: every replica's
        # equals devices[0]'s, and a scene built from the host alone
        hs = [m.scene_checksum(i) for i in range(3)]
        assert hs[0] == hs[1] == hs[2] == rt.Scene(desc).checksum()
        img, _, _ = m.generate_image(params)
        assert np.array_equal(img, ref)
        m.close()


def test_peer_partition_triangles(rt, atrium):
    desc, params, ref, ref_st = atrium
    img, _, st = rt.MultiScene(desc, [0, 0, 0], peer=True).generate_image(params, stats=True)
    assert np.array_equal(img, ref)
    for k in STAT_KEYS:
        assert st[k] == ref_st[k], k


def test_ppm_bytes_same_for_any_n(rt, orc, cornell):
    """The fused device tonemap + bytes on the gathered tiles: identical for every
    N, and the host tonemap's bytes exactly (test_gpu_post)."""
    desc, params, ref, _ = cornell
    outs = [rt.MultiScene(desc, [0] * n, peer=True).generate_image(params, ppm_bytes=True)[1] for n in (1, 4)]
    assert np.array_equal(outs[0], outs[1])
    host = orc.ppm_bytes(orc.tonemap_gamma(ref.reshape(-1, 3))).reshape(outs[0].shape)
    assert np.array_equal(outs[0], host)


def test_rccl_gather(rt, cornell):
    """The RCCL form over every visible GPU (ncclCommInitAll + one ncclGather)."""
    desc, params, ref, ref_st = cornell
    devs = list(range(rt.device_count()))
    m = rt.MultiScene(desc, devs)
    for _ in range(2):
        img, byts, st = m.generate_image(params, ppm_bytes=True, stats=True)
        assert np.array_equal(img, ref)
        assert st["segments"] == ref_st["segments"]
    m.close()


def test_rccl_refuses_repeated_device(rt, cornell):
    desc = cornell[0]
    with pytest.raises(rt.RtError) as e:
        rt.MultiScene(desc, [0, 0])
    assert e.value.code == -1 and "RT_MULTI_PEER" in str(e.value)


def test_multi_scene_handles(rt, cornell):
    import ctypes as C
    desc = cornell[0]
    m = rt.MultiScene(desc, [0, 0], peer=True)
    L = rt.lib()
    assert L.rt_multi_scene(m._h, 0) and L.rt_multi_scene(m._h, 1)
    assert L.rt_multi_scene(m._h, 0) != L.rt_multi_scene(m._h, 1)
    assert L.rt_multi_scene(m._h, 2) is None
    info = rt.rt_scene_info()
    assert L.rt_scene_get_info(C.c_void_p(L.rt_multi_scene(m._h, 1)), C.byref(info)) == 0
    assert info.n_planes == 5
    with pytest.raises(rt.RtError):  # hit-id dumps stay rt_render's
        m.generate_image(cornell[1].replace(flags=rt.RT_FLAG_HIT_IDS))
    m.close()


def test_checksum_tells_scenes_apart(rt, cornell, atrium):
    """rt_scene_checksum is a function of the scene's device bytes: the same description
    hashes equal on every build, different scenes differ."""
    a, b = cornell[0], atrium[0]
    assert rt.Scene(a).checksum() == rt.Scene(a).checksum()
    assert rt.Scene(a).checksum() != rt.Scene(b).checksum()
