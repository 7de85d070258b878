"""The engine surface on the GPU: output placements, pass sizing, depth limits, determinism."""
import numpy as np
import pytest
import torch

import another_raytracer_amd as art
from another_raytracer_amd.distributed import render_frame
from tests.oracle_lib import oracle_render

pytestmark = pytest.mark.gpu


def make(scene="1", W=64, H=40, spp=6, **kw):
    w = art.scene_manager().build(scene)
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, W / H, w.aperture, 10.0, 0.0, 1.0)
    e = art.engine(cam, art.engine_mode.parallel_stripes, width=W, height=H, samples_per_pixel=spp, **kw)
    e.set_scene(w.objects, w.background)
    return e


def test_device_output_equals_host_output(gpu):
    e = make()
    host = np.zeros((40, 64, 3), np.uint8)
    e.run(host)
    dev = torch.zeros((40, 64, 3), dtype=torch.uint8, device="cuda")
    e.run(dev)
    assert np.array_equal(dev.cpu().numpy(), host)
    frame, stats = render_frame(e, band_rows=16)
    assert np.array_equal(frame.cpu().numpy(), host) and stats["segments"] > 0


def test_samples_per_pass_does_not_change_the_image(gpu):
    ref = None
    for spp_pass in (1, 2, 5, 0):
        e = make(samples_per_pass=spp_pass)
        img = np.zeros((40, 64, 3), np.uint8)
        acc = np.zeros((40, 64, 3), np.float64)
        e.run(img, accum=acc)
        if ref is None:
            ref = (img, acc, e.stats["segments"])
        assert np.array_equal(acc, ref[1]) and np.array_equal(img, ref[0]) and e.stats["segments"] == ref[2]


@pytest.mark.parametrize("depth", [0, 1, 3])
def test_depth_limit_matches_oracle(gpu, depth):
    e = make("8", W=32, H=20, spp=4, max_depth=depth)
    img = np.zeros((20, 32, 3), np.uint8)
    acc = np.zeros((20, 32, 3), np.float64)
    e.run(img, accum=acc)
    o = oracle_render("8", 32, 20, 4, mode="pcg", max_depth=depth)
    assert e.stats["segments"] == o["segments"]
    assert np.array_equal(img, o["rgb"])


def test_background_override_and_seed(gpu):
    e = make("c1", spp=2)
    a = np.zeros((40, 64, 3), np.uint8)
    e.run(a)
    e.set_scene(e.world, (0.0, 0.0, 0.0))
    b = np.zeros_like(a)
    e.run(b)
    assert b.sum() < a.sum() // 4  # the sky is the only light of this scene
    e2 = make("c1", spp=2, seed=7)
    c = np.zeros_like(a)
    e2.run(c)
    assert not np.array_equal(c, a)


def test_python_built_scene_renders_like_the_builtin(gpu):
    from tests.test_scene import _python_random_scene
    world = _python_random_scene()
    w = art.scene_manager().build("1")
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, 1.6, w.aperture, 10.0, 0.0, 1.0)
    imgs = []
    for objs in (world, w.objects):
        e = art.engine(cam, width=48, height=30, samples_per_pixel=3)
        e.set_scene(objs, w.background)
        img = np.zeros((30, 48, 3), np.uint8)
        e.run(img)
        imgs.append(img)
    art.reset_scene_rng()
    assert np.array_equal(imgs[0], imgs[1])


def test_adaptive_mode_refuses_accum_and_off_grid_sizes(gpu):
    e = make(W=48, H=36)
    e.m = art.engine_mode.adaptive
    with pytest.raises(ValueError):
        e.run(np.zeros((36, 48, 3), np.uint8), accum=np.zeros((36, 48, 3), np.float64))
    e = make(W=64, H=40)
    e.m = art.engine_mode.adaptive
    with pytest.raises(ValueError, match="big square"):
        e.run(np.zeros((40, 64, 3), np.uint8))


def test_workspace_allocation_failure_leaves_the_scene_usable(gpu, options):
    # a refused workspace allocation (fault point: option test.fault_workspace_bytes) is reported as RT_E_DEVICE, and
    # the next render on the same scene allocates again instead of using a stale size with a null base
    e = make()
    first = np.zeros((40, 64, 3), np.uint8)
    e.run(first)
    big = make(W=256, H=160)
    big._scene = e._scene  # same rt_scene (and renderer workspace), larger frame: the workspace must grow
    options("test.fault_workspace_bytes", 1024)
    with pytest.raises(art.RTError) as err:
        big.run(np.zeros((160, 256, 3), np.uint8))
    assert err.value.code == -3 and "test.fault_workspace_bytes" in str(err.value)
    options("test.fault_workspace_bytes", 0)
    again = np.zeros((40, 64, 3), np.uint8)
    e.run(again)
    assert np.array_equal(again, first)
    grown = np.zeros((160, 256, 3), np.uint8)
    big.run(grown)
    fresh = np.zeros((160, 256, 3), np.uint8)
    make(W=256, H=160).run(fresh)
    assert np.array_equal(grown, fresh)


def test_oversized_samples_per_pass_is_clamped(gpu):
    # samples_per_pass * padded pixels beyond 2^31 slots used to wrap the u32 pass size: it is clamped to the largest
    # pass that fits (1035 samples of a 1920x1080 frame), and the image equals the automatic pass split's
    W, H, spp = 1920, 1080, 2100
    e = make(W=W, H=H, spp=spp, samples_per_pass=2100)
    acc = np.zeros((H, W, 3), np.float64)
    e.run(np.zeros((H, W, 3), np.uint8), accum=acc)
    assert e.stats["samples_per_pass"] * 240 * 135 * 64 <= 2 ** 31 and e.stats["passes"] == 3
    auto = make(W=W, H=H, spp=spp)
    acc2 = np.zeros((H, W, 3), np.float64)
    auto.run(np.zeros((H, W, 3), np.uint8), accum=acc2)
    assert np.array_equal(acc, acc2) and e.stats["segments"] == auto.stats["segments"]


@pytest.mark.parametrize("band_rows", [1, 7, 16])
def test_render_multi_one_gpu_matches_render(gpu, band_rows):
    # rt_render_multi through its RCCL path (ncclCommInitAll, ncclGather to devices[0], unpack kernel) with one GPU
    # reproduces rt_render bit for bit, into host and device memory
    from another_raytracer_amd.distributed import multi_engine
    W, H, spp = 160, 90, 8
    w = art.scene_manager().build("1")
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, W / H, w.aperture, 10.0, 0.0, 1.0)
    e = art.engine(cam, art.engine_mode.single, width=W, height=H, samples_per_pixel=spp)
    e.set_scene(w.objects, w.background)
    ref = np.zeros((H, W, 3), np.uint8)
    e.run(ref)
    m = multi_engine("1", [0], cam, W, H, spp, band_rows=band_rows, background=w.background)
    host = np.zeros((H, W, 3), np.uint8)
    m.run(host)
    assert np.array_equal(host, ref) and m.stats["segments"] == e.stats["segments"] and m.stats["local_rows"] == H
    dev = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda:0")
    m.run(dev)
    assert np.array_equal(dev.cpu().numpy(), ref)


def test_render_multi_rejects_duplicate_devices(gpu):
    from another_raytracer_amd.distributed import multi_engine
    w = art.scene_manager().build("c1")
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, 2.0, w.aperture, 10.0, 0.0, 1.0)
    with pytest.raises(art.RTError, match="only once"):
        multi_engine("c1", [0, 0], cam, 32, 16, 1)


def test_progressive_snapshots_equal_one_shot_renders(gpu):
    # rt_render_progressive: after each pass the snapshot equals a one-shot render of that many samples bit for bit
    # (samples are keyed by (pixel, sample index) and summed in order), and the last one the whole frame
    W, H, spp = 96, 54, 8
    e = make(W=W, H=H, spp=spp)
    img = np.zeros((H, W, 3), np.uint8)
    acc = np.zeros((H, W, 3), np.float64)
    snaps = []
    e.run_progressive(img, lambda done, total: snaps.append((done, img.copy(), acc.copy())), accum=acc, samples_per_pass=3)
    assert [s[0] for s in snaps] == [3, 6, 8]
    for done, rgb, sums in snaps:
        one = make(W=W, H=H, spp=done)
        r1 = np.zeros((H, W, 3), np.uint8)
        a1 = np.zeros((H, W, 3), np.float64)
        one.run(r1, accum=a1)
        assert np.array_equal(rgb, r1) and np.array_equal(sums, a1)
    assert e.stats["primary"] == W * H * spp


def test_progressive_callback_can_stop_early(gpu):
    W, H, spp = 64, 40, 9
    e = make(W=W, H=H, spp=spp)
    img = np.zeros((H, W, 3), np.uint8)
    seen = []
    e.run_progressive(img, lambda done, total: seen.append(done) or done >= 4, samples_per_pass=2)
    assert seen == [2, 4] and e.stats["primary"] == W * H * 4
    four = make(W=W, H=H, spp=4)
    r4 = np.zeros((H, W, 3), np.uint8)
    four.run(r4)
    assert np.array_equal(img, r4)


@pytest.mark.parametrize("name", ["1", "9", "8"])
def test_loaded_scene_renders_bit_identically(gpu, name, tmp_path):
    # rt_scene_save -> rt_scene_load (no OBJ parse, no image decode, no BVH build): the same frame, bit for bit
    W, H, spp = 64, 40, 4
    built = art.scene_manager().build(name)
    art.save_scene(built, tmp_path / "s.artscene")
    frames = []
    for w in (built, art.scene_manager().load(tmp_path / "s.artscene")):
        cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, W / H, w.aperture, 10.0, 0.0, 1.0)
        e = art.engine(cam, art.engine_mode.single, width=W, height=H, samples_per_pixel=spp)
        e.set_scene(w.objects, w.background)
        img = np.zeros((H, W, 3), np.uint8)
        acc = np.zeros((H, W, 3), np.float64)
        e.run(img, accum=acc)
        frames.append((img, acc, e.stats["segments"]))
    assert np.array_equal(frames[0][0], frames[1][0]) and np.array_equal(frames[0][1], frames[1][1]) and frames[0][2] == frames[1][2]


def _multi(scene="1", W=64, H=40, spp=4, band_rows=8):
    from another_raytracer_amd.distributed import multi_engine
    w = art.scene_manager().build(scene)
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, W / H, w.aperture, 10.0, 0.0, 1.0)
    return multi_engine(scene, [0], cam, W, H, spp, band_rows=band_rows, background=w.background)


def test_render_multi_phase_times(gpu):
    # rt_multi_times: the renders, the gather and the unpack of the last call, each timed, and the collectives counted
    m = _multi()
    img = torch.zeros((40, 64, 3), dtype=torch.uint8, device="cuda:0")
    m.run(img)
    t = m.times()
    assert t["ngpus"] == 1 and t["collectives"] == 1 and t["slowest_device"] == 0
    assert 0 < t["render_ms_min"] <= t["render_ms_max"] <= t["total_ms"]
    assert t["gather_ms"] >= 0 and t["unpack_ms"] > 0 and t["wait_ms"] >= 0
    assert t["render_ms_max"] + t["gather_ms"] + t["unpack_ms"] <= t["total_ms"] * 1.05 + 0.5
    assert abs(t["total_ms"] - m.stats["ms"]) < 1e-9
    m.run(img)
    assert m.times()["collectives"] == 2


@pytest.mark.parametrize("timeout_ms", [float("inf"), 1e300])
def test_render_multi_without_deadline(gpu, options, timeout_ms):
    # multi.timeout_ms = inf (or beyond the clock's range) is no deadline: creation and the gather complete instead of
    # aborting at a deadline in the past (r5's duration_cast of inf gave INT64_MIN)
    art.set_option("multi.timeout_ms", timeout_ms)
    m = _multi()
    img = torch.zeros((40, 64, 3), dtype=torch.uint8, device="cuda:0")
    m.run(img)
    assert m.times()["collectives"] == 1 and int(img.sum()) > 0


def test_render_multi_failed_render_starts_no_collective(gpu, options):
    # a device whose render fails (fault injection: its workspace growth is refused) ends rt_render_multi with RT_E_DEVICE
    # before the gather -- no collective starts -- and the multi renders correctly afterwards
    m = _multi()
    first = np.zeros((40, 64, 3), np.uint8)
    m.run(first)
    assert m.times()["collectives"] == 1
    m.width, m.height = 256, 160  # a larger frame: the renderer's workspace must grow
    options("test.fault_workspace_bytes", 1024)
    with pytest.raises(art.RTError) as err:
        m.run(np.zeros((160, 256, 3), np.uint8))
    assert err.value.code == -3 and "test.fault_workspace_bytes" in str(err.value)
    assert m.times()["collectives"] == 1
    options("test.fault_workspace_bytes", 0)
    m.width, m.height = 64, 40
    again = np.zeros((40, 64, 3), np.uint8)
    m.run(again)
    assert np.array_equal(again, first) and m.times()["collectives"] == 2


def test_render_multi_gather_failure_aborts_and_is_reported(gpu, options):
    # a collective that fails in flight (fault point after ncclGroupEnd, as a peer error or an expired multi.timeout_ms
    # deadline would) aborts the communicators and returns RT_E_DEVICE; that rt_multi then refuses to render, and a new
    # one works
    m = _multi()
    ref = np.zeros((40, 64, 3), np.uint8)
    m.run(ref)
    options("test.fault_gather_abort", 1)
    with pytest.raises(art.RTError) as err:
        m.run(np.zeros((40, 64, 3), np.uint8))
    assert err.value.code == -3 and "injected" in str(err.value)
    options("test.fault_gather_abort", 0)
    with pytest.raises(art.RTError, match="unusable"):
        m.run(np.zeros((40, 64, 3), np.uint8))
    del m
    fresh = np.zeros((40, 64, 3), np.uint8)
    _multi().run(fresh)
    assert np.array_equal(fresh, ref)


@pytest.mark.parametrize("where", [1, 2])
def test_failure_inside_an_rccl_group_leaves_the_thread_usable(gpu, options, where):
    # an error between ncclGroupStart and ncclGroupEnd (fault point test.fault_rccl_group: 1 = inside
    # rt_multi_create's communicator-init group, 2 = inside rt_render_multi's gather group) must close the group and
    # abort the communicators before it is reported, or the calling thread stays inside the group and its next
    # collectives are absorbed into it.  After the failure a new rt_multi on this same thread creates, renders and
    # matches rt_render.
    ref = np.zeros((40, 64, 3), np.uint8)
    make(spp=4).run(ref)
    options("test.fault_rccl_group", where)
    with pytest.raises(art.RTError) as err:
        m = _multi()
        m.run(np.zeros((40, 64, 3), np.uint8))
    assert err.value.code == -3 and "injected" in str(err.value) and "aborted" in str(err.value)
    if where == 2:  # the multi whose gather failed refuses further renders
        with pytest.raises(art.RTError, match="unusable"):
            m.run(np.zeros((40, 64, 3), np.uint8))
        del m
    options("test.fault_rccl_group", 0)
    for _ in range(2):  # a second create + render on the same thread: no stale group state
        fresh = np.zeros((40, 64, 3), np.uint8)
        m2 = _multi()
        m2.run(fresh)
        assert np.array_equal(fresh, ref) and m2.times()["collectives"] == 1
        del m2


def test_multi_create_uploads_the_scene(gpu):
    # rt_multi_create uploads the scene to every device before it returns (a timed first render of a fresh
    # multi_engine must not include the upload; the reference times engine::run only, main.cpp:44-46)
    m = _multi("8")
    info = m.scene_info()
    assert info["device_bytes_f64"] > 0  # before any render
    m.run(np.zeros((40, 64, 3), np.uint8))
    assert m.scene_info()["device_bytes_f64"] == info["device_bytes_f64"]
