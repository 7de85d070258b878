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
