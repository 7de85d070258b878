"""HIP path (through the C ABI) vs the oracle — the parity gate (SURVEY.md §8(d) tolerances).

* The f64 path (the only arithmetic, ABI 2) vs oracle/restate.cpp ORC_PCG (same PCG streams, same f64 operation
  order): every scene, bit-identical RGB8 frame, bit-identical f64 per-pixel radiance sums and the exact segment count.
* Independence from the partition: band-interleaved renders reassemble to the bit-identical image.
* Statistical parity with the reference program itself (independent RNG, SURVEY.md §8(d) tolerance 3), f64 path:
  - configs[0] (tests/golden/render_c1_400x225x64.npz): RMSE <= 1.1x the oracle's seed-to-seed noise floor;
  - the headline scene (alias 1) at 384x216x16, the cow mesh scene at 384x216x16 and the Next-Week final at
    384x216x32 (tests/golden/render_stat_*.npz: the reference's single and 4-thread stripes renders): RMSE vs the
    single render <= 1.1x the single-vs-stripes RMSE, the same on 8x8 block means (x1.25: noise / 8, so a bias of
    ~1 LSB shows), the per-channel mean within 0.5 LSB, and segments per primary within 1 %.
"""
import os

import numpy as np
import pytest

import another_raytracer_amd as art
from tests.oracle_lib import oracle_render

pytestmark = pytest.mark.gpu

SCENES = ["c1", "1", "2", "3", "4", "5", "6", "7", "8", "cow", "dino", "9"]


def gpu_render(scene, W, H, spp, precision="f64", seed=0, band=None, accum=True, global_scene=False, split_shade=False,
               wavefront=False, max_depth=50, samples_per_pass=0):
    world = art.scene_manager().build(scene)
    cam = art.camera(world.lookfrom, world.lookat, (0, 1, 0), world.vfov, W / H, world.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.single, width=W, height=H, samples_per_pixel=spp, precision=precision,
                     seed=seed, max_depth=max_depth, samples_per_pass=samples_per_pass)
    eng.set_scene(world.objects, world.background)
    eng.global_scene = global_scene
    eng.split_shade = split_shade
    eng.wavefront = wavefront
    band_rows, band_count, band_index = band or (None, 1, 0)
    rows = H if band is None else len(eng.local_rows(band_rows, band_count, band_index))
    img = np.zeros((rows, W, 3), np.uint8)
    acc = np.zeros((rows, W, 3), np.float64) if accum else None
    eng.run(img, accum=acc, band_rows=band_rows, band_count=band_count, band_index=band_index)
    return {"rgb": img, "acc": acc, "segments": eng.stats["segments"], "stats": eng.stats, "engine": eng}


def lsb_stats(a, b):
    d = np.abs(a.astype(np.int64) - b.astype(np.int64))
    rmse = float(np.sqrt(np.mean(d.astype(np.float64) ** 2)))
    within1 = float(np.mean(d.max(axis=-1) <= 1))
    return rmse, within1, int(d.max())


@pytest.mark.parametrize("scene", SCENES)
def test_f64_matches_oracle_pcg(gpu, scene):
    W, H, spp = 64, 36, 8
    g = gpu_render(scene, W, H, spp, "f64")
    o = oracle_render(scene, W, H, spp, mode="pcg")
    rmse, within1, dmax = lsb_stats(g["rgb"], o["rgb"])
    print(f"{scene}: rmse {rmse:.4f} within1 {within1:.5f} max {dmax} segs {g['segments']} vs {o['segments']}")
    assert np.array_equal(g["rgb"], o["rgb"]), (rmse, within1, dmax)
    assert np.array_equal(g["acc"], o["acc"])
    assert g["segments"] == o["segments"]


F_CODE16 = 1 << 7  # layout.h feature bit of the 16-bit-child-code instantiations


def test_scene_kernel_map(gpu):
    # the persistent kernel every builtin scene runs (rt_stats.kernel_*) is the one tests/test_kernel_resources.py
    # checks for spills
    from tests.test_kernel_resources import SCENE_KERNELS
    for scene, key in SCENE_KERNELS.items():
        st = gpu_render(scene, 32, 18, 1)["stats"]
        got = (st["kernel_features"], st["kernel_textures"], st["kernel_lds_mode"])
        assert got == key, (scene, got, key)
        assert st["extend_variant"] == (3 if key[2] == 3 else 4), (scene, st)


@pytest.mark.parametrize("scene", ["cow", "dino", "8", "5"])
def test_32bit_code_kernels_match_oracle_pcg(gpu, options, scene):
    # a scene whose BVH codes do not fit 16 bits (> 32768 nodes or > 8192 primitive references) takes the k_paths_g
    # instantiations without F_CODE16 (float keys, 32-bit stack entries); option render.codes16 = 0 forces that path on
    # scenes that fit, so its traversal is pinned for triangle scenes (cow: LM 2, dino: LM 1) and triangle-free ones
    # (final, Cornell).  rt_stats names the kernel that ran (the test must see the 32-bit-code kernel run).
    W, H, spp = 48, 27, 4
    default = gpu_render(scene, W, H, spp)["stats"]
    options("render.codes16", 0)
    g = gpu_render(scene, W, H, spp)
    o = oracle_render(scene, W, H, spp, mode="pcg")
    assert g["stats"]["extend_variant"] == 4
    assert g["stats"]["kernel_features"] & F_CODE16 == 0, g["stats"]
    assert default["kernel_features"] & F_CODE16, default
    assert np.array_equal(g["rgb"], o["rgb"]) and np.array_equal(g["acc"], o["acc"]) and g["segments"] == o["segments"]


def test_band_partition_is_bit_identical(gpu):
    W, H, spp = 80, 50, 4
    full = gpu_render("1", W, H, spp)
    for bands, brows in ((2, 16), (3, 8), (8, 4)):
        img = np.zeros_like(full["rgb"])
        acc = np.zeros_like(full["acc"])
        segs = 0
        for b in range(bands):
            part = gpu_render("1", W, H, spp, band=(brows, bands, b))
            rows = part["engine"].local_rows(brows, bands, b)
            img[rows] = part["rgb"]
            acc[rows] = part["acc"]
            segs += part["segments"]
        assert np.array_equal(img, full["rgb"])
        assert np.array_equal(acc, full["acc"])
        assert segs == full["segments"]


@pytest.mark.parametrize("max_depth", [1, 3, 50])
def test_extend_variants_are_bit_identical(gpu, max_depth):
    # the benchmark scene runs the persistent-path kernel (variant 3); it must reproduce the per-depth fused LDS kernel
    # (2), the split-shade LDS kernel (1), the persistent HBM-scene kernel (4) and the per-depth HBM kernels (0) bit
    # for bit, including the last-bounce cut-off
    W, H, spp = 160, 90, 8
    mega = gpu_render("1", W, H, spp, "f64", max_depth=max_depth)
    fused = gpu_render("1", W, H, spp, "f64", wavefront=True, max_depth=max_depth)
    split = gpu_render("1", W, H, spp, "f64", split_shade=True, max_depth=max_depth)
    glb = gpu_render("1", W, H, spp, "f64", global_scene=True, max_depth=max_depth)
    glb_wf = gpu_render("1", W, H, spp, "f64", global_scene=True, wavefront=True, max_depth=max_depth)
    assert tuple(r["stats"]["extend_variant"] for r in (mega, fused, split, glb, glb_wf)) == (3, 2, 1, 4, 0)
    for other in (fused, split, glb, glb_wf):
        assert np.array_equal(mega["acc"], other["acc"])
        assert np.array_equal(mega["rgb"], other["rgb"])
        assert mega["segments"] == other["segments"]


def test_persistent_paths_pass_split_is_bit_identical(gpu):
    # several passes (samples_per_pass) and one pass, with partial 8x8 tiles (padding slots): identical sums
    W, H, spp = 100, 52, 12
    one = gpu_render("1", W, H, spp, "f64")
    many = gpu_render("1", W, H, spp, "f64", samples_per_pass=5)
    assert one["stats"]["extend_variant"] == 3 and many["stats"]["passes"] == 3
    assert np.array_equal(one["acc"], many["acc"]) and one["segments"] == many["segments"]


@pytest.mark.parametrize("W,H,spp", [(2, 2, 1), (9, 3, 3), (13, 70, 2), (130, 2, 5)])
def test_persistent_paths_small_and_ragged_frames(gpu, W, H, spp):
    # k_paths takes its camera rays from a per-wave ring filled 64 slots at a time: a pass shorter than one batch
    # (2x2x1: 64 slots, 60 of them padding), batches made mostly of padding slots of partial 8x8 tiles, and passes
    # that end inside a batch must all trace exactly the oracle's paths
    g = gpu_render("1", W, H, spp)
    o = oracle_render("1", W, H, spp, mode="pcg")
    assert g["stats"]["extend_variant"] == 3
    assert np.array_equal(g["rgb"], o["rgb"])
    assert np.array_equal(g["acc"], o["acc"])
    assert g["segments"] == o["segments"]


@pytest.mark.parametrize("scene", ["7", "3"])
def test_lds_ring_kernels_small_ragged_split_and_banded(gpu, scene):
    # the triangle-free LM 1 kernels take their camera rays from a per-wave LDS ring filled 64 slots at a time
    # (kernels.hip ring_fill_g / ring_take_g): passes shorter than one batch, batches of padding slots of partial 8x8
    # tiles, passes that end inside a batch, several passes, and band partitions must all trace exactly the oracle's
    # paths
    from tests.test_kernel_resources import SCENE_KERNELS
    for W, H, spp in ((2, 2, 1), (9, 3, 3), (13, 70, 2), (130, 2, 5)):
        g = gpu_render(scene, W, H, spp)
        o = oracle_render(scene, W, H, spp, mode="pcg")
        st = g["stats"]
        assert (st["kernel_features"], st["kernel_textures"], st["kernel_lds_mode"]) == SCENE_KERNELS[scene]
        assert np.array_equal(g["rgb"], o["rgb"]) and np.array_equal(g["acc"], o["acc"]) and g["segments"] == o["segments"], (W, H, spp)
    W, H, spp = 100, 52, 12
    one = gpu_render(scene, W, H, spp)
    many = gpu_render(scene, W, H, spp, samples_per_pass=5)
    assert many["stats"]["passes"] == 3
    assert np.array_equal(one["acc"], many["acc"]) and one["segments"] == many["segments"]
    img = np.zeros_like(one["rgb"])
    segs = 0
    for b in range(3):
        part = gpu_render(scene, W, H, spp, band=(8, 3, b))
        img[part["engine"].local_rows(8, 3, b)] = part["rgb"]
        segs += part["segments"]
    assert np.array_equal(img, one["rgb"]) and segs == one["segments"]


def test_general_scenes_use_the_hbm_kernels(gpu):
    # triangles/rects/media (or no BVH) never take the LDS variants: persistent paths over the HBM scene (4), or the
    # per-depth HBM kernels (0) with RT_WAVEFRONT
    assert gpu_render("cow", 32, 18, 2)["stats"]["extend_variant"] == 4
    assert gpu_render("cow", 32, 18, 2, wavefront=True)["stats"]["extend_variant"] == 0


@pytest.mark.parametrize("scene", ["cow", "8", "5", "6", "7", "9", "4"])
@pytest.mark.parametrize("max_depth", [1, 50])
def test_hbm_persistent_paths_match_wavefront(gpu, scene, max_depth):
    # every feature (triangles, rects, boxes, transforms, media, noise/image textures, lights) through k_paths_g is bit
    # for bit the per-depth wavefront render
    W, H, spp = 48, 27, 4
    a = gpu_render(scene, W, H, spp, "f64", max_depth=max_depth)
    b = gpu_render(scene, W, H, spp, "f64", wavefront=True, max_depth=max_depth)
    assert a["stats"]["extend_variant"] == 4 and b["stats"]["extend_variant"] == 0
    assert np.array_equal(a["acc"], b["acc"]) and np.array_equal(a["rgb"], b["rgb"])
    assert a["segments"] == b["segments"]


def test_statistical_parity_with_reference_config0(gpu):
    ref = np.load("tests/golden/render_c1_400x225x64.npz")
    W, H, spp = int(ref["W"]), int(ref["H"]), int(ref["spp"])
    floor = np.mean([lsb_stats(oracle_render("c1", W, H, spp, mode="pcg", seed=s)["rgb"], ref["rgb"])[0] for s in (11, 12)])
    gpu_rmse = np.mean([lsb_stats(gpu_render("c1", W, H, spp, "f64", seed=s, accum=False)["rgb"], ref["rgb"])[0]
                        for s in (21, 22)])
    print(f"rmse vs reference: gpu {gpu_rmse:.3f} oracle floor {floor:.3f}")
    assert gpu_rmse <= 1.1 * floor


def _block_means(x, k=8):
    H, W, _ = x.shape
    return x[:H // k * k, :W // k * k].astype(np.float64).reshape(H // k, k, W // k, k, 3).mean(axis=(1, 3))


def _rmse(a, b):
    return float(np.sqrt(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)))


STAT = {"1": "render_stat_1_384x216x16.npz", "cow": "render_stat_cow_384x216x16.npz", "8": "render_stat_8_384x216x32.npz",
        "dino": "render_stat_dino_384x216x16.npz"}


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("scene", list(STAT))
def test_statistical_parity_headline_scene_f64(gpu, scene, seed):
    """The f64 GPU path vs the reference program's own render (independent RNG) of the headline scene, the cow mesh
    (triangle.h:22-88 under the mist medium, constant_medium.h:37-82) and the Next-Week final (boxes, instances, two
    media, textures)."""
    ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", STAT[scene]))
    W, H, spp = int(ref["W"]), int(ref["H"]), int(ref["spp"])
    single, stripes = ref["rgb_single"], ref["rgb_stripes"]
    floor, bfloor = _rmse(single, stripes), _rmse(_block_means(single), _block_means(stripes))
    g = gpu_render(scene, W, H, spp, "f64", seed=seed, accum=False)
    rmse, brmse = _rmse(g["rgb"], single), _rmse(_block_means(g["rgb"]), _block_means(single))
    bias = (g["rgb"].astype(np.float64) - single).mean(axis=(0, 1))
    print(f"scene {scene} seed {seed}: rmse {rmse:.3f} (floor {floor:.3f}) block rmse {brmse:.3f} (floor {bfloor:.3f}) bias {bias}")
    assert rmse <= 1.1 * floor
    assert brmse <= 1.25 * bfloor
    assert np.all(np.abs(bias) <= 0.5)
    # same light transport: segments per primary within 1 % of the reference's
    r_ref = int(ref["segments_single"]) / (W * H * spp)
    assert abs(g["segments"] / (W * H * spp) - r_ref) / r_ref < 0.01


def test_segments_match_reference_rate(gpu):
    # segments per primary ray of the reference (golden, mt) vs the HIP path: same light transport
    ref = np.load("tests/golden/render_c1_400x225x64.npz")
    g = gpu_render("c1", 400, 225, 64, "f64", accum=False)
    r_ref = int(ref["segments"]) / (400 * 225 * 64)
    r_gpu = g["segments"] / (400 * 225 * 64)
    assert abs(r_gpu - r_ref) / r_ref < 0.01, (r_gpu, r_ref)


def gpu_render_adaptive(scene, W, H, spp, band=None, seed=0, **kw):
    world = art.scene_manager().build(scene)
    cam = art.camera(world.lookfrom, world.lookat, (0, 1, 0), world.vfov, W / H, world.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.adaptive, width=W, height=H, samples_per_pixel=spp, seed=seed, **kw)
    eng.set_scene(world.objects, world.background)
    band_rows, band_count, band_index = band or (None, 1, 0)
    rows = H if band is None else len(eng.local_rows(band_rows, band_count, band_index))
    img = np.zeros((rows, W, 3), np.uint8)
    eng.run(img, band_rows=band_rows, band_count=band_count, band_index=band_index)
    return img, eng


@pytest.mark.parametrize("scene", ["c1", "1", "8", "cow", "7", "3", "9"])
def test_adaptive_matches_oracle_pcg(gpu, scene):
    """engine_mode::adaptive (engine.h:96-333) on the GPU vs the oracle's restatement on the same streams: bit-exact
    frame and the exact segment count (every distinct pixel traced once)."""
    from tests.oracle_lib import oracle_render_adaptive
    W, H, spp = 96, 48, 8
    img, eng = gpu_render_adaptive(scene, W, H, spp)
    o = oracle_render_adaptive(scene, W, H, spp, mode="pcg")
    rmse, within1, dmax = lsb_stats(img, o["rgb"])
    print(f"adaptive {scene}: rmse {rmse:.4f} max {dmax} segs {eng.stats['segments']} vs {o['segments']}")
    assert np.array_equal(img, o["rgb"])
    assert eng.stats["segments"] == o["segments"]


def test_adaptive_launch_forms_agree(gpu):
    """The capsule (the reference's default run) in adaptive mode two ways -- device-counted levels (one pass per level,
    entry-major slots, no host round trip) and host-counted levels (samples_per_pass < spp: sample-major slots, the
    list sizes read back between levels) -- gives one frame and one segment count."""
    W, H, spp = 120, 96, 6
    lv, e1 = gpu_render_adaptive("9", W, H, spp)
    mp, e2 = gpu_render_adaptive("9", W, H, spp, samples_per_pass=2)
    assert e1.stats["passes"] == 4 and e2.stats["passes"] >= 4
    assert np.array_equal(lv, mp)
    assert e1.stats["segments"] == e2.stats["segments"]
    assert e1.stats["primary"] == e2.stats["primary"]


def test_adaptive_band_partition_is_bit_identical(gpu):
    W, H, spp = 120, 72, 4
    full, e = gpu_render_adaptive("1", W, H, spp)
    img = np.zeros_like(full)
    segs = 0
    for b in range(2):
        part, eng = gpu_render_adaptive("1", W, H, spp, band=(12, 2, b))
        img[eng.local_rows(12, 2, b)] = part
        segs += eng.stats["segments"]
    assert np.array_equal(img, full)
    assert segs == e.stats["segments"]


@pytest.mark.parametrize("scene,spp,per_pass", [("1", 10, 3), ("cow", 9, 0), ("4", 6, 5), ("8", 8, 2)])
def test_parallel_images_matches_oracle_pcg(gpu, scene, spp, per_pass):
    """engine_mode::parallel_images (engine.h:378-445): four float partial images of spp/4 samples, summed and written
    with the full spp.  RGB8, the f64 sums and the segment count equal the oracle's, with passes that split the
    quarters (samples_per_pass 3 of m = 2, 5 of m = 1, 2 of m = 2)."""
    from tests.oracle_lib import oracle_render_images
    W, H = 64, 36
    world = art.scene_manager().build(scene)
    cam = art.camera(world.lookfrom, world.lookat, (0, 1, 0), world.vfov, W / H, world.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.parallel_images, width=W, height=H, samples_per_pixel=spp, samples_per_pass=per_pass)
    eng.set_scene(world.objects, world.background)
    img = np.zeros((H, W, 3), np.uint8)
    acc = np.zeros((H, W, 3), np.float64)
    eng.run(img, accum=acc)
    o = oracle_render_images(scene, W, H, spp, mode="pcg")
    assert np.array_equal(img, o["rgb"])
    assert np.array_equal(acc, o["acc"])
    assert eng.stats["segments"] == o["segments"]
    assert eng.stats["primary"] == W * H * 4 * (spp // 4)


def test_parallel_images_below_four_spp_is_black(gpu):
    """spp < 4: the reference's four partial images get spp/4 = 0 samples each, so every pixel is write_color(0, spp)."""
    world = art.scene_manager().build("1")
    cam = art.camera(world.lookfrom, world.lookat, (0, 1, 0), world.vfov, 2.0, world.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.parallel_images, width=32, height=16, samples_per_pixel=3)
    eng.set_scene(world.objects, world.background)
    img = np.full((16, 32, 3), 7, np.uint8)
    eng.run(img)
    assert not img.any() and eng.stats["segments"] == 0
