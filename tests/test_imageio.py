import numpy as np

from another_raytracer_amd import imageio


def test_png_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)
    assert imageio.save_image(str(tmp_path / "a.png"), 23, 17, 3, img)
    back = imageio.load_image(str(tmp_path / "a.png"))
    assert np.array_equal(back, img)
    assert open(tmp_path / "a.png", "rb").read(8) == b"\x89PNG\r\n\x1a\n"


def test_raw_texel_asset_loads():
    im = imageio.load_image("assets/earthmap.rgb")
    assert im.shape == (512, 1024, 3)
