"""libart's JPEG / PNG decoder (csrc/imagedec.cpp, rt_image_load) vs the reference's own stb_image v2.27 decodes.

* the two texture files of the reference scenes (textures/earthmap.jpg: baseline 4:4:4; models/capsule/capsule.jpg:
  progressive 4:4:4 with an Adobe marker) against the texels `ref_harness texture` wrote from them (assets/*.rgb*);
* tests/golden/images.npz: every variant the decoder handles (4:2:0 / 4:2:2 chroma upsampling, progressive scans,
  restart intervals, grayscale, CMYK, quality 3 and 100, PNG bit depths, palettes, tRNS) with stb's bytes.
Bit-exact in every case.  CPU only (the decoder is host code of the scene build).
"""
import gzip
import os

import numpy as np
import pytest

from another_raytracer_amd.imageio import load_image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = np.load(os.path.join(ROOT, "tests", "golden", "images.npz"))
NAMES = sorted({k.split("__")[0] for k in FIX.files})


def raw_asset(path):
    blob = gzip.open(path).read() if path.endswith(".gz") else open(path, "rb").read()
    w, h, c = np.frombuffer(blob[:12], np.int32)
    return np.frombuffer(blob[12:], np.uint8).reshape(h, w, c)


@pytest.mark.parametrize("jpg,asset", [("assets/earthmap.jpg", "assets/earthmap.rgb"),
                                       ("assets/models/capsule/capsule.jpg", "assets/models/capsule/capsule.rgb.gz")])
def test_scene_textures_decode_like_stb(jpg, asset):
    a = load_image(os.path.join(ROOT, jpg))
    assert np.array_equal(a, raw_asset(os.path.join(ROOT, asset)))


@pytest.mark.parametrize("name", NAMES)
def test_image_variants_decode_like_stb(name, tmp_path):
    ext = ".jpg" if name.startswith("jpg") else ".png"
    path = tmp_path / (name + ext)
    path.write_bytes(FIX[f"{name}__file"].tobytes())
    w, h, c = FIX[f"{name}__whc"]
    a = load_image(path)
    assert a.shape == (h, w, c)
    assert np.array_equal(a.reshape(-1), FIX[f"{name}__decoded"])


def test_corrupt_files_fail_loudly(tmp_path):
    from another_raytracer_amd._lib import RTError
    good = FIX["jpg_420__file"].tobytes()
    for i, blob in enumerate([b"", b"\xff\xd8\xff", good[:len(good) // 3], b"\x89PNG\r\n\x1a\n" + b"\x00" * 20, b"GIF89a"]):
        p = tmp_path / f"bad{i}.jpg"
        p.write_bytes(blob)
        with pytest.raises(RTError):
            load_image(p)
