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


def _png(chunks):
    import struct
    import zlib
    out = b"\x89PNG\r\n\x1a\n"
    for typ, data in chunks:
        out += struct.pack(">I", len(data)) + typ + data + struct.pack(">I", zlib.crc32(typ + data) & 0xFFFFFFFF)
    return out


def _rgb_png_chunks(ctype=2, extra=()):
    import struct
    import zlib
    chans = {0: 1, 2: 3}[ctype]
    raw = b"".join(b"\x00" + bytes(range(2 * chans)) for _ in range(2))  # 2x2, filter 0
    return [(b"IHDR", struct.pack(">IIBBBBB", 2, 2, 8, ctype, 0, 0, 0)), *extra, (b"IDAT", zlib.compress(raw))]


def test_truncated_and_malformed_png_chunks_are_refused(tmp_path):
    # a chunk header with fewer than 12 bytes left (8..11) must not pass the length check, and a tRNS colour
    # key shorter than one 16-bit sample per channel must not be read past its end (stb_image: "bad tRNS len")
    import struct
    from another_raytracer_amd._lib import RTError
    ok = _png(_rgb_png_chunks() + [(b"IEND", b"")])
    p = tmp_path / "ok.png"
    p.write_bytes(ok)
    assert load_image(p).shape == (2, 2, 3)
    body = _png(_rgb_png_chunks())
    cases = {
        "trailing_header_8": body + struct.pack(">I", 4) + b"IDAT",
        "trailing_header_10": body + struct.pack(">I", 4) + b"IDAT" + b"\x00\x00",
        "trailing_header_11": body + struct.pack(">I", 0) + b"tEXt" + b"\x00\x00\x00",
        "huge_len": body + struct.pack(">I", 0xFFFFFFF0) + b"IDAT" + b"\x00" * 16,
        "rgb_trns_1_byte": _png(_rgb_png_chunks(2, [(b"tRNS", b"\x05")]) + [(b"IEND", b"")]),
        "rgb_trns_5_bytes": _png(_rgb_png_chunks(2, [(b"tRNS", b"\x00\x01\x00\x02\x00")]) + [(b"IEND", b"")]),
        "gray_trns_1_byte": _png(_rgb_png_chunks(0, [(b"tRNS", b"\x01")]) + [(b"IEND", b"")]),
    }
    for name, blob in cases.items():
        p = tmp_path / f"{name}.png"
        p.write_bytes(blob)
        with pytest.raises(RTError):
            load_image(p)
    # a well-formed key is accepted: gray + tRNS -> gray + alpha
    p = tmp_path / "gray_key.png"
    p.write_bytes(_png(_rgb_png_chunks(0, [(b"tRNS", b"\x00\x01")]) + [(b"IEND", b"")]))
    a = load_image(p)
    assert a.shape == (2, 2, 2) and list(a[:, :, 1].reshape(-1)) == [255, 0, 255, 0]


def test_png_chunk_order_matches_stb(tmp_path):
    # tRNS / PLTE / IHDR ordering as stb_image v2.27 decides it -- empty and repeated tRNS, tRNS before the
    # palette or after image data, colour keys whose high byte stb masks, chunks before IHDR -- against what stb itself
    # returned for the same files (tests/golden/png_chunks.npz, tools/gen_png_chunk_fixtures.py via ref_harness)
    from another_raytracer_amd._lib import RTError
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "png_chunks.npz"))
    names = sorted({k.split("__")[0] for k in g.files})
    assert len(names) >= 20
    for name in names:
        p = tmp_path / f"{name}.png"
        p.write_bytes(g[name + "__png"].tobytes())
        if not bool(g[name + "__ok"]):
            with pytest.raises(RTError):
                load_image(p)
            continue
        w, h, c = (int(x) for x in g[name + "__whc"])
        a = load_image(p)
        assert a.shape == (h, w, c), name
        assert np.array_equal(a.reshape(-1), g[name + "__data"]), name
