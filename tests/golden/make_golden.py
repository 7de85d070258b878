"""Regenerate the golden fixtures from the reference itself (oracle/_ref/ref_harness).

Run in the build container only (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py

Everything written here is DATA: inputs and outputs of the unmodified reference program
(/root/reference/src compiled by oracle/Makefile, driven by oracle/ref_harness.cpp).  The
fixtures pin:
  * kat.json           first 32 random_double() of the reference's global mt19937 (tracer_utils.h:27-31)
  * scenes.json        per scene: the 8 random_double() following the scene build (RNG consumption of the
                       scene build incl. BVH-build draws) and the sha256 of the canonical scene dump
  * render_<scene>.npz reference renders (engine_mode::single semantics): RGB8, f64 per-pixel sums and the
                       exact segment count (world.hit calls)
  * render_stat_<scene>_384x216x<spp>.npz  the headline scene (alias 1, 16 spp), the cow and dino mesh scenes (16 spp)
                       and the Next-Week final (alias 8, 32 spp) rendered by the reference twice with independent sample
                       sequences -- engine_mode::single, and parallel_stripes with 4 threads (its shared global RNG)
                       -- for the statistical parity test of the f64 GPU path (SURVEY.md §8(d) tolerance 3: the
                       pair's RMSE is the noise floor); `make_golden.py stat [scene ...]` makes only these
  * images.npz         small JPEG / PNG files of every variant libart's decoder handles (baseline, progressive,
                       4:4:4 / 4:2:2 / 4:2:0, grayscale, CMYK, restart intervals, extreme quantizers; PNG gray 1..16
                       bits, palette +- tRNS, RGB(A), gray+alpha) made with PIL from a fixed pattern, each with the
                       bytes the reference's stb_image decodes from it (`ref_harness texture`); `make_golden.py images`
  * render_adaptive_<scene>.npz  engine_mode::adaptive renders (engine.h:96-333, its 4 stripes run in order):
                       RGB8 and segment count (`python tests/golden/make_golden.py adaptive` makes only these)
  * render_images_<scene>.npz  engine_mode::parallel_images renders (engine.h:378-445, its 4 partial images traced
                       in order): RGB8, the pixel_acc sums and the segment count (`make_golden.py images_mode`)
Assets written by the same harness: assets/*.tris (the reference's post-triangulation triangle lists: cow,
dino, capsule incl. its texture coordinates; the oracle's mesh input and the pin of the product's OBJ loader),
assets/earthmap.rgb and assets/models/capsule/capsule.rgb.gz (stb_image-decoded texels, the latter gzipped).
`python tests/golden/make_golden.py scene NAME` (re)makes one scene's fixtures without touching the others.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
REF = "/root/reference"

SCENES = ["c1", "1", "2", "3", "4", "5", "6", "7", "8", "cow", "dino", "9"]
SMALL = (64, 36, 4)          # every scene, RGB + f64 sums + segments
CONFIG1 = ("c1", 400, 225, 64)  # BASELINE configs[0]: the CPU reference path at full size
ADAPTIVE = ["c1", "1", "8", "cow"]
ADAPTIVE_SIZE = (96, 48, 4)     # multiples of the 12-px big square (engine.h:178-179)


def run(*args):
    return subprocess.run([HARNESS, *map(str, args)], check=True, capture_output=True, text=True).stdout


def render(scene, W, H, spp, tmp="/tmp/golden_ref"):
    info = json.loads(run("render", scene, W, H, spp, tmp).strip().splitlines()[-1])
    rgb = np.fromfile(tmp + ".rgb", np.uint8).reshape(H, W, 3)
    acc = np.fromfile(tmp + ".acc", np.float64).reshape(H, W, 3)
    return rgb, acc, info


def adaptive_fixtures():
    W, H, spp = ADAPTIVE_SIZE
    for sc in ADAPTIVE:
        tmp = "/tmp/golden_adaptive"
        info = json.loads(run("render", sc, W, H, spp, tmp, "adaptive").strip().splitlines()[-1])
        rgb = np.fromfile(tmp + ".rgb", np.uint8).reshape(H, W, 3)
        np.savez_compressed(os.path.join(HERE, f"render_adaptive_{sc}_{W}x{H}x{spp}.npz"), rgb=rgb,
                            segments=np.int64(info["segments"]), W=W, H=H, spp=spp)
        print("adaptive", sc, info)


# engine_mode::parallel_images (engine.h:378-445; the four partial images traced in order): spp not a multiple of 4,
# so 4 * (spp / 4) samples are traced and write_color divides by spp, as the reference does
IMAGES = [("c1", 48, 27, 10), ("4", 40, 24, 6)]


def images_mode_fixtures():
    for sc, W, H, spp in IMAGES:
        tmp = "/tmp/golden_images"
        info = json.loads(run("render", sc, W, H, spp, tmp, "images").strip().splitlines()[-1])
        rgb = np.fromfile(tmp + ".rgb", np.uint8).reshape(H, W, 3)
        acc = np.fromfile(tmp + ".acc", np.float64).reshape(H, W, 3)
        np.savez_compressed(os.path.join(HERE, f"render_images_{sc}_{W}x{H}x{spp}.npz"), rgb=rgb, acc=acc,
                            segments=np.int64(info["segments"]), W=W, H=H, spp=spp)
        print("images", sc, info)


STAT = [("1", 384, 216, 16), ("cow", 384, 216, 16), ("8", 384, 216, 32), ("dino", 384, 216, 16)]


def stat_fixtures(only=None):
    for sc, W, H, spp in STAT:
        if only is None or sc in only:
            stat_fixture(sc, W, H, spp)


def stat_fixture(sc, W, H, spp):
    rgb, acc, info = render(sc, W, H, spp)
    tmp = "/tmp/golden_stat_stripes"
    info2 = json.loads(run("render", sc, W, H, spp, tmp, "stripes", 4).strip().splitlines()[-1])
    rgb2 = np.fromfile(tmp + ".rgb", np.uint8).reshape(H, W, 3)
    np.savez_compressed(os.path.join(HERE, f"render_stat_{sc}_{W}x{H}x{spp}.npz"), rgb_single=rgb, rgb_stripes=rgb2,
                        segments_single=np.int64(info["segments"]), segments_stripes=np.int64(info2["segments"]),
                        W=W, H=H, spp=spp)
    print("stat", sc, info, info2)


def image_fixtures():
    import io

    from PIL import Image
    rng = np.random.default_rng(1)
    W, H = 53, 37
    yy, xx = np.mgrid[0:H, 0:W]
    rgb = np.stack([(xx * 255 // W), (yy * 255 // H), ((xx + yy) * 4) % 256], -1).astype(np.int32)
    rgb = np.clip(rgb + rng.integers(-40, 41, rgb.shape), 0, 255).astype(np.uint8)
    gray = rgb.mean(-1).astype(np.uint8)
    out = {}

    def add(name, img, fmt, **kw):
        buf = io.BytesIO()
        img.save(buf, fmt, **kw)
        data = buf.getvalue()
        path = f"/tmp/golden_img_{name}"
        with open(path, "wb") as f:
            f.write(data)
        run("texture", path, path + ".raw")
        blob = open(path + ".raw", "rb").read()
        w, h, c = np.frombuffer(blob[:12], np.int32)
        dec = np.frombuffer(blob[12:], np.uint8)
        out[f"{name}__file"] = np.frombuffer(data, np.uint8)
        out[f"{name}__decoded"] = dec
        out[f"{name}__whc"] = np.array([w, h, c], np.int32)
        print("image", name, len(data), "bytes ->", w, h, c, len(dec))

    im = Image.fromarray(rgb, "RGB")
    add("jpg_444", im, "JPEG", quality=90, subsampling=0)
    add("jpg_422", im, "JPEG", quality=85, subsampling=1)
    add("jpg_420", im, "JPEG", quality=75, subsampling=2)
    add("jpg_420_prog", im, "JPEG", quality=80, subsampling=2, progressive=True)
    add("jpg_444_prog", im, "JPEG", quality=95, subsampling=0, progressive=True)
    add("jpg_444_optimized", im, "JPEG", quality=70, subsampling=0, optimize=True)
    add("jpg_q100", im, "JPEG", quality=100, subsampling=0)
    add("jpg_q3", im, "JPEG", quality=3, subsampling=2)
    add("jpg_restart", im, "JPEG", quality=85, subsampling=2, restart_marker_blocks=3)
    add("jpg_restart_prog", im, "JPEG", quality=85, subsampling=0, progressive=True, restart_marker_rows=1)
    add("jpg_gray", Image.fromarray(gray, "L"), "JPEG", quality=85)
    add("jpg_gray_prog", Image.fromarray(gray, "L"), "JPEG", quality=85, progressive=True)
    add("jpg_cmyk", im.convert("CMYK"), "JPEG", quality=90)
    add("png_rgb", im, "PNG")
    add("png_rgba", Image.fromarray(np.dstack([rgb, gray]), "RGBA"), "PNG")
    add("png_gray", Image.fromarray(gray, "L"), "PNG")
    add("png_la", Image.fromarray(np.dstack([gray, 255 - gray]), "LA"), "PNG")
    add("png_gray1", Image.fromarray(gray > 128), "PNG")
    add("png_pal", im.convert("P", palette=Image.ADAPTIVE, colors=16), "PNG")
    add("png_pal_trns", im.convert("P", palette=Image.ADAPTIVE, colors=16), "PNG", transparency=3)
    add("png_gray16", Image.fromarray((gray.astype(np.uint16) * 257 + 3).astype(np.uint16), "I;16"), "PNG")
    pal4 = im.convert("P", palette=Image.ADAPTIVE, colors=4)
    add("png_pal2bit", pal4, "PNG", bits=2)
    np.savez_compressed(os.path.join(HERE, "images.npz"), **out)


def scene_fixtures(sc):
    """probe + dump hash (scenes.json entry) and the SMALL render of one scene."""
    # the harness may log texture loads on stdout first: the values are the last 8 lines
    probe = [float(x) for x in run("probe", sc, 8).strip().splitlines()[-8:]]
    run("dump", sc, "/tmp/golden_dump.json")
    dump = open("/tmp/golden_dump.json", "rb").read()
    W, H, spp = SMALL
    rgb, acc, info = render(sc, W, H, spp)
    np.savez_compressed(os.path.join(HERE, f"render_{sc}_{W}x{H}x{spp}.npz"), rgb=rgb, acc=acc,
                        segments=np.int64(info["segments"]), W=W, H=H, spp=spp)
    print(sc, info)
    return {"probe": probe, "dump_sha256": hashlib.sha256(dump).hexdigest(), "dump_len": len(dump)}


def assets_fixtures():
    assets = os.path.join(ROOT, "assets")
    os.makedirs(os.path.join(assets, "models", "capsule"), exist_ok=True)
    run("mesh", "cow", os.path.join(assets, "cow.tris"))
    run("mesh", "dino", os.path.join(assets, "dino.tris"))
    run("mesh", "capsule", os.path.join(assets, "capsule.tris"))
    run("texture", f"{REF}/textures/earthmap.jpg", os.path.join(assets, "earthmap.rgb"))
    raw = "/tmp/golden_capsule.rgb"
    run("texture", f"{REF}/models/capsule/capsule.jpg", raw)
    import gzip
    with open(raw, "rb") as fi, gzip.GzipFile(os.path.join(assets, "models", "capsule", "capsule.rgb.gz"), "wb", 9,
                                                mtime=0) as fo:
        fo.write(fi.read())


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle ref")
    if sys.argv[1:] == ["adaptive"]:
        adaptive_fixtures()
        return
    if sys.argv[1:2] == ["stat"]:
        stat_fixtures(sys.argv[2:] or None)
        return
    if sys.argv[1:] == ["images"]:
        image_fixtures()
        return
    if sys.argv[1:] == ["images_mode"]:
        images_mode_fixtures()
        return
    if sys.argv[1:2] == ["scene"]:
        path = os.path.join(HERE, "scenes.json")
        scenes = json.load(open(path))
        for sc in sys.argv[2:]:
            scenes[sc] = scene_fixtures(sc)
        with open(path, "w") as f:
            json.dump(scenes, f, indent=1)
        return
    assets_fixtures()

    kat = [float(x) for x in run("kat", 32).split()]
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"seed": 5489, "random_double": kat}, f, indent=1)

    scenes = {sc: scene_fixtures(sc) for sc in SCENES}
    with open(os.path.join(HERE, "scenes.json"), "w") as f:
        json.dump(scenes, f, indent=1)

    sc, W, H, spp = CONFIG1
    rgb, acc, info = render(sc, W, H, spp)
    np.savez_compressed(os.path.join(HERE, f"render_{sc}_{W}x{H}x{spp}.npz"), rgb=rgb,
                        acc=acc.astype(np.float64), segments=np.int64(info["segments"]), W=W, H=H, spp=spp)
    print(sc, info)
    adaptive_fixtures()
    stat_fixtures()
    image_fixtures()
    images_mode_fixtures()


if __name__ == "__main__":
    main()
