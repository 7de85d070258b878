"""Golden vectors for PNG chunk-order edge cases (tRNS / PLTE / IHDR ordering), decoded by stb_image v2.27 itself: each
crafted file goes through the reference's own imageio::load_image (oracle/_ref/ref_harness texture, built from
/root/reference/src by oracle/Makefile), and the outcome -- refused, or width / height / channels / bytes -- is saved
to tests/golden/png_chunks.npz for tests/test_imagedec.py.  Run in the build container:
    python tools/gen_png_chunk_fixtures.py"""
import os
import struct
import subprocess
import sys
import tempfile
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def png(chunks):
    out = b"\x89PNG\r\n\x1a\n"
    for typ, data in chunks:
        out += struct.pack(">I", len(data)) + typ + data + struct.pack(">I", zlib.crc32(typ + data) & 0xFFFFFFFF)
    return out


def ihdr(w, h, depth, ctype):
    return (b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))


def idat(rows):
    return (b"IDAT", zlib.compress(b"".join(b"\x00" + r for r in rows)))


PAL = (b"PLTE", bytes(range(30, 30 + 15)))  # 5 entries
PIDX = idat([bytes([0, 1, 2, 3]), bytes([4, 3, 2, 1])])  # 4x2, 8-bit palette indices
GRAY = idat([bytes([5, 7, 5, 9]), bytes([5, 5, 0, 255])])  # 4x2 gray 8
GRAY2 = idat([bytes([0b00011011]), bytes([0b01010101])])  # 4x2 gray 2-bit: 0 1 2 3 / 1 1 1 1
RGB = idat([bytes([1, 2, 3, 4, 5, 6]), bytes([1, 2, 3, 9, 9, 9])])  # 2x2 RGB 8
END = (b"IEND", b"")

CASES = {
    "pal_trns_empty": [ihdr(4, 2, 8, 3), PAL, (b"tRNS", b""), PIDX, END],
    "pal_trns_before_plte": [ihdr(4, 2, 8, 3), (b"tRNS", b"\x10"), PAL, PIDX, END],
    "pal_trns_after_idat": [ihdr(4, 2, 8, 3), PAL, PIDX, (b"tRNS", b"\x10"), END],
    "pal_trns_twice": [ihdr(4, 2, 8, 3), PAL, (b"tRNS", b"\x01\x02\x03\x04\x05"), (b"tRNS", b"\x99\x98"), PIDX, END],
    "pal_trns_too_long": [ihdr(4, 2, 8, 3), PAL, (b"tRNS", b"\x01" * 6), PIDX, END],
    "pal_trns_short": [ihdr(4, 2, 8, 3), PAL, (b"tRNS", b"\x00\x40"), PIDX, END],
    "pal_plte_bad_len": [ihdr(4, 2, 8, 3), (b"PLTE", b"\x01\x02\x03\x04"), PIDX, END],
    "pal_no_plte": [ihdr(4, 2, 8, 3), PIDX, END],
    "pal_plte_after_idat": [ihdr(4, 2, 8, 3), PAL, PIDX, (b"PLTE", bytes(range(100, 115))), END],
    "gray_trns_empty": [ihdr(4, 2, 8, 0), (b"tRNS", b""), GRAY, END],
    "gray_trns_after_idat": [ihdr(4, 2, 8, 0), GRAY, (b"tRNS", b"\x00\x05"), END],
    "gray_key_high_byte": [ihdr(4, 2, 8, 0), (b"tRNS", b"\x01\x05"), GRAY, END],
    "gray_key": [ihdr(4, 2, 8, 0), (b"tRNS", b"\x00\x05"), GRAY, END],
    "gray2_key_high_byte": [ihdr(4, 2, 2, 0), (b"tRNS", b"\x01\x01"), GRAY2, END],
    "gray2_key": [ihdr(4, 2, 2, 0), (b"tRNS", b"\x00\x02"), GRAY2, END],
    "rgb_key_twice": [ihdr(2, 2, 8, 2), (b"tRNS", b"\x00\x01\x00\x02\x00\x03"), (b"tRNS", b"\x00\x09\x00\x09\x00\x09"), RGB, END],
    "rgb_suggested_plte": [ihdr(2, 2, 8, 2), PAL, (b"tRNS", b"\x00\x01\x00\x02\x00\x03"), RGB, END],
    "rgba_trns": [ihdr(1, 1, 8, 6), (b"tRNS", b"\x00\x01\x00\x02\x00\x03"), idat([b"\x01\x02\x03\x04"]), END],
    "text_before_ihdr": [(b"tEXt", b"a\x00b"), ihdr(4, 2, 8, 0), GRAY, END],
    "two_ihdr": [ihdr(4, 2, 8, 0), ihdr(4, 2, 8, 0), GRAY, END],
}


def stb_decode(blob):
    with tempfile.TemporaryDirectory() as d:
        src, out = os.path.join(d, "x.png"), os.path.join(d, "x.bin")
        open(src, "wb").write(blob)
        r = subprocess.run([HARNESS, "texture", src, out], capture_output=True)
        if r.returncode != 0:
            return None
        raw = open(out, "rb").read()
        w, h, c = struct.unpack_from("<3i", raw)
        return w, h, c, np.frombuffer(raw[12:], np.uint8)


def main():
    if not os.path.exists(HARNESS):
        sys.exit(f"{HARNESS} missing: build it with `make -C oracle ref` (needs /root/reference)")
    out = {}
    for name, chunks in CASES.items():
        blob = png(chunks)
        res = stb_decode(blob)
        out[name + "__png"] = np.frombuffer(blob, np.uint8)
        out[name + "__ok"] = np.array(res is not None)
        if res is not None:
            out[name + "__whc"] = np.array(res[:3], np.int32)
            out[name + "__data"] = res[3]
        print(name, "refused" if res is None else res[:3])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "png_chunks.npz"), **out)


if __name__ == "__main__":
    main()
