"""imageio surface of the reference (src/utils/imageio.{h,cpp}): save_image writes a PNG (stdlib zlib encoder in
place of stb_image_write), load_image reads PNGs written here and the raw texel assets (int32 w, h, bpp + bytes)."""
import struct
import zlib

import numpy as np


def save_image(path, width, height, bytes_per_pixel, data):  # imageio.cpp:17-20
    a = np.asarray(data.cpu() if hasattr(data, "cpu") else data, dtype=np.uint8).reshape(height, width, bytes_per_pixel)
    color_type = {1: 0, 2: 4, 3: 2, 4: 6}[bytes_per_pixel]
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(height))

    def chunk(tag, payload):
        return struct.pack(">I", len(payload)) + tag + payload + struct.pack(">I", zlib.crc32(tag + payload) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", width, height, 8, color_type, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)
    return True


def load_image(path):  # imageio.cpp:11-15 -> (array (H, W, C) uint8)
    with open(path, "rb") as f:
        blob = f.read()
    if blob[:8] != b"\x89PNG\r\n\x1a\n":
        w, h, c = np.frombuffer(blob[:12], np.int32)
        return np.frombuffer(blob[12:], np.uint8)[: w * h * c].reshape(h, w, c).copy()
    pos, idat, hdr = 8, b"", None
    while pos < len(blob):
        n, tag = struct.unpack(">I4s", blob[pos:pos + 8])
        payload = blob[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", payload)
        elif tag == b"IDAT":
            idat += payload
        pos += 12 + n
    w, h, depth, ctype = hdr[0], hdr[1], hdr[2], hdr[3]
    c = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    if depth != 8:
        raise ValueError("only 8-bit PNGs are supported")
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, w * c + 1)
    out = np.zeros((h, w * c), np.int32)
    prev = np.zeros(w * c, np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        cur = np.zeros(w * c, np.int32)
        for x in range(w * c):
            a = cur[x - c] if x >= c else 0
            b = prev[x]
            cc = prev[x - c] if x >= c else 0
            if f == 0: v = line[x]
            elif f == 1: v = line[x] + a
            elif f == 2: v = line[x] + b
            elif f == 3: v = line[x] + (a + b) // 2
            else:
                p = a + b - cc
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - cc)
                v = line[x] + (a if pa <= pb and pa <= pc else b if pb <= pc else cc)
            cur[x] = v & 0xFF
        out[y] = cur
        prev = cur
    return out.astype(np.uint8).reshape(h, w, c)
