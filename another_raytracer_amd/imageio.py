"""imageio surface of the reference (src/utils/imageio.{h,cpp}): save_image writes a PNG (stdlib zlib encoder in
place of stb_image_write); load_image decodes JPEG / PNG through libart (rt_image_load) and reads raw texel assets."""
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


def load_image(path):  # imageio.cpp:11-15 -> array (H, W, C) uint8
    """stbi_load(path, .., 0): JPEG / PNG decoded by libart (rt_image_load, csrc/imagedec.cpp), native channels; a raw
    texel asset (int32 w, h, bpp + bytes) is read as is."""
    import ctypes
    import os

    from ._lib import check, lib
    if os.fspath(path).endswith(".rgb"):
        with open(path, "rb") as f:
            blob = f.read()
        w, h, c = np.frombuffer(blob[:12], np.int32)
        return np.frombuffer(blob[12:], np.uint8)[: w * h * c].reshape(h, w, c).copy()
    w, h, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    px = ctypes.POINTER(ctypes.c_uint8)()
    check(lib.rt_image_load(os.fspath(path).encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c), ctypes.byref(px)), "load_image")
    try:
        return np.ctypeslib.as_array(px, shape=(h.value, w.value, c.value)).copy()
    finally:
        lib.rt_image_free(px)
