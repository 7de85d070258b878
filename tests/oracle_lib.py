"""ctypes access to the oracle (oracle/_ref/liboracle.so) — TEST INFRASTRUCTURE.  Used only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker / CPU baseline, never as the product."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_ref", "liboracle.so")
REF_HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
ASSETS = os.path.join(ROOT, "assets")
MODES = {"mt": 0, "pcg": 1}

_lib = None


def oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "restate"], check=True)
        lib = ctypes.CDLL(ORACLE_SO)
        lib.orc_last_error.restype = ctypes.c_char_p
        lib.orc_dump.restype = ctypes.c_size_t
        lib.orc_render.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
        lib.orc_render_rows.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
        lib.orc_render_adaptive.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
        lib.orc_render_images.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
        lib.orc_set_asset_dir(ASSETS.encode())
        _lib = lib
    return _lib


def oracle_render(scene, W, H, spp, mode="pcg", seed=0, row0=0, nrows=None, threads=0, max_depth=50):
    lib = oracle()
    nrows = H if nrows is None else nrows
    rgb = np.zeros((nrows, W, 3), np.uint8)
    acc = np.zeros((nrows, W, 3), np.float64)
    segs, ms = ctypes.c_longlong(), ctypes.c_double()
    r = lib.orc_render(str(scene).encode(), W, H, spp, max_depth, MODES[mode], seed, row0, nrows, threads,
                       rgb.ctypes.data, acc.ctypes.data, ctypes.byref(segs), ctypes.byref(ms))
    if r != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return {"rgb": rgb, "acc": acc, "segments": segs.value, "ms": ms.value}


def oracle_render_rows(scene, W, H, spp, rows, seed=0, threads=0, max_depth=50):
    """pcg-mode render of the listed global rows of a WxH frame (dynamic (row, column chunk) work items)."""
    lib = oracle()
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    n = len(rows)
    rgb = np.zeros((n, W, 3), np.uint8)
    acc = np.zeros((n, W, 3), np.float64)
    segs, ms = ctypes.c_longlong(), ctypes.c_double()
    r = lib.orc_render_rows(str(scene).encode(), W, H, spp, max_depth, seed, rows.ctypes.data, n, threads, rgb.ctypes.data,
                            acc.ctypes.data, ctypes.byref(segs), ctypes.byref(ms))
    if r != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return {"rgb": rgb, "acc": acc, "segments": segs.value, "ms": ms.value}


def oracle_trace_rays(scene, rays):
    """Closest hits (t, normals) of rays (n x 7: o, d, tm) in the scene's world (hittable_list::hit)."""
    lib = oracle()
    rays = np.ascontiguousarray(rays, dtype=np.float64)
    n = len(rays)
    t = np.zeros(n, np.float64)
    nrm = np.zeros((n, 3), np.float64)
    r = lib.orc_trace_rays(str(scene).encode(), rays.ctypes.data_as(ctypes.c_void_p), ctypes.c_longlong(n),
                           t.ctypes.data_as(ctypes.c_void_p), nrm.ctypes.data_as(ctypes.c_void_p))
    if r != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return t, nrm


def oracle_render_adaptive(scene, W, H, spp, mode="pcg", seed=0, threads=0, max_depth=50):
    lib = oracle()
    rgb = np.zeros((H, W, 3), np.uint8)
    segs, ms = ctypes.c_longlong(), ctypes.c_double()
    r = lib.orc_render_adaptive(str(scene).encode(), W, H, spp, max_depth, MODES[mode], seed, threads, rgb.ctypes.data,
                                ctypes.byref(segs), ctypes.byref(ms))
    if r != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return {"rgb": rgb, "segments": segs.value, "ms": ms.value}


def oracle_render_images(scene, W, H, spp, mode="pcg", seed=0, threads=0, max_depth=50):
    """engine_mode::parallel_images (engine.h:378-445): four float partial images of spp/4 samples summed."""
    lib = oracle()
    rgb = np.zeros((H, W, 3), np.uint8)
    acc = np.zeros((H, W, 3), np.float64)
    segs, ms = ctypes.c_longlong(), ctypes.c_double()
    r = lib.orc_render_images(str(scene).encode(), W, H, spp, max_depth, MODES[mode], seed, threads, rgb.ctypes.data,
                              acc.ctypes.data, ctypes.byref(segs), ctypes.byref(ms))
    if r != 0:
        raise RuntimeError(lib.orc_last_error().decode())
    return {"rgb": rgb, "acc": acc, "segments": segs.value, "ms": ms.value}


def oracle_dump(scene):
    lib = oracle()
    n = lib.orc_dump(str(scene).encode(), None, 0)
    buf = ctypes.create_string_buffer(n)
    lib.orc_dump(str(scene).encode(), buf, n)
    return buf.value.decode()


def oracle_kat(n):
    out = (ctypes.c_double * n)()
    oracle().orc_kat(n, out)
    return list(out)


def oracle_probe(scene, k):
    out = (ctypes.c_double * k)()
    if oracle().orc_probe(str(scene).encode(), k, out) != 0:
        raise RuntimeError(oracle().orc_last_error().decode())
    return list(out)
