"""ctypes binding of libart.so (include/art.h).

The HIP path is the only compute path: if libart.so is missing this module raises ImportError at import time
instead of falling back to anything (there is no CPU fallback in the product).
"""
import ctypes
import os

try:
    # torch-ROCm ships its own libamdhip64.so.7.  Importing torch first makes libart's DT_NEEDED on the same SONAME bind
    # to that already-loaded runtime, so a process that uses both has ONE HIP runtime (device pointers, streams and
    # events are shared).  Loaded the other way round, torch cannot initialise its GPUs.
    import torch  # noqa: F401
except ImportError:
    pass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ART_LIB") or os.path.join(_HERE, "libart.so")  # ART_LIB: A/B another build

RT_OK = 0
RT_FP64 = 0  # the only fp_mode since ABI 2 (include/art.h)
RT_ABI_VERSION = 5
RT_OUT_DEVICE, RT_PROFILE, RT_GLOBAL_SCENE, RT_SPLIT_SHADE, RT_ADAPTIVE, RT_WAVEFRONT, RT_PARALLEL_IMAGES = 1, 2, 4, 8, 16, 32, 64
ERRORS = {-1: "RT_E_INVALID", -2: "RT_E_SCENE", -3: "RT_E_DEVICE", -4: "RT_E_INTERNAL"}


class rt_camera(ctypes.Structure):
    _fields_ = [("lookfrom", ctypes.c_double * 3), ("lookat", ctypes.c_double * 3), ("vup", ctypes.c_double * 3),
                ("vfov", ctypes.c_double), ("aspect", ctypes.c_double), ("aperture", ctypes.c_double),
                ("focus_dist", ctypes.c_double), ("time0", ctypes.c_double), ("time1", ctypes.c_double)]


class rt_params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("seed", ctypes.c_uint64), ("fp_mode", ctypes.c_int32),
                ("band_rows", ctypes.c_int32), ("band_count", ctypes.c_int32), ("band_index", ctypes.c_int32),
                ("samples_per_pass", ctypes.c_int32), ("flags", ctypes.c_int32), ("stream", ctypes.c_void_p),
                ("background", ctypes.c_double * 3)]


class rt_stats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("primary", ctypes.c_uint64), ("ms", ctypes.c_double),
                ("extend_ms", ctypes.c_double), ("shade_ms", ctypes.c_double),
                ("extend_launches", ctypes.c_uint64), ("shade_launches", ctypes.c_uint64),
                ("passes", ctypes.c_int32), ("samples_per_pass", ctypes.c_int32), ("local_rows", ctypes.c_int32),
                ("extend_variant", ctypes.c_int32), ("kernel_features", ctypes.c_uint32), ("kernel_textures", ctypes.c_uint32),
                ("kernel_lds_mode", ctypes.c_int32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class rt_scene_info(ctypes.Structure):
    _fields_ = [("lookfrom", ctypes.c_double * 3), ("lookat", ctypes.c_double * 3), ("vfov", ctypes.c_double),
                ("aperture", ctypes.c_double), ("background", ctypes.c_double * 3),
                ("spheres", ctypes.c_int64), ("triangles", ctypes.c_int64), ("rects", ctypes.c_int64),
                ("boxes", ctypes.c_int64), ("bvh_nodes", ctypes.c_int64), ("objects", ctypes.c_int64),
                ("materials", ctypes.c_int64), ("textures", ctypes.c_int64), ("has_media", ctypes.c_int32),
                ("max_bvh_depth", ctypes.c_int32), ("device_bytes_f64", ctypes.c_uint64)]


class rt_multi_times(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("render_ms_max", ctypes.c_double), ("render_ms_min", ctypes.c_double),
                ("gather_ms", ctypes.c_double), ("unpack_ms", ctypes.c_double), ("wait_ms", ctypes.c_double),
                ("collectives", ctypes.c_uint64), ("slowest_device", ctypes.c_int32), ("ngpus", ctypes.c_int32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


# rt_progress_fn (include/art.h): int (*)(void* user, int32_t samples_done, int32_t spp, const uint8_t*, const double*)
rt_progress_fn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p)

# Every symbol include/art.h declares, with its ctypes signature (tests/test_abi.py checks the header agrees).
_P, _I, _D, _S = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
_DP = ctypes.POINTER(ctypes.c_double)
_IP = ctypes.POINTER(ctypes.c_int)
SIGNATURES = {
    "rt_abi_version": (_I, []),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_device_count": (_I, []),
    "rt_option_set": (_I, [ctypes.c_char_p, _D]),
    "rt_option_get": (_I, [ctypes.c_char_p, _DP]),
    "rt_scene_build": (_I, [ctypes.c_char_p, ctypes.c_char_p, _I, ctypes.POINTER(_P)]),
    "rt_scene_info_get": (_I, [_P, ctypes.POINTER(rt_scene_info)]),
    "rt_scene_dump": (_S, [_P, ctypes.c_char_p, _S]),
    "rt_scene_destroy": (None, [_P]),
    "rt_scene_save": (_I, [_P, ctypes.c_char_p]),
    "rt_scene_load": (_I, [ctypes.c_char_p, _I, ctypes.POINTER(_P)]),
    "rt_render": (_I, [_P, ctypes.POINTER(rt_camera), ctypes.POINTER(rt_params), _P, _P, ctypes.POINTER(rt_stats)]),
    "rt_render_progressive": (_I, [_P, ctypes.POINTER(rt_camera), ctypes.POINTER(rt_params), _P, _P, rt_progress_fn, _P,
                                   ctypes.POINTER(rt_stats)]),
    "rt_trace_rays": (_I, [_P, _P, ctypes.c_int64, ctypes.c_int32, _P, _P]),
    "rt_image_load": (_I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                           ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))]),
    "rt_image_free": (None, [ctypes.POINTER(ctypes.c_uint8)]),
    "rt_local_rows": (_I, [ctypes.POINTER(rt_params), ctypes.POINTER(ctypes.c_int32)]),
    "rt_band_block_rows": (_I, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "rt_unpack_bands": (_I, [_P, _S, _P, _S, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P]),
    "rt_multi_create": (_I, [ctypes.c_char_p, ctypes.c_char_p, _IP, _I, ctypes.POINTER(_P)]),
    "rt_multi_from_graph": (_I, [_P, _IP, _I, ctypes.POINTER(_P)]),
    "rt_multi_destroy": (None, [_P]),
    "rt_render_multi": (_I, [_P, ctypes.POINTER(rt_camera), ctypes.POINTER(rt_params), _P, ctypes.POINTER(rt_stats)]),
    "rt_multi_ngpus": (_I, [_P]),
    "rt_multi_scene_info": (_I, [_P, ctypes.POINTER(rt_scene_info)]),
    "rt_multi_device_stats": (_I, [_P, _I, ctypes.POINTER(rt_stats)]),
    "rt_multi_times_get": (_I, [_P, ctypes.POINTER(rt_multi_times)]),
    "rt_graph_new": (_P, []),
    "rt_graph_free": (None, [_P]),
    "rt_graph_random_double": (_I, [_P, _DP]),
    "rt_tex_solid": (_I, [_P, _D, _D, _D]),
    "rt_tex_checker": (_I, [_P, _I, _I]),
    "rt_tex_noise": (_I, [_P, _D]),
    "rt_tex_image": (_I, [_P, _I, _I, _I, _P]),
    "rt_tex_bary_image": (_I, [_P, _DP, _I]),
    "rt_mesh_parse": (_I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "rt_mesh_build": (_I, [_P, ctypes.c_char_p, _IP]),
    "rt_mat_lambertian": (_I, [_P, _I]),
    "rt_mat_metal": (_I, [_P, _D, _D, _D, _D]),
    "rt_mat_dielectric": (_I, [_P, _D]),
    "rt_mat_diffuse_light": (_I, [_P, _I]),
    "rt_obj_sphere": (_I, [_P, _DP, _D, _I]),
    "rt_obj_moving_sphere": (_I, [_P, _DP, _DP, _D, _D, _D, _I]),
    "rt_obj_triangle": (_I, [_P, _DP, _DP, _DP, _I]),
    "rt_obj_rect": (_I, [_P, _I, _D, _D, _D, _D, _D, _I]),
    "rt_obj_box": (_I, [_P, _DP, _DP, _I]),
    "rt_obj_list": (_I, [_P, _I, _IP]),
    "rt_obj_bvh": (_I, [_P, _I, _IP]),
    "rt_obj_translate": (_I, [_P, _I, _DP]),
    "rt_obj_rotate_y": (_I, [_P, _I, _D]),
    "rt_obj_constant_medium": (_I, [_P, _I, _D, _I]),
    "rt_graph_add_world": (_I, [_P, _I]),
    "rt_graph_clear_world": (_I, [_P]),
    "rt_graph_set_view": (_I, [_P, _DP, _DP, _D, _D, _DP]),
    "rt_graph_compile": (_I, [_P, _I, ctypes.POINTER(_P)]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(or `make -C another_raytracer_amd/csrc`); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != RT_ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {lib.rt_abi_version()}, this binding expects {RT_ABI_VERSION}: rebuild it")
    return lib


lib = _load()


class RTError(RuntimeError):
    def __init__(self, code, where):
        msg = lib.rt_last_error().decode(errors="replace")
        super().__init__(f"{where} failed ({ERRORS.get(code, code)}): {msg}")
        self.code = code


def check(code, where):
    if code < 0:
        raise RTError(code, where)
    return code


def set_option(name, value):
    """rt_option_set (include/art.h): a process-wide library option; name None resets every option to its default."""
    check(lib.rt_option_set(None if name is None else name.encode(), float(value)), f"rt_option_set({name})")


def get_option(name):
    v = ctypes.c_double()
    check(lib.rt_option_get(name.encode(), ctypes.byref(v)), f"rt_option_get({name})")
    return v.value


def dvec(v):
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def _elf_sections(data):
    """(name, type, offset, size) of every section of a little-endian ELF64 image."""
    import struct
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError("not a little-endian ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    hdr = [struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stroff = hdr[shstrndx][4]
    return [(data[stroff + h[0]:data.index(b"\0", stroff + h[0])].decode(), h[1], h[4], h[5]) for h in hdr]


# the parts of a gfx950 code object that define what runs: kernel metadata (register and LDS use, arguments), kernel
# descriptors and machine code -- not the symbol tables, which carry hipcc's path-derived __hip_cuid_* names
_CODE_SECTIONS = (".note", ".rodata", ".text")


def kernel_build_id(path=None):
    """Identity of the device code in libart.so: the first 16 hex digits of a SHA-256 over the `.note`, `.rodata` and
    `.text` sections of every gfx950 code object in its `.hip_fatbin` offload bundles, in bundle order.  It depends on
    the kernels alone: host-only rebuilds, and rebuilds of the same sources at another path (whose `__hip_cuid_*` symbol
    names differ), keep it.  PMC summaries (tools/pmc_summary.py) are stamped with it, and bench.py uses a summary's
    per-segment counters only when the stamp equals the loaded build."""
    import hashlib
    import struct
    with open(path or LIB_PATH, "rb") as f:
        data = f.read()
    fb = [s for s in _elf_sections(data) if s[0] == ".hip_fatbin"]
    if not fb:
        raise ValueError("no .hip_fatbin section")
    _, _, off, size = fb[0]
    fat = data[off:off + size]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    h = hashlib.sha256()
    pos, objects = 0, 0
    while True:
        b = fat.find(magic, pos)
        if b < 0:
            break
        n, = struct.unpack_from("<Q", fat, b + len(magic))
        p = b + len(magic) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen]
            p += 24 + tlen
            if not triple.startswith(b"hipv4-amdgcn") or esize == 0:
                continue
            co = fat[b + eoff:b + eoff + esize]
            if co[:4] != b"\x7fELF":
                raise ValueError("compressed or unknown code object in the offload bundle")
            h.update(triple)
            for name, typ, soff, ssize in _elf_sections(co):
                if name in _CODE_SECTIONS:
                    h.update(name.encode() + struct.pack("<Q", ssize) + co[soff:soff + ssize])
            objects += 1
        pos = b + 1
    if objects == 0:
        raise ValueError("no gfx950 code object in .hip_fatbin")
    return h.hexdigest()[:16]
