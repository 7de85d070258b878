"""Flat-scene files (rt_scene_save / rt_scene_load, csrc/scenefile.cpp) on the CPU: a saved scene loads back to the same
compiled scene (saving the loaded scene writes the same bytes), the scene_manager view survives, loading skips the
rebuild, and damaged files are refused with a reason.  The GPU render of a loaded scene: tests/test_gpu_api.py."""
import time

import numpy as np
import pytest

import another_raytracer_amd as art


@pytest.mark.parametrize("name", ["1", "8", "9", "cow", "c1"])
def test_save_load_roundtrip_is_exact(name, tmp_path):
    w = art.scene_manager().build(name)
    a = tmp_path / "a.artscene"
    art.save_scene(w, a)
    loaded = art.scene_manager().load(a)
    b = tmp_path / "b.artscene"
    art.save_scene(loaded, b)
    assert a.read_bytes() == b.read_bytes()
    for k in ("lookfrom", "lookat", "vfov", "aperture", "background", "spheres", "triangles", "rects", "boxes", "bvh_nodes",
              "objects", "materials", "textures", "has_media", "max_bvh_depth"):
        assert w.info[k] == loaded.info[k], k
    assert (loaded.lookfrom, loaded.lookat, loaded.vfov, loaded.aperture) == (w.lookfrom, w.lookat, w.vfov, w.aperture)


def test_loading_skips_the_rebuild(tmp_path):
    t0 = time.perf_counter()
    w = art.scene_manager().build("9")  # the capsule: OBJ/MTL parse, earcut, JPEG decode, SAH build
    t1 = time.perf_counter()
    art.save_scene(w, tmp_path / "capsule.artscene")
    t2 = time.perf_counter()
    art.scene_manager().load(tmp_path / "capsule.artscene")
    t3 = time.perf_counter()
    print(f"build {t1 - t0:.3f} s, save {t2 - t1:.3f} s, load {t3 - t2:.3f} s")
    assert t3 - t2 < t1 - t0


def test_damaged_files_are_refused(tmp_path):
    w = art.scene_manager().build("1")
    p = tmp_path / "s.artscene"
    art.save_scene(w, p)
    blob = bytearray(p.read_bytes())
    cases = {"bad magic": b"XXXXXXXX" + bytes(blob[8:]), "truncated": bytes(blob[:-100]),
             "checksum": bytes(blob[:-1]) + bytes([blob[-1] ^ 0x5A]), "version": bytes(blob[:8]) + b"\x07\x00\x00\x00" + bytes(blob[12:]),
             "empty": b""}
    for why, data in cases.items():
        q = tmp_path / f"bad_{why.replace(' ', '_')}.artscene"
        q.write_bytes(data)
        with pytest.raises(art.RTError) as e:
            art.scene_manager().load(q)
        assert e.value.code == -2, why
    with pytest.raises(art.RTError):
        art.scene_manager().load(tmp_path / "missing.artscene")


class _Header(__import__("ctypes").Structure):
    """csrc/scenefile.cpp FileHeader (13 arrays: spheres, tris, rects, boxes, primrefs, nodes, objs, world, mats, texs,
    perlins, images, texels)."""
    import ctypes as _c
    _fields_ = [("magic", _c.c_char * 8), ("version", _c.c_uint32), ("header_bytes", _c.c_uint32), ("record_bytes", _c.c_uint32 * 13),
                ("features", _c.c_uint32), ("has_media", _c.c_int32), ("max_bvh_depth", _c.c_int32), ("max_stack", _c.c_int32),
                ("background", _c.c_double * 3), ("lookfrom", _c.c_double * 3), ("lookat", _c.c_double * 3), ("vfov", _c.c_double),
                ("aperture", _c.c_double), ("offset", _c.c_uint64 * 13), ("count", _c.c_uint64 * 13), ("payload_bytes", _c.c_uint64),
                ("checksum", _c.c_uint64)]


def _fnv1a(data):
    h = 1469598103934665603
    for b in data:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_tampered_header_and_payload_are_refused(tmp_path):
    # the header is outside the checksum, so its array table must not wrap and its derived fields
    # (max_stack sizes the LDS traversal stacks) must equal what the arrays imply; a payload whose indices point
    # outside the arrays is refused even when its checksum is right
    import ctypes
    w = art.scene_manager().build("1")
    p = tmp_path / "s.artscene"
    art.save_scene(w, p)
    blob = bytes(p.read_bytes())
    hsz = ctypes.sizeof(_Header)
    h0 = _Header.from_buffer_copy(blob[:hsz])
    assert h0.header_bytes == hsz and h0.magic == b"ARTSCN"
    start = (hsz + 63) // 64 * 64
    assert art.scene_manager().load(p) is not None

    def with_header(**kw):
        h = _Header.from_buffer_copy(blob[:hsz])
        for k, v in kw.items():
            if isinstance(v, tuple):
                getattr(h, k)[v[0]] = v[1]
            else:
                setattr(h, k, v)
        return bytes(h) + blob[hsz:]

    def with_payload(edit):
        h = _Header.from_buffer_copy(blob[:hsz])
        pay = bytearray(blob[start:])
        edit(h, pay)
        h.checksum = _fnv1a(pay)
        return bytes(h) + blob[hsz:start] + bytes(pay)

    def prim0_out_of_range(h, pay):
        off = h.offset[4] - start
        pay[off:off + 4] = (h.count[0] + 5).to_bytes(4, "little")  # sphere index past the spheres

    def child_to_parent(h, pay):
        off = h.offset[5] - start + 96  # node 0's child[0] (BvhNode: 6 x float4 planes, then int32 child[4])
        pay[off:off + 4] = (0).to_bytes(4, "little")  # node 0 -> node 0: a cycle the GPU would walk forever

    def empty_slot_box(h, pay):
        # the first node with an empty child slot gets a finite box there (lox..hiz: 6 x float4, child[4] at +96)
        import struct
        base = h.offset[5] - start
        for n in range(h.count[5]):
            o = base + 128 * n
            ch = struct.unpack_from("<4i", pay, o + 96)
            if -1 in ch:
                c = ch.index(-1)
                for plane, v in enumerate((0.0, 1.0, 0.0, 1.0, 0.0, 1.0)):
                    struct.pack_into("<f", pay, o + 16 * plane + 4 * c, v)
                return
        raise AssertionError("no empty slot in scene 1's BVH")

    cases = {
        "empty slot box": with_payload(empty_slot_box),
        "offset wraps": with_header(offset=(0, 2 ** 64 - 64)),
        "count wraps": with_header(count=(5, 2 ** 61)),
        "count past end": with_header(count=(12, h0.count[12] + 10 ** 6)),
        "max_stack too small": with_header(max_stack=max(h0.max_stack - 1, 0) if h0.max_stack else 5),
        "max_stack too large": with_header(max_stack=1000),
        "features": with_header(features=h0.features | 2),
        "has_media": with_header(has_media=1 - h0.has_media),
        "primref out of range": with_payload(prim0_out_of_range),
        "bvh cycle": with_payload(child_to_parent),
    }
    for why, data in cases.items():
        q = tmp_path / f"bad_{why.replace(' ', '_')}.artscene"
        q.write_bytes(data)
        with pytest.raises(art.RTError) as e:
            art.scene_manager().load(q)
        assert e.value.code == -2, why
