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
