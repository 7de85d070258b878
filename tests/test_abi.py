"""The C ABI boundary (include/art.h <-> libart.so <-> the ctypes mirror), host-only: no compute calls."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import another_raytracer_amd as art
from another_raytracer_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "art.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_\w+)\s*\(", text)))


def test_every_declared_symbol_is_exported_and_bound():
    decl = declared_functions()
    assert len(decl) >= 30
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (rt_\w+)", nm))
    assert set(decl) <= exported, set(decl) - exported
    assert set(decl) == set(_lib.SIGNATURES), set(decl) ^ set(_lib.SIGNATURES)
    assert _lib.lib.rt_abi_version() == _lib.RT_ABI_VERSION == 5


def test_struct_layouts_match_the_header(tmp_path):
    src = tmp_path / "layout.c"
    fields = {"rt_camera": [f for f, _ in _lib.rt_camera._fields_], "rt_params": [f for f, _ in _lib.rt_params._fields_],
              "rt_stats": [f for f, _ in _lib.rt_stats._fields_], "rt_scene_info": [f for f, _ in _lib.rt_scene_info._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "art.h"', "int main(void) {"]
    for st, fs in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0; }")
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    c = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines())
    for st, fs in fields.items():
        cls = getattr(_lib, st)
        assert int(c[st]) == ctypes.sizeof(cls), st
        for f in fs:
            assert int(c[f"{st}.{f}"]) == getattr(cls, f).offset, f"{st}.{f}"


OPTIONS = {  # include/art.h rt_option_set: name -> default
    "compile.world_merge": 2, "compile.hoist": 1, "bvh.collapse": 0, "bvh.collapse_ci": 0.6, "bvh.dp_binary_leaf": 1,
    "bvh.sah_ci": 1.5, "bvh.sah_leaf": 4, "bvh.sbvh": 1.5, "bvh.sbvh_alpha": 1e-5, "render.codes16": 1,
    "render.lds_nodes_max": 4294967295, "render.leaf2": 1, "render.tex_bary": 1, "multi.rccl_blocking": 0, "test.fault_workspace_bytes": 0,
    "test.fault_gather_abort": 0, "test.fault_rccl_group": 0,
}


def test_options_defaults_set_get_and_reset():
    art.set_option(None, 0)
    for name, default in OPTIONS.items():
        assert art.get_option(name) == pytest.approx(default), name
    art.set_option("compile.world_merge", 1)
    art.set_option("test.fault_workspace_bytes", 1 << 20)
    art.set_option("multi.timeout_ms", 2500)
    assert art.get_option("compile.world_merge") == 1 and art.get_option("test.fault_workspace_bytes") == 1 << 20
    assert art.get_option("multi.timeout_ms") == 2500
    art.set_option(None, 0)  # NULL name: every option back to its default
    assert art.get_option("compile.world_merge") == 2 and art.get_option("test.fault_workspace_bytes") == 0
    assert art.get_option("multi.timeout_ms") == 120000  # unset: ART_MULTI_TIMEOUT_MS (not set here) or 120 s


def test_infinite_multi_timeout_is_accepted():
    # "no deadline" (ADVICE r5): inf is inside the option's range; multi.hip turns it (or anything whose nanoseconds
    # overflow the clock) into no deadline instead of an undefined duration_cast (tests/test_gpu_api.py renders with it)
    art.set_option("multi.timeout_ms", float("inf"))
    try:
        assert art.get_option("multi.timeout_ms") == float("inf")
    finally:
        art.set_option(None, 0)


@pytest.mark.parametrize("name,value", [("no.such.option", 1), ("compile.world_merge", 3), ("compile.hoist", 0.5),
                                        ("bvh.sah_leaf", 0), ("bvh.sah_ci", -1), ("test.fault_rccl_group", 7)])
def test_options_refuse_unknown_names_and_out_of_range_values(name, value):
    before = {n: art.get_option(n) for n in OPTIONS}
    with pytest.raises(art.RTError) as e:
        art.set_option(name, value)
    assert e.value.code == -1 and name in str(e.value)
    assert {n: art.get_option(n) for n in OPTIONS} == before  # a refused value changes nothing


def test_environment_knobs_no_longer_change_the_tree():
    # the r4 builder knobs were environment variables; now only rt_option_set changes the compiled scene (a stray
    # variable in an embedding application's environment is ignored)
    import sys
    code = ("import sys; sys.path.insert(0, {root!r}); import another_raytracer_amd as art; "
            "w = art.scene_manager().build('8'); print(w.info['bvh_nodes'], w.info['objects'])").format(root=ROOT)
    env = dict(os.environ, ART_WORLD_MERGE="0", ART_BVH_COLLAPSE="1", ART_HOIST="0", ART_SAH_LEAF="2", ART_CODE16="0",
               ART_FAULT_WORKSPACE_BYTES="1", ART_FAULT_GATHER_ABORT="1")
    plain = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True, timeout=300).stdout.split()
    knobs = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True, timeout=300).stdout.split()
    assert plain == knobs == ["566", "6"]
    art.set_option("compile.world_merge", 0)
    try:
        info = art.scene_manager().build("8").info
    finally:
        art.set_option("compile.world_merge", 2)
    assert info["objects"] > 6  # the option does take effect


@pytest.mark.parametrize("H,band_rows,bands", [(1080, 16, 1), (1080, 16, 8), (37, 4, 3), (5, 16, 4), (225, 8, 7)])
def test_band_partition_covers_every_row_once(H, band_rows, bands):
    from another_raytracer_amd.distributed import band_rows_of
    seen = []
    for b in range(bands):
        p = _lib.rt_params(width=8, height=H, spp=1, max_depth=1, band_rows=band_rows, band_count=bands, band_index=b)
        n = _lib.lib.rt_local_rows(ctypes.byref(p), None)
        rows = (ctypes.c_int32 * max(n, 1))()
        _lib.lib.rt_local_rows(ctypes.byref(p), rows)
        got = list(rows[:n])
        assert got == sorted(got) and got == band_rows_of(H, band_rows, bands, b)
        seen += got
    assert sorted(seen) == list(range(H))


def _scene():
    return art.scene_manager().build("c1")


def test_invalid_parameters_are_rejected_before_any_device_work():
    w = _scene()
    cam = _lib.rt_camera()
    st = _lib.rt_stats()
    for bad in (dict(width=1, height=10, spp=1), dict(width=10, height=10, spp=0), dict(width=10, height=10, spp=1, max_depth=-1),
                dict(width=10, height=10, spp=1, band_rows=0), dict(width=10, height=10, spp=1, band_count=2, band_index=2),
                dict(width=10, height=10, spp=1, fp_mode=7)):
        p = _lib.rt_params(max_depth=bad.pop("max_depth", 50), band_rows=bad.pop("band_rows", 1),
                           band_count=bad.pop("band_count", 1), band_index=bad.pop("band_index", 0), **bad)
        rc = _lib.lib.rt_render(w.objects._native, ctypes.byref(cam), ctypes.byref(p), None, None, ctypes.byref(st))
        assert rc == -1, bad  # RT_E_INVALID
        assert _lib.lib.rt_last_error()
    assert _lib.lib.rt_render(None, ctypes.byref(cam), None, None, None, None) == -1


def test_graph_builder_rejects_bad_ids():
    g = _lib.lib.rt_graph_new()
    try:
        assert _lib.lib.rt_mat_lambertian(g, 99) == -1
        assert b"texture" in _lib.lib.rt_last_error()
        assert _lib.lib.rt_obj_rect(g, 5, 0, 1, 0, 1, 0, 0) == -1
        out = ctypes.c_void_p()
        assert _lib.lib.rt_graph_compile(g, 0, ctypes.byref(out)) == -2  # empty world: "Invalid input scene!"
        assert b"Invalid input scene" in _lib.lib.rt_last_error()
    finally:
        _lib.lib.rt_graph_free(g)


def test_empty_world_returns_minus_one_like_engine_run(capsys):
    eng = art.engine(art.camera((0, 0, 0), (0, 0, -1), (0, 1, 0), 90, 2.0, 0, 10), width=8, height=4)
    eng.set_scene(art.hittable_list(), (0, 0, 0))
    assert eng.run(np.zeros((4, 8, 3), np.uint8)) == -1  # engine.h:32-36
    assert "Invalid input scene!" in capsys.readouterr().out


@pytest.mark.skipif(_lib.lib.rt_device_count() > 0, reason="checks the no-device failure path")
def test_render_without_a_device_fails_loudly():
    w = _scene()
    eng = art.engine(art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, 2.0, 0, 10), width=8, height=4, samples_per_pixel=1)
    eng.set_scene(w.objects, w.background)
    with pytest.raises(art.RTError, match="RT_E_DEVICE"):
        eng.run(np.zeros((4, 8, 3), np.uint8))


def test_adaptive_mode_rejects_off_grid_sizes_like_the_reference():
    """engine.h:178-179 throws std::logic_error off the 12-px grid: RT_E_INVALID here, before any device work."""
    w = _scene()
    cam = _lib.rt_camera()
    st = _lib.rt_stats()
    for kw in (dict(width=50, height=36), dict(width=48, height=30), dict(width=48, height=48, band_rows=8, band_count=2)):
        p = _lib.rt_params(spp=1, max_depth=50, band_rows=kw.pop("band_rows", kw["height"]), band_count=kw.pop("band_count", 1),
                           band_index=0, flags=_lib.RT_ADAPTIVE, **kw)
        assert _lib.lib.rt_render(w.objects._native, ctypes.byref(cam), ctypes.byref(p), None, None, ctypes.byref(st)) == -1
        assert b"big square" in _lib.lib.rt_last_error()
    acc = np.zeros((12, 24, 3), np.float64)
    p = _lib.rt_params(width=24, height=12, spp=1, max_depth=50, band_rows=12, band_count=1, band_index=0, flags=_lib.RT_ADAPTIVE)
    assert _lib.lib.rt_render(w.objects._native, ctypes.byref(cam), ctypes.byref(p), None, acc.ctypes.data_as(ctypes.c_void_p),
                              ctypes.byref(st)) == -1
    eng = art.engine(art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, 2.0, 0, 10), art.engine_mode.adaptive, width=50, height=36)
    eng.set_scene(w.objects, w.background)
    with pytest.raises(ValueError, match="big square"):
        eng.run(np.zeros((36, 50, 3), np.uint8))


def test_multi_entry_points_validate_without_a_gpu():
    # argument errors are reported before any device work; without a GPU the multi-GPU renderer fails loudly
    # (RT_E_DEVICE), it never falls back to anything
    import ctypes
    m = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    assert _lib.lib.rt_multi_create(b"c1", b"assets", devs, 0, ctypes.byref(m)) == -1
    assert _lib.lib.rt_multi_create(None, b"assets", devs, 1, ctypes.byref(m)) == -1
    assert _lib.lib.rt_multi_create(b"no_such_scene", b"assets", devs, 1, ctypes.byref(m)) == -2
    if not torch_has_gpu():
        assert _lib.lib.rt_multi_create(b"c1", b"assets", devs, 1, ctypes.byref(m)) == -3
        assert m.value is None
    assert _lib.lib.rt_render_multi(None, None, None, None, None) == -1
    assert _lib.lib.rt_multi_times_get(None, None) == -1


def torch_has_gpu():
    import torch
    return torch.cuda.device_count() > 0
