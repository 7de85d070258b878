"""PMC summaries are stamped with the device code they measured (another_raytracer_amd._lib.kernel_build_id: SHA-256 of
the gfx950 code objects' .note/.rodata/.text in libart.so's .hip_fatbin) and bench.py prices a run only with a summary of
the same build (CPU)."""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from another_raytracer_amd import _lib  # noqa: E402

def test_build_id_does_not_depend_on_the_build_path(tmp_path):
    # the same sources built at another path (hipcc's __hip_cuid_* symbols are derived from it) give the same id, so
    # a PMC summary stays attached to the device code it measured wherever libart.so was built
    bid = _lib.kernel_build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0
    src = os.path.join(ROOT, "another_raytracer_amd", "csrc")
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not in this image")
    dst = tmp_path / "elsewhere" / "another_raytracer_amd" / "csrc"
    shutil.copytree(src, dst)
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "elsewhere" / "include")
    out = tmp_path / "elsewhere" / "libart.so"
    jobs = str(min(8, os.cpu_count() or 2))
    subprocess.run(["make", "-C", str(dst), "-j" + jobs, f"OUT={out}", f"OBJDIR={tmp_path / 'obj'}", str(out)], check=True,
                   capture_output=True, timeout=1200)
    assert _lib.kernel_build_id(str(out)) == bid


def test_build_id_refuses_non_elf(tmp_path):
    p = tmp_path / "x.so"
    p.write_bytes(b"not an elf file at all")
    with pytest.raises(ValueError):
        _lib.kernel_build_id(str(p))


def test_latest_pmc_only_matches_the_same_build(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"precision": "f64", "scene": "1", "extend_variant": 3, "dominant_kernel": "art::k_paths",
            "kernels": {"art::k_paths": {"per_segment_wave_instructions": {"insts_valu": 34.0}}}}
    json.dump({**base, "libart_build": "aaaaaaaaaaaaaaaa", "tag": "old"}, open(prof / "r9a_pmc_scene1_f64.json", "w"))
    json.dump({**base, "tag": "unstamped"}, open(prof / "r9b_pmc_scene1_f64.json", "w"))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.latest_pmc("f64", "1", 3, "bbbbbbbbbbbbbbbb") is None  # another build, and an unstamped summary
    got = bench.latest_pmc("f64", "1", 3, "aaaaaaaaaaaaaaaa")
    assert got is not None and got["tag"] == "old"
    assert bench.latest_pmc("f64", "cow", 3, "aaaaaaaaaaaaaaaa") is None  # another scene
