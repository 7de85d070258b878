"""PMC summaries are stamped with the device code they measured (another_raytracer_amd._lib.kernel_build_id: SHA-256 of
libart.so's .hip_fatbin section) and bench.py prices a run only with a summary of the same build (CPU)."""
import hashlib
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

OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"


def test_build_id_is_the_fatbin_hash(tmp_path):
    bid = _lib.kernel_build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0
    if not os.path.exists(OBJCOPY):
        pytest.skip("llvm-objcopy not in this image")
    out = tmp_path / "fatbin"
    subprocess.run([OBJCOPY, f"--dump-section=.hip_fatbin={out}", _lib.LIB_PATH, str(tmp_path / "copy.so")], check=True)
    assert hashlib.sha256(out.read_bytes()).hexdigest()[:16] == bid


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
