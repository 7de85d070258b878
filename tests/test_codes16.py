"""layout.h's 16-bit child codes (the packed-key traversal of the k_paths_g F_CODE16 kernels, BvhNode::pad): round trip
and ordering against kNodeEmpty, on the host (tests/native/codes16_check.cpp, g++).  The device derives the codes from
the 32-bit ones at upload (kernels.hip build_device_scene) and the GPU parity suite renders every scene through them."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_leaf16_codes_round_trip(tmp_path):
    exe = tmp_path / "codes16_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "another_raytracer_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "codes16_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip() == f"ok {4 * 8192 - 1}"
