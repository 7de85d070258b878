"""get_sphere_uv (sphere.h:24-37) as the product computes it: csrc/sphere_uv.h (glibc 2.35's acos / atan2 restated in
glibc_trig.h, one code for host and device) against glibc's acos / atan2, the reference's libm.
tests/native/sphere_uv_check.cpp is built with g++ here and run over 2^20 uniform unit normals and 2^20 normals placed
on the earth texture's texel edges (1024 x 512, scene_manager.cpp:117) nudged by -4..+4 ulps.

The bar ("sphere u, v"): every acos / atan2 result, every u and v, and so every texel choice equals the
reference's, including the exact cases (signed zeros, poles, infinities, huge y / x).  tools/uv_check.hip checks on the
GPU that the device computes the host's bits over 2^24 normals of each kind."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "sphere_uv_check.cpp")
CSRC = os.path.join(ROOT, "another_raytracer_amd", "csrc")


@pytest.fixture(scope="module")
def report(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("uv") / "sphere_uv_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I", CSRC, SRC, "-o", exe], check=True)
    out = subprocess.run([exe, str(1 << 20)], check=True, capture_output=True, text=True).stdout
    rows = {}
    for line in out.splitlines():
        key, rest = line.split(" ", 1)
        rows[key] = {k: int(v) for k, v in re.findall(r"(\w+)[ =](\d+)", rest)}
    return rows


def test_acos_atan2_bits_equal_glibc(report):
    assert report["max_ulp"]["acos"] == 0 and report["max_ulp"]["atan2"] == 0, report["max_ulp"]
    for s in ("random", "adversarial"):
        assert report[s]["n"] == 1 << 20
        assert report[s]["acos_differs"] == 0 and report[s]["atan2_differs"] == 0, report[s]


def test_exact_cases_agree_bit_for_bit(report):
    assert report["special"]["n"] > 150
    assert report["special"]["differs"] == 0, report["special"]


@pytest.mark.parametrize("normals", ["random", "adversarial"])
def test_u_v_and_texel_equal_the_reference(report, normals):
    # the adversarial set puts every normal within 4 ulps of a texel edge: any last-bit difference would flip texels
    r = report[normals]
    assert r["u_bits_differ"] == 0 and r["v_bits_differ"] == 0 and r["texel_differs"] == 0, r
