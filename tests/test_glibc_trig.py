"""csrc/glibc_trig.h (the renderer's restatement of glibc 2.35's acos and atan2, get_sphere_uv's acos(-y) and
atan2(-z, x) of sphere.h:24-37) against the C library's own functions, on the host, bit for bit: uniform unit vectors
(the arguments get_sphere_uv passes), every acos interval, every atan2 octant and |y / x| band, the special values
(signed zeros, infinities, NaNs, subnormals, |x| = 1) and random doubles of every exponent.  The device runs the same
source (tools/uv_check compares it there).  CPU only: builds tests/native/glibc_trig_check.cpp with g++.
"""
import hashlib
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBM = "/lib/x86_64-linux-gnu/libm.so.6"
N = 4_000_000  # per set; the checker runs 9.5 N + 462 calls of each side (~4 s)


def libm_pin(header="glibc_trig_data.h"):
    """Why the host's libm is not the build the restatement follows (None when it is): glibc_trig.h / glibc_log.h
    restate glibc 2.35's x86-64 FMA / AVX2 ifunc variants with tables read from one libm.so.6 (the hash in the generated
    header).  Another glibc, or a CPU without FMA / AVX2 (glibc's ifunc then selects its generic build, whose last bits
    can differ), is a different reference: the bit-exact comparison does not apply there."""
    if not os.path.exists(LIBM):
        return "no " + LIBM
    digest = hashlib.sha256(open(LIBM, "rb").read()).hexdigest()[:16]
    if digest not in open(os.path.join(ROOT, "another_raytracer_amd", "csrc", header)).read():
        return f"libm sha256 {digest} is not the build {header} was generated from"
    flags = set()
    if os.path.exists("/proc/cpuinfo"):
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    if not {"fma", "avx2"} <= flags:
        return "CPU without FMA / AVX2: glibc selects its generic acos / atan2 / log"
    return None


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_restated_acos_atan2_equal_glibc(tmp_path):
    why = libm_pin()
    if why:
        pytest.skip(why)
    exe = tmp_path / "glibc_trig_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "another_raytracer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "glibc_trig_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(N)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith(f"mismatches 0 of {N * 19 // 2 + 462}"), out.stdout


def test_generated_data_matches_this_libm(tmp_path):
    """The header is what tools/gen_glibc_trig.py reads from this image's libm (regenerating changes nothing)."""
    if not os.path.exists(LIBM) or shutil.which("objdump") is None:
        pytest.skip("no libm.so.6 / objdump")
    digest = hashlib.sha256(open(LIBM, "rb").read()).hexdigest()[:16]
    path = os.path.join(ROOT, "another_raytracer_amd", "csrc", "glibc_trig_data.h")
    head = open(path).read()
    if digest not in head:
        pytest.skip("another libm build than the one the header was generated from")
    out = tmp_path / "glibc_trig_data.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_glibc_trig.py"), LIBM, str(out)], check=True,
                   capture_output=True)
    assert out.read_text() == head
