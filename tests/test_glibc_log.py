"""csrc/glibc_log.h (the renderer's restatement of glibc's log, hit_medium's log(random_double()) of
constant_medium.h:61) against the C library's own log, on the host: every value a uniform draw takes (k * 2^-24,
k < 2^24) and a million random positive normal doubles, bit for bit.  The device runs the same source
(tools/log_check compares it there: profiles/r2_log_check.json).  CPU only: builds tests/native/glibc_log_check.cpp
with g++.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_restated_log_equals_glibc(tmp_path):
    from tests.test_glibc_trig import libm_pin
    why = libm_pin("glibc_log_data.h")  # the same pin as the acos / atan2 restatement
    if why:
        pytest.skip(why)
    exe = tmp_path / "glibc_log_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "another_raytracer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "glibc_log_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "1000000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith(f"mismatches 0 of {(1 << 24) + 1000000}")


def test_generated_data_matches_this_libm():
    """The header's constants are the ones this image's libm holds (regenerating changes nothing)."""
    libm = "/lib/x86_64-linux-gnu/libm.so.6"
    if not os.path.exists(libm) or shutil.which("objdump") is None:
        pytest.skip("no libm.so.6 / objdump")
    import hashlib
    digest = hashlib.sha256(open(libm, "rb").read()).hexdigest()[:16]
    head = open(os.path.join(ROOT, "another_raytracer_amd", "csrc", "glibc_log_data.h")).read()
    if digest not in head:
        pytest.skip("another libm build than the one the header was generated from")
    assert "kLn2hi = 0x1.62e42fefa3800p-1" in head
