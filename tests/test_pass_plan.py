"""pass_plan.h's path_chunk -- how many path slots a persistent kernel's wave claims per atomic on the pass counter
(kernels.hip k_paths / k_paths_g; r4r_ab_path_chunk.txt) -- built with g++ and checked on the host: its values at the
BASELINE configs' pass sizes and its invariants (a power of two in [64, 2048], monotone in the pass size, at least 64
claims per wave of a full CU above the minimum)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_path_chunk(tmp_path):
    exe = tmp_path / "pass_plan_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "another_raytracer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "pass_plan_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout
