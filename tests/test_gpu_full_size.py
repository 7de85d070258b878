"""HIP path at the BASELINE.json configurations' full sizes and full sample counts vs the oracle — parity at scale.

The small-image parity tests (test_gpu_parity.py) cover every scene at 64x36.  Here, for each GPU config (C2 random
spheres 1920x1080x1024, C3 cow 1920x1080x512, C4 Next-Week final 1920x1080x4096, C5 dino 4096x4096x8192):
  1. the GPU renders the WHOLE frame at the config's own spp (C5 on one GPU: 64 passes of 2^31 path slots);
  2. the GPU renders the row-interleaved band partition that holds exactly every `stride`-th row (band_rows 1,
     band_count stride, band_index 0: rows 0, stride, 2*stride, ...) -- the same kernels, counting the segments of
     just those rows;
  3. the oracle (oracle/restate.cpp pcg mode: the same PCG streams and f64 operation order) renders the same rows,
     spread over the host threads in (row, 64-px chunk) work items.
Asserted, bit for bit: the full frame's sampled rows == the band render (RGB8 and f64 radiance sums), the band
render == the oracle rows (RGB8 and sums), and the band render's segment count == the oracle's.
  4. every config also checks the rows tests/golden/make_full_size.py aimed at the geometry (24 C2 rows through the
     three r = 1 spheres and the small static / moving spheres, 24 cow-silhouette rows, 16 rows through the Next-Week
     box field, fog sphere and sphere cluster, 48 dino rows = 1.2 % of C5's pixels) against the
     oracle's committed render of them: the whole frame's RGB8 and the SHA-256 of each row's f64 sums.
"""
import hashlib
import os

import numpy as np
import pytest

from tests.oracle_lib import oracle_render_rows
from tests.test_gpu_parity import gpu_render

pytestmark = pytest.mark.gpu

# (scene, W, H, spp, row stride): BASELINE.json configs[1..4] at their full resolution and spp
CONFIGS = [
    ("1", 1920, 1080, 1024, 64),
    ("cow", 1920, 1080, 512, 64),
    ("8", 1920, 1080, 4096, 135),
    ("dino", 4096, 4096, 8192, 1024),
]


def host_threads():
    """The box's CPU share (OMP_NUM_THREADS is set to it there), else at most 16."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() and int(env) > 0 else min(16, os.cpu_count() or 4)


@pytest.mark.parametrize("scene,W,H,spp,stride", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_full_size_frame_matches_oracle_rows(gpu, scene, W, H, spp, stride):
    rows = np.arange(0, H, stride)
    band = gpu_render(scene, W, H, spp, band=(1, stride, 0))
    assert np.array_equal(band["engine"].local_rows(1, stride, 0), rows)
    o = oracle_render_rows(scene, W, H, spp, rows, threads=host_threads())
    full = gpu_render(scene, W, H, spp)
    print(f"{scene} {W}x{H}x{spp}: frame segments {full['segments']} ({full['stats']['passes']} passes); rows {len(rows)} "
          f"segments {band['segments']} (oracle {o['segments']}, {o['ms'] / 1e3:.1f} s)")
    assert np.array_equal(full["rgb"][rows], band["rgb"]) and np.array_equal(full["acc"][rows], band["acc"])
    assert np.array_equal(band["rgb"], o["rgb"])
    assert np.array_equal(band["acc"], o["acc"])
    assert band["segments"] == o["segments"]
    fx = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"fullsize_{scene}.npz")
    if os.path.exists(fx):
        g = np.load(fx)
        assert (int(g["W"]), int(g["H"]), int(g["spp"])) == (W, H, spp)
        grows = g["rows"]
        assert np.array_equal(full["rgb"][grows], g["rgb"]), f"{scene}: aimed rows differ in RGB8"
        got = [hashlib.sha256(np.ascontiguousarray(full["acc"][r], dtype="<f8").tobytes()).hexdigest() for r in grows]
        bad = [int(r) for r, a, b in zip(grows, got, g["acc_sha256"]) if a != str(b)]
        assert not bad, f"{scene}: f64 sums differ on rows {bad}"
        print(f"{scene}: {len(grows)} aimed rows ({100.0 * len(grows) / H:.2f} % of the frame) equal the oracle's")
    else:
        raise AssertionError(f"missing fixture {fx}")
