"""The multi-GPU partition and gather layout (include/art.h rt_local_rows / rt_band_block_rows / rt_unpack_bands, the
rules rt_render_multi's ncclGather and unpack kernel use: csrc/multi.hip, csrc/layout.h band_*), on the CPU for
N = 1..8 ranks, band heights 1..16 and frame heights that do not divide into band_rows x N.  The reference's
ancestor is _run_parallel_stripes' 4 contiguous stripes (engine.h:335-376); here band b of band_rows rows belongs to
rank b % N."""
import ctypes

import numpy as np
import pytest

from another_raytracer_amd import _lib
from another_raytracer_amd.distributed import band_rows_of, block_rows, unpack_bands

HEIGHTS = [1, 2, 7, 8, 9, 37, 135, 1080, 1081, 4096]


def _rows_py(H, band_rows, n, r):
    """Restatement: every global row y with (y // band_rows) % n == r, in increasing order."""
    return [y for y in range(H) if (y // band_rows) % n == r]


@pytest.mark.parametrize("n", range(1, 9))
@pytest.mark.parametrize("band_rows", [1, 3, 8, 16])
def test_partition_covers_every_row_once(n, band_rows):
    for H in HEIGHTS:
        sets = [band_rows_of(H, band_rows, n, r) for r in range(n)]
        for r in range(n):
            assert sets[r] == _rows_py(H, band_rows, n, r), (H, band_rows, n, r)
        assert sorted(y for s in sets for y in s) == list(range(H))
        assert block_rows(H, band_rows, n) == max(len(s) for s in sets)


@pytest.mark.parametrize("n", range(1, 9))
def test_unpack_rebuilds_the_frame(n):
    rng = np.random.default_rng(n)
    for H in (1, 9, 37, 135, 1081):
        for band_rows in (1, 7, 8):
            W = 5 + n  # odd row byte counts too (the device kernel's narrow path)
            frame = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
            blk = block_rows(H, band_rows, n)
            packed = np.full((n * blk, W, 3), 0xAB, np.uint8)  # padding rows hold garbage
            for r in range(n):
                rows = band_rows_of(H, band_rows, n, r)
                packed[r * blk: r * blk + len(rows)] = frame[rows]
            out = np.zeros_like(frame)
            unpack_bands(packed, out, H, band_rows, n)
            assert np.array_equal(out, frame), (H, band_rows, n)


def test_1080p_over_8_gpus_is_balanced():
    # 8-row bands split 1080 rows (135 bands) over 8 GPUs as seven ranks of 136 rows and one of 128
    sizes = [len(band_rows_of(1080, 8, 8, r)) for r in range(8)]
    assert sizes == [136] * 7 + [128] and sum(sizes) == 1080
    assert block_rows(1080, 8, 8) == max(sizes) == 136


def test_bad_arguments_are_refused():
    assert _lib.lib.rt_band_block_rows(0, 8, 2) == -1 and _lib.lib.rt_band_block_rows(10, 0, 2) < 0 and _lib.lib.rt_band_block_rows(10, 8, 0) < 0
    buf = (ctypes.c_uint8 * 12)()
    assert _lib.lib.rt_unpack_bands(None, 12, buf, 12, 2, 2, 1, 1, 0, None) < 0
    assert _lib.lib.rt_unpack_bands(buf, 12, buf, 12, 2, 2, 0, 1, 0, None) < 0


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_unpack_refuses_buffers_that_do_not_match_the_layout(n):
    # rt_unpack_bands reads n * block_rows rows of `packed` and writes H rows of `frame`: a buffer of any other size is
    # refused (RT_E_INVALID) before a byte moves, so a caller passing ABI 3's unpadded block cannot over-read
    H, W, band_rows = 37, 5, 4
    blk = block_rows(H, band_rows, n)
    packed = np.zeros((n * blk, W, 3), np.uint8)
    frame = np.zeros((H, W, 3), np.uint8)
    pp, fp = packed.ctypes.data_as(ctypes.c_void_p), frame.ctypes.data_as(ctypes.c_void_p)
    assert _lib.lib.rt_unpack_bands(pp, packed.nbytes, fp, frame.nbytes, W, H, band_rows, n, 0, None) == 0
    for pb, fb in ((packed.nbytes - W * 3, frame.nbytes), (packed.nbytes + 1, frame.nbytes), (packed.nbytes, frame.nbytes - 3),
                   (0, frame.nbytes)):
        assert _lib.lib.rt_unpack_bands(pp, pb, fp, fb, W, H, band_rows, n, 0, None) == -1
        assert b"bytes" in _lib.lib.rt_last_error()
    with pytest.raises(ValueError, match="layout needs"):
        unpack_bands(packed[: n * blk - 1], frame, H, band_rows, n)
    with pytest.raises(ValueError, match="frame has shape"):
        unpack_bands(packed, frame[:-1], H, band_rows, n)
