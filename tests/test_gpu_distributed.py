"""The one-process-per-GPU driver (distributed.py: band partition + gather_frame, what bench.py --gpus N runs under
torchrun) with libart renders: 2 and 3 ranks share the one GPU of the box, render their row bands on it and gather
over gloo (RCCL needs a GPU per rank; rt_render_multi's RCCL path is tested in test_gpu_api.py).  Rank 0's frame must
equal a single-process render bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import another_raytracer_amd as art
from tests.dist_render_worker import BAND, H, SCENE, SPP, W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_on_libart_rebuild_the_single_gpu_frame(gpu, world, tmp_path):
    out = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_port()}", os.path.join(ROOT, "tests", "dist_render_worker.py"), str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    w = art.scene_manager().build(SCENE)
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, W / H, w.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.parallel_stripes, width=W, height=H, samples_per_pixel=SPP)
    eng.set_scene(w.objects, w.background)
    ref = np.zeros((H, W, 3), np.uint8)
    eng.run(ref)
    assert np.array_equal(np.load(out), ref)
    assert BAND == 8


@pytest.mark.parametrize("n", range(1, 9))
def test_device_unpack_of_gathered_blocks(gpu, n):
    """What rank 0 runs after the RCCL gather of bench.py --gpus N under torchrun (gather_frame): unpack_bands on CUDA
    tensors (libart's unpack kernel on torch's stream) rebuilds the frame from the N padded blocks, padding rows ignored,
    for heights that do not divide into band_rows x N and odd row byte counts."""
    import torch
    from another_raytracer_amd.distributed import band_rows_of, block_rows, unpack_bands
    rng = np.random.default_rng(100 + n)
    for H, W, band_rows in ((1080, 1920, 8), (1081, 37, 8), (37, 5, 1), (9, 64, 7)):
        frame = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        blk = block_rows(H, band_rows, n)
        packed = np.full((n * blk, W, 3), 0xAB, np.uint8)
        for r in range(n):
            rows = band_rows_of(H, band_rows, n, r)
            packed[r * blk: r * blk + len(rows)] = frame[rows]
        out = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda:0")
        unpack_bands(torch.from_numpy(packed).to("cuda:0"), out, H, band_rows, n)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), frame), (H, W, band_rows, n)
