"""Worker of tests/test_gpu_distributed.py (run under torch.distributed.run, one GPU shared by every rank): renders
this rank's row bands with libart on cuda:0 (render_frame's band partition) and gathers them to rank 0 with
gather_frame over a gloo group (CPU tensors: RCCL needs one GPU per rank).  Rank 0 writes the frame to argv[1]."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import another_raytracer_amd as art  # noqa: E402
from another_raytracer_amd.distributed import band_rows_of, block_rows, gather_frame  # noqa: E402

SCENE, W, H, SPP, BAND = "8", 96, 54, 4, 8


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    w = art.scene_manager().build(SCENE)
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, W / H, w.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.parallel_stripes, width=W, height=H, samples_per_pixel=SPP)
    eng.set_scene(w.objects, w.background)
    rows = band_rows_of(H, BAND, world, rank)
    send = torch.zeros((block_rows(H, BAND, world), W, 3), dtype=torch.uint8, device="cuda:0")  # padded gather block
    if rows:
        eng.run(send[: len(rows)], band_rows=BAND, band_count=world, band_index=rank)
    frame = gather_frame(send.cpu(), H, BAND)
    if rank == 0:
        np.save(sys.argv[1], frame.numpy())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
