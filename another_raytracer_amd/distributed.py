"""Multi-GPU frame rendering, two drivers of the same partition (row-interleaved bands, one RCCL gather):

* one process per GPU (torch.distributed over RCCL; bench.py under torchrun): render_frame / gather_frame below;
* one process, one host thread per GPU, RCCL inside libart (rt_render_multi, include/art.h): multi_engine below.


The reference splits an image into 4 contiguous row stripes on 4 threads (engine.h:335-376).  Here rank r of N
renders every global row y with (y // band_rows) % N == r (band_rows = 8: sky rows are cheap and object rows
expensive, so interleaving balances the load; 8-row bands keep the kernels' 8x8 pixel tiles on 8 consecutive image
rows, and split 1080 rows over 8 GPUs as 136/135 rows where 16-row bands gave 144/128), packs its rows contiguously, and rank 0 gathers the packed RGB8
blocks (RCCL over xGMI; the only collective of the path) and un-interleaves them.  Every pixel's RNG stream is keyed
by (seed, global pixel, sample), so the gathered image is bit-identical to a single-GPU render (tests/).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from ._lib import RT_OUT_DEVICE, check, lib, rt_params, rt_stats

DEFAULT_BAND_ROWS = 8


def band_rows_of(height, band_rows, band_count, band_index):
    """Global row indices owned by one band partition: libart's own rule (rt_local_rows, the kernels' global_row)."""
    p = rt_params()
    p.width, p.height = 2, int(height)
    p.band_rows, p.band_count, p.band_index = int(band_rows), int(band_count), int(band_index)
    n = check(lib.rt_local_rows(ctypes.byref(p), None), "rt_local_rows")
    rows = (ctypes.c_int32 * max(n, 1))()
    lib.rt_local_rows(ctypes.byref(p), rows)
    return list(rows[:n])


def gather_frame(local, height, band_rows, group=None, dst=0):
    """Gather each rank's packed rows (tensor [rows_r, W, C]) to `dst` and place them; returns the [H, W, C] frame on
    dst (None elsewhere).  Blocks are padded to the largest band so the collective moves equal-sized buffers."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    width, chans = local.shape[1], local.shape[2]
    max_rows = max(len(band_rows_of(height, band_rows, world, r)) for r in range(world))
    send = torch.zeros((max_rows, width, chans), dtype=local.dtype, device=local.device)
    send[: local.shape[0]] = local
    if world == 1:
        return local.clone()
    gather_list = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list, dst=dst, group=group)
    if rank != dst:
        return None
    frame = torch.empty((height, width, chans), dtype=local.dtype, device=local.device)
    for r in range(world):
        rows = band_rows_of(height, band_rows, world, r)
        if rows:
            idx = torch.tensor(rows, device=local.device, dtype=torch.long)
            frame.index_copy_(0, idx, gather_list[r][: len(rows)])
    return frame


def render_frame(eng, band_rows=DEFAULT_BAND_ROWS, group=None, dst=0, device=None, profile=False, out_local=None):
    """Renders `eng`'s frame across all ranks of `group` and gathers it on `dst`.  Returns (frame_or_None, stats)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    rows = band_rows_of(eng.height, band_rows, world, rank)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    local = out_local if out_local is not None else torch.empty((len(rows), eng.width, 3), dtype=torch.uint8, device=dev)
    if rows:
        eng.run(local, band_rows=band_rows, band_count=world, band_index=rank, profile=profile)
    stats = dict(eng.stats)
    if world == 1:
        return local, stats
    return gather_frame(local, eng.height, band_rows, group=group, dst=dst), stats


class multi_engine:
    """The engine surface over rt_render_multi: one process drives `devices` (one host thread and one RCCL rank per
    GPU), each GPU renders the bands b with b % len(devices) == its index, and one ncclGather assembles the frame on
    devices[0].  `scene` is a builtin scene name (scene_manager names) or a hittable_list built in Python."""

    def __init__(self, scene, devices, cam, width, height, samples_per_pixel, max_depth=50, seed=0,
                 band_rows=DEFAULT_BAND_ROWS, background=None, asset_dir=None):
        from .scene import ASSET_DIR, _g
        self.devices = [int(d) for d in devices]
        self.cam, self.width, self.height = cam, int(width), int(height)
        self.samples_per_pixel, self.max_depth, self.seed, self.band_rows = int(samples_per_pixel), int(max_depth), int(seed), int(band_rows)
        devs = (ctypes.c_int * len(self.devices))(*self.devices)
        self._m = ctypes.c_void_p()
        if isinstance(scene, str):
            check(lib.rt_multi_create(scene.encode(), (asset_dir or ASSET_DIR).encode(), devs, len(self.devices),
                                      ctypes.byref(self._m)), "rt_multi_create")
        else:
            g = _g()
            check(lib.rt_graph_clear_world(g), "rt_graph_clear_world")
            for o in scene.objects:
                check(lib.rt_graph_add_world(g, o.id), "rt_graph_add_world")
            check(lib.rt_multi_from_graph(g, devs, len(self.devices), ctypes.byref(self._m)), "rt_multi_from_graph")
        self.background = tuple(background) if background is not None else (0.0, 0.0, 0.0)
        self.stats = {}

    def run(self, out):
        """Renders the whole frame into `out` (uint8 H x W x 3: numpy, or a torch tensor on devices[0]); returns ms."""
        from .engine import _pointer
        p = rt_params()
        p.width, p.height, p.spp, p.max_depth, p.seed = self.width, self.height, self.samples_per_pixel, self.max_depth, self.seed
        p.band_rows, p.band_count, p.band_index = self.band_rows, 1, 0
        for c in range(3):
            p.background[c] = self.background[c]
        ptr, dev = _pointer(out, self.width * self.height * 3)
        if dev:
            p.flags |= RT_OUT_DEVICE
        st = rt_stats()
        check(lib.rt_render_multi(self._m, ctypes.byref(self.cam.c), ctypes.byref(p), ctypes.c_void_p(ptr), ctypes.byref(st)),
              "rt_render_multi")
        self.stats = st.as_dict()
        return st.ms

    def __del__(self):
        if getattr(self, "_m", None) and self._m.value and lib is not None:
            lib.rt_multi_destroy(self._m)
            self._m = None
