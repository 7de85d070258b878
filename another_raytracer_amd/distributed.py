"""Multi-GPU frame rendering: one process per GPU (torch.distributed over RCCL), row-interleaved bands, one gather.

The reference splits an image into 4 contiguous row stripes on 4 threads (engine.h:335-376).  Here rank r of N
renders every global row y with (y // band_rows) % N == r (band_rows = 16: sky rows are cheap and object rows
expensive, so interleaving balances the load), packs its rows contiguously, and rank 0 gathers the packed RGB8
blocks (RCCL over xGMI; the only collective of the path) and un-interleaves them.  Every pixel's RNG stream is keyed
by (seed, global pixel, sample), so the gathered image is bit-identical to a single-GPU render (tests/).
"""
import torch
import torch.distributed as dist

DEFAULT_BAND_ROWS = 16


def band_rows_of(height, band_rows, band_count, band_index):
    """Global row indices owned by one band partition (same rule as rt_local_rows / kernels.hip global_row)."""
    rows = []
    ly = 0
    while True:
        gy = (ly // band_rows) * (band_rows * band_count) + band_index * band_rows + (ly % band_rows)
        if gy >= height:
            return rows
        rows.append(gy)
        ly += 1


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
