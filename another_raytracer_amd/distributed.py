"""Multi-GPU frame rendering, two drivers of the same partition (row-interleaved bands, one RCCL gather):

* one process per GPU (torch.distributed over RCCL; bench.py under torchrun): frame_renderer / gather_frame below --
  each rank renders its bands into its padded gather block, one dist.gather moves the blocks, and libart's
  rt_unpack_bands places the rows (the same layout and unpack kernel as rt_render_multi);
* one process, one host thread per GPU, RCCL inside libart (rt_render_multi, include/art.h): multi_engine below.


The reference splits an image into 4 contiguous row stripes on 4 threads (engine.h:335-376).  Here rank r of N
renders every global row y with (y // band_rows) % N == r (band_rows = 8: sky rows are cheap and object rows
expensive, so interleaving balances the load; 8-row bands keep the kernels' 8x8 pixel tiles on 8 consecutive image
rows, and split 1080 rows over 8 GPUs as seven ranks of 136 rows and one of 128, where 16-row bands gave 144/128), packs its rows contiguously, and rank 0 gathers the packed RGB8
blocks (RCCL over xGMI; the only collective of the path) and un-interleaves them.  Every pixel's RNG stream is keyed
by (seed, global pixel, sample), so the gathered image is bit-identical to a single-GPU render (tests/).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from ._lib import RT_OUT_DEVICE, RT_PROFILE, check, lib, rt_multi_times, rt_params, rt_stats

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


def block_rows(height, band_rows, world):
    """Rows of every rank's gather block: the largest band set's row count (libart's rt_band_block_rows)."""
    return check(lib.rt_band_block_rows(int(height), int(band_rows), int(world)), "rt_band_block_rows")


def unpack_bands(packed, frame, height, band_rows, world, stream=None):
    """Places `world` concatenated band blocks (packed: [world * block_rows, W, 3] uint8) into frame [H, W, 3]: libart's
    rt_unpack_bands, the same code rt_render_multi runs after its ncclGather (a kernel on the tensors' device, on
    `stream` or torch's current stream; numpy arrays are unpacked on the host).  Both shapes are checked against the
    layout here, and rt_unpack_bands refuses buffers whose byte sizes do not match it."""
    width = int(frame.shape[1])
    block = block_rows(height, band_rows, world)
    if tuple(packed.shape) != (int(world) * block, width, 3):
        raise ValueError(f"packed has shape {tuple(packed.shape)}, the {world}-way layout needs ({int(world) * block}, {width}, 3)")
    if tuple(frame.shape) != (int(height), width, 3):
        raise ValueError(f"frame has shape {tuple(frame.shape)}, expected ({int(height)}, {width}, 3)")
    nbytes = lambda a: a.numel() * a.element_size() if isinstance(a, torch.Tensor) else a.nbytes
    pbytes, fbytes = nbytes(packed), nbytes(frame)
    if isinstance(packed, torch.Tensor):
        assert packed.is_contiguous() and frame.is_contiguous() and packed.dtype == torch.uint8 and frame.dtype == torch.uint8
        if packed.is_cuda:
            assert frame.is_cuda and frame.device == packed.device, "packed and frame must be on one device"
            st = stream if stream is not None else torch.cuda.current_stream(packed.device).cuda_stream
            check(lib.rt_unpack_bands(ctypes.c_void_p(packed.data_ptr()), pbytes, ctypes.c_void_p(frame.data_ptr()), fbytes, width,
                                      int(height), int(band_rows), int(world), RT_OUT_DEVICE, ctypes.c_void_p(st)), "rt_unpack_bands")
            return frame
        packed, frame_np = packed.numpy(), frame.numpy()
    else:
        frame_np = frame
    assert packed.flags.c_contiguous and frame_np.flags.c_contiguous and packed.dtype == np.uint8 and frame_np.dtype == np.uint8
    check(lib.rt_unpack_bands(packed.ctypes.data_as(ctypes.c_void_p), pbytes, frame_np.ctypes.data_as(ctypes.c_void_p), fbytes, width,
                              int(height), int(band_rows), int(world), 0, None), "rt_unpack_bands")
    return frame


def gather_frame(send, height, band_rows, group=None, dst=0, recv=None, frame=None):
    """Gathers every rank's padded block `send` ([block_rows, W, C]: its band rows first, as rendered in place by
    render_frame) to `dst` with one collective (RCCL on GPUs, gloo on CPU), then places the rows with rt_unpack_bands.
    Returns the [H, W, C] frame on dst (None elsewhere).  A `send` that is not exactly one padded block is refused on
    every rank before the collective (the unpadded [rows_r, W, C] form of ABI 3 included): each rank checks its own
    block, and the layout is the same on every rank.  A wrong `recv` or `frame` exists on dst alone, where the peers
    may already be inside the collective: dst then still joins it with a correctly sized buffer of its own and raises
    once the collective has completed, so no peer is left blocked in dist.gather."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    block = block_rows(height, band_rows, world)
    if send.dim() != 3 or send.shape[0] != block:
        raise ValueError(f"send must be this rank's padded gather block of {block} rows (block_rows({height}, {band_rows}, {world})), "
                         f"got shape {tuple(send.shape)}")
    if rank != dst:
        dist.gather(send, None, dst=dst, group=group)
        return None
    width, chans = send.shape[1], send.shape[2]
    bad = None
    if recv is not None and (tuple(recv.shape) != (world * block, width, chans) or recv.dtype != send.dtype or recv.device != send.device
                             or not recv.is_contiguous()):
        bad = ValueError(f"recv must be one contiguous {send.dtype} buffer of {world} blocks of {block} rows on {send.device}, "
                         f"got shape {tuple(recv.shape)} {recv.dtype} on {recv.device}")
        recv = None
    if frame is not None and (tuple(frame.shape) != (int(height), width, chans) or frame.dtype != send.dtype):
        bad = bad or ValueError(f"frame must have shape {(int(height), width, chans)} and dtype {send.dtype}, got {tuple(frame.shape)} {frame.dtype}")
    if recv is None:
        recv = torch.empty((world * block, width, chans), dtype=send.dtype, device=send.device)
    dist.gather(send, list(recv.chunk(world)), dst=dst, group=group)  # views of one contiguous buffer
    if bad is not None:  # raised only now: every peer's gather has completed
        raise bad
    if frame is None:
        frame = torch.empty((height, width, chans), dtype=send.dtype, device=send.device)
    return unpack_bands(recv, frame, height, band_rows, world)


class frame_renderer:
    """One rank's share of a multi-process frame (one process per GPU): renders its bands straight into its padded
    gather block and gathers on `dst` (the buffers are allocated once, so a step allocates nothing)."""

    def __init__(self, eng, band_rows=DEFAULT_BAND_ROWS, group=None, dst=0, device=None):
        self.eng, self.band_rows, self.group, self.dst = eng, int(band_rows), group, dst
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.rows = band_rows_of(eng.height, self.band_rows, self.world, self.rank)
        self.block = block_rows(eng.height, self.band_rows, self.world)
        self.send = torch.zeros((self.block, eng.width, 3), dtype=torch.uint8, device=self.device)
        self.recv = self.frame = None
        if self.world > 1 and self.rank == dst:
            self.recv = torch.empty((self.world * self.block, eng.width, 3), dtype=torch.uint8, device=self.device)
            self.frame = torch.empty((eng.height, eng.width, 3), dtype=torch.uint8, device=self.device)

    def __call__(self, profile=False):
        """Returns (frame on dst / None elsewhere, this rank's render stats)."""
        if self.rows:
            self.eng.run(self.send[: len(self.rows)], band_rows=self.band_rows, band_count=self.world, band_index=self.rank,
                         profile=profile)
            stats = dict(self.eng.stats)
        else:
            stats = {"segments": 0, "primary": 0, "ms": 0.0, "extend_ms": 0.0, "shade_ms": 0.0, "extend_launches": 0,
                     "shade_launches": 0, "passes": 0, "samples_per_pass": 0, "local_rows": 0, "extend_variant": -1,
                     "kernel_features": 0, "kernel_textures": 0, "kernel_lds_mode": -1}
        if self.world == 1:
            return self.send, stats
        return gather_frame(self.send, self.eng.height, self.band_rows, self.group, self.dst, self.recv, self.frame), stats


def render_frame(eng, band_rows=DEFAULT_BAND_ROWS, group=None, dst=0, device=None, profile=False):
    """Renders `eng`'s frame across all ranks of `group` and gathers it on `dst`.  Returns (frame_or_None, stats)."""
    return frame_renderer(eng, band_rows, group, dst, device)(profile=profile)


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
        self.info = self.scene_info()
        # engine::set_scene(world, background) (engine.h:24-28): a builtin scene's own background unless overridden
        self.background = tuple(background) if background is not None else (
            tuple(self.info["background"]) if isinstance(scene, str) else (0.0, 0.0, 0.0))
        self.stats = {}

    def run(self, out, profile=False):
        """Renders the whole frame into `out` (uint8 H x W x 3: numpy, or a torch tensor on devices[0]); returns ms.
        profile: time every path-kernel launch with HIP events (stats extend_ms; per device in device_stats)."""
        from .engine import _pointer
        if isinstance(out, torch.Tensor) and out.is_cuda and out.device.index != self.devices[0]:
            raise ValueError(f"a device output must live on devices[0] = cuda:{self.devices[0]}, not {out.device}")
        p = rt_params()
        p.width, p.height, p.spp, p.max_depth, p.seed = self.width, self.height, self.samples_per_pixel, self.max_depth, self.seed
        p.band_rows, p.band_count, p.band_index = self.band_rows, 1, 0
        for c in range(3):
            p.background[c] = self.background[c]
        ptr, dev = _pointer(out, self.width * self.height * 3)
        if dev:
            p.flags |= RT_OUT_DEVICE
        if profile:
            p.flags |= RT_PROFILE
        st = rt_stats()
        check(lib.rt_render_multi(self._m, ctypes.byref(self.cam.c), ctypes.byref(p), ctypes.c_void_p(ptr), ctypes.byref(st)),
              "rt_render_multi")
        self.stats = st.as_dict()
        return st.ms

    def scene_info(self):
        """rt_multi_scene_info: the scene_manager view and sizes (device_bytes_f64: uploaded on each device at creation)."""
        from ._lib import rt_scene_info
        info = rt_scene_info()
        check(lib.rt_multi_scene_info(self._m, ctypes.byref(info)), "rt_multi_scene_info")
        return {f: (tuple(getattr(info, f)) if isinstance(getattr(info, f), ctypes.Array) else getattr(info, f)) for f, _ in info._fields_}

    def device_stats(self):
        """Per-device stats of the last run (devices[k] at index k): segments, kernel time, rows."""
        out = []
        for k in range(len(self.devices)):
            st = rt_stats()
            check(lib.rt_multi_device_stats(self._m, k, ctypes.byref(st)), "rt_multi_device_stats")
            out.append(st.as_dict())
        return out

    def times(self):
        """rt_multi_times of the last run: renders (slowest / fastest device), gather, unpack, collectives issued."""
        t = rt_multi_times()
        check(lib.rt_multi_times_get(self._m, ctypes.byref(t)), "rt_multi_times_get")
        return t.as_dict()

    def __del__(self):
        if getattr(self, "_m", None) and self._m.value and lib is not None:
            lib.rt_multi_destroy(self._m)
            self._m = None
