"""engine / camera surface of the reference (src/engine/engine.h, src/engine/camera.h), on libart.so.

`engine.run(out)` is the drop-in for engine<W,H,C>::run (engine.h:30-54): it renders every pixel with the
reference's sampling (`_stochastic_sample`, engine.h:58-68) and integrator (`_ray_color`, engine.h:447-466) on the
GPU and writes write_color's RGB8 (color.h:6-22) into `out`.  The reference's compile-time tracer_constants
(tracer_constants.h:6-14) are constructor arguments here.
"""
import ctypes
import enum

import numpy as np

from ._lib import RT_ADAPTIVE, RT_FP64, RT_PARALLEL_IMAGES, rt_progress_fn, RT_GLOBAL_SCENE, RT_OUT_DEVICE, RT_PROFILE, RT_SPLIT_SHADE, RT_WAVEFRONT, check, dvec, lib, rt_camera, rt_params, rt_stats
from .scene import compile_world


class tracer_constants:  # tracer_constants.h:6-14
    aspect_ratio = 4.0 / 3.0
    image_width = 720
    image_height = int(image_width / aspect_ratio)
    color_channels = 3
    samples_per_pixel = 100
    max_depth = 50


class engine_mode(enum.Enum):  # engine.h:10-16
    single = 0
    adaptive = 1
    parallel_stripes = 2
    parallel_images = 3


class camera:  # camera.h:8-36
    def __init__(self, lookfrom, lookat, vup, vfov, aspect_ratio, aperture, focus_dist, time0=0.0, time1=0.0):
        self.c = rt_camera(dvec(lookfrom), dvec(lookat), dvec(vup), float(vfov), float(aspect_ratio), float(aperture),
                           float(focus_dist), float(time0), float(time1))


def _pointer(out, nbytes):
    """(address, is_device) of a writable uint8 buffer: numpy array or torch tensor (CPU or CUDA/HIP)."""
    if isinstance(out, np.ndarray):
        if not out.flags.c_contiguous or out.dtype != np.uint8 or out.nbytes < nbytes:
            raise ValueError(f"output must be a C-contiguous uint8 array of >= {nbytes} bytes")
        return out.ctypes.data, False
    if hasattr(out, "data_ptr"):
        if not out.is_contiguous() or out.element_size() * out.numel() < nbytes:
            raise ValueError(f"output tensor must be contiguous with >= {nbytes} bytes")
        return out.data_ptr(), out.device.type != "cpu"
    raise TypeError("output must be a numpy array or a torch tensor")


class engine:
    """engine<W,H,C>(const camera&, engine_mode) (engine.h:19-476)."""

    def __init__(self, cam, mode=engine_mode.single, width=tracer_constants.image_width,
                 height=tracer_constants.image_height, samples_per_pixel=tracer_constants.samples_per_pixel,
                 max_depth=tracer_constants.max_depth, device=0, seed=0, precision="f64", samples_per_pass=0):
        self.cam, self.m = cam, mode
        self.width, self.height = int(width), int(height)
        self.samples_per_pixel, self.max_depth = int(samples_per_pixel), int(max_depth)
        self.device, self.seed = int(device), int(seed)
        if precision != "f64":
            raise ValueError("precision must be 'f64': the reference's double arithmetic is the only mode (ABI 2)")
        self.precision = precision
        self.samples_per_pass = int(samples_per_pass)
        # True forces the global-memory extend kernel even when the scene fits the LDS-resident variant (A/B, tests)
        self.global_scene = False
        # True keeps shading in separate per-material k_shade launches even when it could be fused (A/B, tests)
        self.split_shade = False
        # True runs the fused LDS kernel once per bounce depth instead of the persistent-path kernel (A/B, tests)
        self.wavefront = False
        self.world = None
        self.background = (0.0, 0.0, 0.0)
        self._scene = None
        self.stats = {}

    def set_scene(self, world, background):  # engine.h:24-28
        self.world = world
        self.background = tuple(float(x) for x in background)
        self._scene = None if world is None or world.empty() else compile_world(world, self.device)

    def scene_info(self):
        """rt_scene_info of the engine's compiled scene (device_bytes_f64 is set once a render uploaded it)."""
        from ._lib import rt_scene_info
        if self._scene is None:
            raise ValueError("no scene set")
        info = rt_scene_info()
        check(lib.rt_scene_info_get(self._scene, ctypes.byref(info)), "rt_scene_info_get")
        return {f: (tuple(getattr(info, f)) if isinstance(getattr(info, f), ctypes.Array) else getattr(info, f)) for f, _ in info._fields_}

    def params(self, band_rows=None, band_count=1, band_index=0, flags=0, stream=None):
        p = rt_params()
        p.width, p.height = self.width, self.height
        p.spp, p.max_depth, p.seed = self.samples_per_pixel, self.max_depth, self.seed
        p.fp_mode = RT_FP64
        p.band_rows = band_rows or self.height
        p.band_count, p.band_index = band_count, band_index
        p.samples_per_pass, p.flags = self.samples_per_pass, flags
        p.stream = stream
        for c in range(3):
            p.background[c] = self.background[c]
        return p

    def run(self, output_image, accum=None, band_rows=None, band_count=1, band_index=0, profile=False, stream=None):
        """Renders into output_image (uint8, local_rows x W x 3).  Returns elapsed ms, or -1 on an empty world
        (engine.h:32-36).  `accum` (optional, float64 local_rows x W x 3) receives the per-pixel radiance sums.
        engine_mode.adaptive runs _run_adaptive (engine.h:151-333) on the GPU; engine_mode.parallel_images runs
        _run_parallel_images (engine.h:378-445: four float partial images of spp/4 samples, summed); single and
        parallel_stripes compute the same image (their only difference is the reference's CPU threading)."""
        if self._scene is None:
            print("Invalid input scene!")
            return -1
        adaptive = self.m == engine_mode.adaptive
        if adaptive and (self.width % 12 or self.height % 12):
            # engine.h:178-179
            raise ValueError("for adaptive strategy image size should perfectly fit big square size for now!!")
        if adaptive and accum is not None:
            raise ValueError("engine_mode.adaptive interpolates most pixels: there are no radiance sums to return")
        flags = ((RT_PROFILE if profile else 0) | (RT_GLOBAL_SCENE if self.global_scene else 0)
                 | (RT_SPLIT_SHADE if self.split_shade else 0) | (RT_ADAPTIVE if adaptive else 0)
                 | (RT_PARALLEL_IMAGES if self.m == engine_mode.parallel_images else 0)
                 | (RT_WAVEFRONT if self.wavefront else 0))
        p = self.params(band_rows, band_count, band_index, flags, stream)
        rows = check(lib.rt_local_rows(ctypes.byref(p), None), "rt_local_rows")
        nbytes = rows * self.width * 3
        ptr, dev = _pointer(output_image, nbytes)
        acc_ptr = None
        if accum is not None:
            acc_ptr, acc_dev = _pointer(accum.view(np.uint8) if isinstance(accum, np.ndarray) else accum, nbytes * 8)
            if acc_dev != dev:
                raise ValueError("output_image and accum must both live on the host or both on the device")
        if dev:
            p.flags |= RT_OUT_DEVICE
        st = rt_stats()
        check(lib.rt_render(self._scene, ctypes.byref(self.cam.c), ctypes.byref(p), ctypes.c_void_p(ptr),
                            ctypes.c_void_p(acc_ptr) if acc_ptr else None, ctypes.byref(st)), "engine.run")
        self.stats = st.as_dict()
        return int(round(st.ms))

    def run_progressive(self, output_image, callback, accum=None, samples_per_pass=0):
        """Progressive render (rt_render_progressive): the frame is traced in passes of samples_per_pass samples
        (0: spp / 8); after each pass callback(samples_done, spp) runs with output_image (and accum) holding the frame
        of the samples so far.  A truthy return value stops the render.  Returns elapsed ms, or -1 on an empty world."""
        if self._scene is None:
            print("Invalid input scene!")
            return -1
        if self.m in (engine_mode.adaptive, engine_mode.parallel_images):
            raise ValueError("progressive rendering traces whole frames of consecutive samples "
                             "(engine_mode.adaptive / parallel_images are not progressive)")
        p = self.params(None, 1, 0, 0, None)
        p.samples_per_pass = int(samples_per_pass)
        nbytes = self.height * self.width * 3
        ptr, dev = _pointer(output_image, nbytes)
        acc_ptr = None
        if accum is not None:
            acc_ptr, acc_dev = _pointer(accum.view(np.uint8) if isinstance(accum, np.ndarray) else accum, nbytes * 8)
            if acc_dev != dev:
                raise ValueError("output_image and accum must both live on the host or both on the device")
        if dev:
            p.flags |= RT_OUT_DEVICE
        errors = []

        def trampoline(_user, done, spp, _rgb, _acc):
            try:
                return 1 if callback(int(done), int(spp)) else 0
            except BaseException as e:  # an exception must not unwind through the C frames: stop and re-raise after
                errors.append(e)
                return 1

        cb = rt_progress_fn(trampoline)
        st = rt_stats()
        check(lib.rt_render_progressive(self._scene, ctypes.byref(self.cam.c), ctypes.byref(p), ctypes.c_void_p(ptr),
                                        ctypes.c_void_p(acc_ptr) if acc_ptr else None, cb, None, ctypes.byref(st)),
              "engine.run_progressive")
        if errors:
            raise errors[0]
        self.stats = st.as_dict()
        return int(round(st.ms))

    def local_rows(self, band_rows, band_count, band_index):
        p = self.params(band_rows, band_count, band_index)
        n = check(lib.rt_local_rows(ctypes.byref(p), None), "rt_local_rows")
        rows = (ctypes.c_int32 * max(n, 1))()
        lib.rt_local_rows(ctypes.byref(p), rows)
        return np.array(rows[:n], dtype=np.int64)
