"""Benchmark: Msamples/s (primary + secondary rays) of the HIP path on BASELINE.json's headline workload.

    python bench.py [--gpus N --steps K --warmup W] [--scene 1 --width 1920 --height 1080 --spp 1024]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...     (one process per GPU)

One step = one full frame of configs[1] ("'One Weekend' final random-spheres scene, 1920x1080, 1024 spp"), split into
row-interleaved bands (8 rows; band b on GPU b mod N) and gathered as RGB8 on GPU 0.  Two drivers of that partition:
  * plain `python bench.py --gpus N` (the default, N = 1): this process drives GPUs 0..N-1 through the C ABI,
    rt_render_multi (csrc/multi.hip: one host thread and one RCCL rank per GPU, ncclGather of the packed band blocks to
    GPU 0 + an unpack kernel).  Fewer than N visible GPUs is an error, never a silent 1-GPU run.
  * under torchrun (WORLD_SIZE = N ranks; --gpus must equal it): one process per GPU, each renders its bands into its
    padded block, dist.gather over RCCL to rank 0, libart's rt_unpack_bands places the rows (the same layout and unpack
    kernel).
The total work per step is fixed as N grows ("scaling": "strong"); value = all segments traced on all GPUs / wall time
of the K timed steps (max over ranks under torchrun), gather and unpack included.  A segment is one ray traced through
the world (one world.hit call of engine.h:453), counted exactly on the device.
C5 (BASELINE configs[4]): python bench.py --gpus 8 --scene dino --width 4096 --height 4096 --spp 8192 --steps 1 --warmup 1
(the scene is uploaded by rt_multi_create, before any step; the warm-up render allocates the pass workspace, so the one
timed step is the render alone -- the reference times engine::run only, main.cpp:44-46)

Extra fields:
  roofline      the dominant kernel (k_paths / k_paths_g) on the slowest GPU, each launch timed live with HIP events on
                its render stream during the timed steps.  bound "hbm": achieved = SURVEY.md §8(d) algorithmic bytes per
                launch (128 B per segment + 12 B per pixel + the flat scene) / average launch time, vs 8 TB/s; `traffic`
                = measured HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE per segment, MI355X_MICROARCH.md "HBM")
                from the committed PMC summary (profiles/*pmc*.json) stamped with this library's device-code build id,
                else null.  The kernels' actual limiter, VALU issue and lane divergence, is under `valu`
                from the same build-matched summary: VALU lane-slots issued per second vs 78.6 T/s, lane_util,
                useful_frac.
  cpu_baseline  the reference itself (oracle/_ref/ref_harness = /root/reference/src compiled unmodified), its own
                CPU-parallel mode (engine.h:335-376: 4 row stripes, 4 threads, shared global RNG) on a bounded sample
                of the same workload (same scene, full 1920x1080, reduced spp), median and spread of 5 runs, N = 1 only;
                plus `all_cores`: the oracle's restatement on every host thread the job may use (median of 5).
  parity        the timed frame itself checked per pixel, after the timed steps: a bounded set of full-spp rows of the
                last timed step's RGB8 against the oracle's CPU restatement driven by the same PCG streams (rmse_lsb,
                max_dlsb, within_1lsb, bit_exact; SURVEY.md §8(d) tolerance: RMSE <= 1.0 LSB).
  config.phases where the step time goes: rt_multi_times (renders slowest/fastest device, ncclGather, unpack) with the
                one-process driver; per-rank render and step times under torchrun.
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# MI355X_MICROARCH.md: a wave issues one VALU instruction per 2 cycles per SIMD (64 lanes), 256 CUs x 4 SIMDs at the
# 2.4 GHz max clock: 78.6 T lane-instructions/s (x 2 flops per FMA = the guide's 157.3 TF f32 vector peak)
VALU_PEAK_TLANE = 256 * 4 * 64 / 2 * 2.4e9 / 1e12
# algorithmic bytes of the path = 128 B per segment (a 64-B fp32 path record read once and written
# once per bounce) + 12 B per pixel (f32 RGB accumulator write) + one pass over the flat scene.  The same figure for
# every kernel variant, so `achieved` compares variants and rounds on one scale.
SURVEY_SEG_BYTES = 128
SURVEY_PIX_BYTES = 12
# Bytes the extend kernel of each variant really moves per unit, reported beside it:
#   0/1 (split shading): queue id 4 + ray line (f32 32 B / f64 64 B) + hit record 16 + material-queue id 4 per segment;
#   2 (fused, one launch per depth): a non-primary segment reads its queue id and whole path record and, when it
#     continues, writes the record back plus the next queue id; every path ends with one radiance record;
#   3 (persistent paths): the path lives in registers; only the final radiance record of every path is written.
EXTEND_BYTES = {"f32": 4 + 32 + 16 + 4, "f64": 4 + 64 + 16 + 4}
PATH_BYTES = {"f32": 64, "f64": 128}
RES_BYTES = {"f32": 16, "f64": 24}


def extend_moved_bytes(precision, variant, segments, primary):
    """Bytes the extend launches of the timed region move by construction (variant-specific)."""
    if variant in (3, 4):  # persistent paths: the radiance record per path only
        return primary * RES_BYTES[precision]
    if variant == 2:
        rec = PATH_BYTES[precision]
        return (segments - primary) * (4 + rec + rec + 4) + primary * RES_BYTES[precision]
    return EXTEND_BYTES[precision] * segments


def survey_algorithmic_bytes(segments, pixels, scene_bytes):
    return SURVEY_SEG_BYTES * segments + SURVEY_PIX_BYTES * pixels + scene_bytes


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (default 1; under torchrun: WORLD_SIZE)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--precision", default="f64", choices=["f64"])  # the reference's double (ABI 2: the only mode)
    ap.add_argument("--band-rows", type=int, default=8)  # distributed.DEFAULT_BAND_ROWS
    ap.add_argument("--samples-per-pass", type=int, default=0)
    ap.add_argument("--no-profile", action="store_true", help="skip per-launch HIP events (no roofline)")
    ap.add_argument("--global-scene", action="store_true", help="force the global-memory extend kernel (A/B vs LDS scene)")
    ap.add_argument("--split-shade", action="store_true", help="keep per-material k_shade launches (A/B vs fused shading)")
    ap.add_argument("--wavefront", action="store_true", help="one fused extend launch per depth (A/B vs persistent paths)")
    ap.add_argument("--cpu-baseline-spp", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the timed frame's rows")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="rt_option_set before the scene is built (builder experiments, e.g. bvh.sah_ci=1.0; repeatable)")
    return ap.parse_args()


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def cpu_baseline(args, repeats=9):
    """Two CPU figures on the box's host cores, each the median of `repeats` bounded samples of the same workload
    (same scene, full width and height, reduced spp: the per-segment cost does not depend on spp):
      * the reference itself (oracle/_ref/ref_harness = /root/reference/src compiled unmodified by oracle/Makefile) in
        its own CPU-parallel mode, engine_mode::parallel_stripes (engine.h:335-376: 4 row stripes on 4 threads sharing
        the global mt19937);
      * all_cores: the oracle's restatement (oracle/_ref/liboracle.so, pcg mode: per-(pixel, sample) streams, no shared
        state) on every host thread this job may use (OMP_NUM_THREADS, else os.cpu_count()), rows taken dynamically."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    threads = 4
    runs, last = [], None
    # one discarded warm-up run first: r6e's first runs came out ~6 % below the rest (clock ramp of the host cores)
    for i in range(repeats + 1):
        # PIN 1: the harness pins its worker t to the t-th CPU of this job's affinity set (sched_setaffinity: no
        # migrations between the host's shared cores, the run-to-run spread of r4/r5 was +-15 %)
        out = subprocess.run([harness, "render", args.scene, str(args.width), str(args.height), str(args.cpu_baseline_spp),
                              "/tmp/bench_cpu_ref", "stripes", str(threads), "1"], capture_output=True, text=True, timeout=900)
        if out.returncode != 0:
            return {"error": out.stderr.strip()[-300:]}
        last = json.loads(out.stdout.strip().splitlines()[-1])
        if i > 0:
            runs.append(last["mseg_per_s"])
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    res = {"value": round(_median(runs), 4), "unit": "Msamples/s", "cores": threads, "kind": "reference",
           "sample": f"scene {args.scene} {args.width}x{args.height}x{args.cpu_baseline_spp}spp "
                     f"({last['segments']} segments, {last['ms'] / 1e3:.1f} s per run), median of {repeats} runs after a discarded "
                     f"warm-up run, engine_mode::parallel_stripes semantics (4 threads pinned to 4 CPUs, shared global mt19937); "
                     f"per-segment cost is spp-independent",
           "runs_Msamples_s": [round(x, 4) for x in runs], "spread_Msamples_s": [round(min(runs), 4), round(max(runs), 4)],
           "max_Msamples_s": round(max(runs), 4), "spread_frac": round((max(runs) - min(runs)) / _median(runs), 4),
           "cpu_model": model, "host_cpus": os.cpu_count()}
    try:
        from tests.oracle_lib import oracle_render
        env = os.environ.get("OMP_NUM_THREADS", "")
        nt = int(env) if env.isdigit() and int(env) > 0 else (os.cpu_count() or 1)
        spp = max(1, args.cpu_baseline_spp * 2)
        ports = []
        for _ in range(repeats):
            o = oracle_render(args.scene, args.width, args.height, spp, mode="pcg", threads=nt)
            ports.append((o["segments"] / (o["ms"] * 1e3), o))
        v, o = sorted(ports, key=lambda t: t[0])[len(ports) // 2]
        res["all_cores"] = {"value": round(v, 4), "unit": "Msamples/s", "cores": nt, "kind": "port",
                            "sample": f"scene {args.scene} {args.width}x{args.height}x{spp}spp ({o['segments']} segments, "
                                      f"{o['ms'] / 1e3:.1f} s per run), median of {repeats} runs, oracle/restate.cpp pcg mode "
                                      f"(the product's RNG contract), dynamic rows over {nt} threads",
                            "runs_Msamples_s": [round(t[0], 4) for t in ports]}
    except Exception as e:  # the port is optional evidence: report, do not fail the bench
        res["all_cores"] = {"error": str(e)[-300:]}
    return res


def frame_parity(args, frame, budget_segments=2.5e8):
    """Per-pixel parity of the timed frame (the last timed step's RGB8 on GPU 0) against the oracle's CPU restatement
    driven by the same PCG streams (oracle/restate.cpp pcg mode, orc_render_rows: full spp, the same rows), outside the
    timed region: RMSE and largest difference in 8-bit levels (LSB) over a bounded set of rows spread over the frame,
    plus the rows through its middle (SURVEY.md §8(d) tolerance 2: RMSE <= 1.0 LSB, >= 99.5 % of pixels within 1 LSB;
    the f64 path is bit-exact).  Test infrastructure as the checker only: the frame was produced by libart alone."""
    import numpy as np
    try:
        from tests.oracle_lib import oracle_render_rows
    except Exception as e:  # the checker is optional evidence: report, do not fail the bench
        return {"error": str(e)[-300:]}
    W, H, spp = args.width, args.height, args.spp
    n = int(max(2, min(16, budget_segments // max(1, W * spp * 3))))
    rows = sorted(set([int(round(i * (H - 1) / max(1, n - 2))) for i in range(n - 1)] + [H // 2]))
    env = os.environ.get("OMP_NUM_THREADS", "")
    nt = int(env) if env.isdigit() and int(env) > 0 else (os.cpu_count() or 1)
    t0 = time.perf_counter()
    o = oracle_render_rows(args.scene, W, H, spp, rows, seed=0, threads=nt, max_depth=args.max_depth)
    got = frame[rows].astype(np.int64)
    d = got - o["rgb"].astype(np.int64)
    return {"rows": rows, "pixels": int(d.shape[0] * d.shape[1]), "spp": spp, "rmse_lsb": float(np.sqrt(np.mean(d.astype(np.float64) ** 2))),
            "max_dlsb": int(np.abs(d).max()), "within_1lsb": float(np.mean(np.all(np.abs(d) <= 1, axis=-1))),
            "bit_exact": bool(np.array_equal(got, o["rgb"])), "tolerance": "RMSE <= 1.0 LSB and >= 99.5 % of pixels within 1 LSB (SURVEY 8(d) 2)",
            "oracle": f"oracle/restate.cpp pcg mode, orc_render_rows over {nt} threads ({o['segments']} segments, {time.perf_counter() - t0:.1f} s)"}


def latest_pmc(precision, scene, variant, build):
    """The newest committed PMC summary (tools/pmc_summary.py format) for this scene and kernel variant whose
    `libart_build` stamp equals the loaded library's device code (another_raytracer_amd._lib.kernel_build_id), or None:
    counters of another build never price this run."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):  # tags sort by round and letter
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (d.get("precision") == precision and str(d.get("scene")) == str(scene) and d.get("extend_variant") == variant
                and d.get("libart_build") == build):
            d["_file"] = os.path.relpath(path, ROOT)
            best = d
    return best


def choose_driver(gpus, world_env, device_count, torchrun=False):
    """How `bench.py --gpus N` runs: ("procs", N) under torchrun (one process per GPU, WORLD_SIZE = N ranks; a single
    torchrun rank too, which is how the one-process-per-GPU A/B switches run on one GPU), else
    ("multi", N): this one process drives N GPUs through the C ABI (rt_render_multi: one host thread and one RCCL rank
    per device, ncclGather + unpack kernel on device 0).  Never silently fewer GPUs than asked: SystemExit instead."""
    if world_env > 1 or torchrun:
        if gpus is not None and gpus != world_env:
            raise SystemExit(f"bench.py: --gpus {gpus} but torchrun started WORLD_SIZE={world_env} ranks")
        return "procs", world_env
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {n})")
    if device_count < n:
        raise SystemExit(f"bench.py: --gpus {n} needs {n} visible GPUs, found {device_count}: refusing to measure fewer")
    return "multi", n


def roofline_of(dev_stats, width, scene_bytes, variant, precision, scene, build):
    """`roofline` of the dominant kernel on the slowest device (the one that sets the step time).  SURVEY.md §8(d)'s
    contract: bound "hbm", achieved = algorithmic bytes per launch (128 B per segment + 12 B per pixel + the flat scene
    once) / the kernel's average launch time measured live with HIP events on its stream; `traffic` = HBM bytes per
    launch from the build-matched PMC summary (2 x FETCH_SIZE + WRITE_SIZE per segment x segments per launch), else null.
    The kernel's real limiter -- VALU issue and lane divergence -- is under `valu` when a build-matched
    PMC summary exists."""
    slow = max(dev_stats, key=lambda d: d["extend_ms"])
    launches = max(int(slow["extend_launches"]), 1)
    per_launch_ms = slow["extend_ms"] / launches
    segs = slow["segments"] / launches
    pixels = slow["local_rows"] * width * slow["steps"] / launches
    alg = survey_algorithmic_bytes(segs, pixels, scene_bytes)
    achieved = alg / (per_launch_ms * 1e-3) / 1e9
    kernel = {3: "k_paths", 4: "k_paths_g"}.get(variant, "k_extend")
    moved = extend_moved_bytes(precision, variant, slow["segments"], slow["primary"])
    pm = latest_pmc(precision, scene, variant, build)
    tr = pm.get("extend_bytes_per_segment") if pm else None
    roof = {"kernel": kernel, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": float(f"{achieved / HBM_PEAK_GBS:.6g}"), "traffic": round(tr * segs) if tr else None,
            "algorithmic_bytes_per_launch": round(alg),
            "algorithmic_bytes": "SURVEY 8(d): 128 B/segment + 12 B/pixel + scene bytes, per launch of the slowest device",
            "segments_per_launch": round(segs), "avg_launch_ms": round(per_launch_ms, 4), "launches": launches,
            "devices": len(dev_stats), "extend_variant": variant, "libart_build": build,
            "moved_bytes_per_segment": round(moved / max(slow["segments"], 1), 2)}
    if pm and variant in (3, 4):
        # VALU lane-instruction slots issued per second: the summary's wave-instructions per segment x 64 lanes x the
        # segments of a launch / the launch time measured here; lane_util = the share of those slots doing work
        k = pm.get("dominant_kernel")
        ps = pm.get("kernels", {}).get(k, {}).get("per_segment_wave_instructions", {})
        if ps.get("insts_valu"):
            slots = ps["insts_valu"] * 64 * segs / (per_launch_ms * 1e-3) / 1e12
            lu = pm.get("valu_lane_util", 0)
            roof["valu"] = {"achieved": round(slots, 3), "peak": round(VALU_PEAK_TLANE, 2), "unit": "Tlane-inst/s",
                            "frac": float(f"{slots / VALU_PEAK_TLANE:.6g}"), "lane_util": lu,
                            "useful_frac": round(slots / VALU_PEAK_TLANE * lu, 4),
                            "valu_wave_insts_per_segment": round(ps["insts_valu"], 2),
                            "issue_util_calibrated": pm.get("valu_issue_util_calibrated"),
                            "wave_frac_wait_waitcnt": pm.get("wave_frac_wait_waitcnt"),
                            "wave_frac_wait_dependency": pm.get("wave_frac_wait_inst_dependency")}
        roof["pmc_summary"] = pm["_file"]
    return roof


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    driver, n = choose_driver(args.gpus, world_env, torch.cuda.device_count(), torchrun="TORCHELASTIC_RUN_ID" in os.environ)
    rank = int(os.environ.get("RANK", "0"))
    if driver == "procs":
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if local_rank >= torch.cuda.device_count():
            raise SystemExit(f"bench.py: rank {rank} has LOCAL_RANK {local_rank} but only {torch.cuda.device_count()} GPUs are visible")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import another_raytracer_amd as art
    from another_raytracer_amd._lib import kernel_build_id
    from another_raytracer_amd.distributed import frame_renderer, multi_engine

    build = kernel_build_id()
    for o in args.option:
        name, _, value = o.partition("=")
        art.set_option(name, float(value))
    profile = not args.no_profile
    if driver == "multi":
        if args.global_scene or args.split_shade or args.wavefront or args.samples_per_pass:
            raise SystemExit("bench.py: --global-scene / --split-shade / --wavefront / --samples-per-pass are one-process-per-GPU "
                             "A/B switches (run them under torchrun)")
        devices = list(range(n))
        probe = art.scene_manager(device=0).build(args.scene)  # the scene_manager view (camera placement)
        cam = art.camera(probe.lookfrom, probe.lookat, (0, 1, 0), probe.vfov, args.width / args.height, probe.aperture, 10.0, 0.0, 1.0)
        del probe
        eng = multi_engine(args.scene, devices, cam, args.width, args.height, args.spp, max_depth=args.max_depth,
                           band_rows=args.band_rows)
        frame = torch.empty((args.height, args.width, 3), dtype=torch.uint8, device=dev)

        def step():
            eng.run(frame, profile=profile)
            times.append(eng.times())
            return eng.stats, eng.device_stats()

        def last_frame():
            return frame

        def sync():
            for d in devices:
                torch.cuda.synchronize(d)

        def scene_bytes_now():  # uploaded at the first render
            return int(eng.scene_info()["device_bytes_f64"])
        parallelism = (f"1 GPU, rt_render_multi (row-bands({args.band_rows}), single-rank gather + unpack)" if n == 1 else
                       f"row-bands({args.band_rows}) over {n} GPUs, one process: rt_render_multi (one host thread + RCCL rank "
                       f"per GPU, ncclGather to GPU 0 + unpack kernel)")
    else:
        world_scene = art.scene_manager(device=dev.index).build(args.scene)
        cam = art.camera(world_scene.lookfrom, world_scene.lookat, (0, 1, 0), world_scene.vfov, args.width / args.height,
                         world_scene.aperture, 10.0, 0.0, 1.0)
        eng = art.engine(cam, art.engine_mode.parallel_stripes, width=args.width, height=args.height,
                         samples_per_pixel=args.spp, max_depth=args.max_depth, device=dev.index, precision=args.precision,
                         samples_per_pass=args.samples_per_pass)
        eng.set_scene(world_scene.objects, world_scene.background)
        eng.global_scene = args.global_scene
        eng.split_shade = args.split_shade
        eng.wavefront = args.wavefront
        fr = frame_renderer(eng, band_rows=args.band_rows, device=dev)

        def step():
            t = time.perf_counter()
            out, st = fr(profile=profile)
            sync()
            last["frame"] = out
            times.append({"total_ms": (time.perf_counter() - t) * 1e3, "render_ms": st["ms"]})
            return st, [st]

        def last_frame():
            return last["frame"]

        def sync():
            torch.cuda.synchronize(dev)

        def scene_bytes_now():  # uploaded at the first render
            return int(eng.scene_info()["device_bytes_f64"])
        parallelism = (f"row-bands({args.band_rows}) over {n} GPUs, one process per GPU (torchrun): dist.gather over RCCL "
                       f"to rank 0 + rt_unpack_bands")

    times, last = [], {}
    for _ in range(args.warmup):
        step()
    del times[:]
    if driver == "procs":
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    segs = primary_segs = 0
    variant = -1
    acc = None  # per-device totals over the timed steps
    for _ in range(args.steps):
        st, per_dev = step()
        segs += st["segments"]
        primary_segs += st["primary"]
        variant = max(variant, st["extend_variant"])
        kid = [st.get("kernel_features", 0), st.get("kernel_textures", 0), st.get("kernel_lds_mode", -1)]
        if acc is None:
            acc = [{"segments": 0, "primary": 0, "extend_ms": 0.0, "extend_launches": 0, "local_rows": d["local_rows"], "steps": 0}
                   for d in per_dev]
        for a, d in zip(acc, per_dev):
            a["segments"] += d["segments"]
            a["primary"] += d["primary"]
            a["extend_ms"] += d["extend_ms"]
            a["extend_launches"] += d["extend_launches"]
            a["steps"] += 1
    sync()
    if driver == "procs":
        dist.barrier()
    elapsed = time.perf_counter() - t0
    phase = None
    scene_bytes = scene_bytes_now()  # uploaded by the first render
    if driver == "procs":
        # max wall time over ranks; all ranks' segments; every rank's per-device totals for the roofline
        mine = torch.tensor([elapsed, float(segs), float(primary_segs), float(variant), acc[0]["segments"], acc[0]["primary"],
                             acc[0]["extend_ms"], acc[0]["extend_launches"], acc[0]["local_rows"], acc[0]["steps"],
                             sum(t["render_ms"] for t in times) / max(len(times), 1), sum(t["total_ms"] for t in times) / max(len(times), 1)],
                            dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(n)]
        dist.all_gather(allr, mine)
        rows = [t.tolist() for t in allr]
        elapsed = max(r[0] for r in rows)
        segs = sum(r[1] for r in rows)
        primary_segs = sum(r[2] for r in rows)
        variant = int(max(r[3] for r in rows))
        acc = [{"segments": r[4], "primary": r[5], "extend_ms": r[6], "extend_launches": r[7], "local_rows": int(r[8]), "steps": int(r[9])}
               for r in rows]
        phase = {"render_ms_per_rank": [round(r[10], 3) for r in rows], "step_ms_per_rank": [round(r[11], 3) for r in rows],
                 "note": "per step, averaged over the timed steps: render = rt_render of the rank's bands (kernels + finalize); "
                         "step = render + dist.gather over RCCL + rt_unpack_bands on rank 0"}
    if rank == 0:
        value = segs / elapsed / 1e6
        primary = args.width * args.height * args.spp * args.steps
        line = {
            "metric": "Msamples/sec (primary+secondary rays) at 1920x1080x1024spp; 1/2/4/8 GPU",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": f"scene_alias {args.scene} ('One Weekend' final random spheres)" if args.scene == "1"
                       else f"scene {args.scene}", "width": args.width, "height": args.height, "spp": args.spp,
                       "max_depth": args.max_depth, "parallelism": parallelism, "driver": driver,
                       "segments_per_step": int(segs / args.steps), "primary_rays_per_step": primary // args.steps,
                       "mprimary_per_s": round(primary / elapsed / 1e6, 3),
                       "kernel_f_tf_lm": kid},
        }
        if args.option:  # the library options this line was measured under (A/B and sweep lines name their setting)
            line["config"]["options"] = {o.partition("=")[0]: float(o.partition("=")[2]) for o in args.option}
        if n > 1:
            line["config"]["per_gpu_kernel_ms_per_step"] = [round(a["extend_ms"] / max(a["steps"], 1), 3) for a in acc]
        if driver == "multi" and times:
            avg = lambda k: round(sum(t[k] for t in times) / len(times), 4)
            phase = {k: avg(k) for k in ("total_ms", "render_ms_max", "render_ms_min", "gather_ms", "unpack_ms", "wait_ms")}
            phase["slowest_device"] = times[-1]["slowest_device"]
            phase["note"] = ("rt_multi_times per step, averaged over the timed steps: render = each device's host thread "
                             "(kernels + finalize), gather = ncclGather on GPU 0's stream (HIP events), unpack = k_unpack_bands")
        if phase:
            line["config"]["phases"] = phase
        if profile and acc and any(a["extend_ms"] > 0 for a in acc):
            line["roofline"] = roofline_of(acc, args.width, scene_bytes, variant, args.precision, args.scene, build)
        if n == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args)
        if not args.no_parity:
            f = last_frame()
            line["parity"] = frame_parity(args, f.cpu().numpy() if hasattr(f, "cpu") else f)
        print(json.dumps(line), flush=True)
    if driver == "procs":
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
