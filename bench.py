"""Benchmark: Msamples/s (primary + secondary rays) of the HIP path on BASELINE.json's headline workload.

    python bench.py [--gpus N --steps K --warmup W] [--scene 1 --width 1920 --height 1080 --spp 1024]

One step = one full frame of configs[1] ("'One Weekend' final random-spheres scene, 1920x1080, 1024 spp"): every
rank renders its row-interleaved bands (another_raytracer_amd/distributed.py) and rank 0 gathers the RGB8 frame over
RCCL.  The total work per step is fixed as N grows ("scaling": "strong"); value = all segments traced by all ranks /
max-over-ranks wall time of the K timed steps.  A segment is one ray traced through the world (one world.hit call of
engine.h:453), counted exactly on the device from the wavefront queue sizes.

Extra fields:
  roofline      dominant kernel (k_paths / k_paths_g, or k_extend for the per-depth variants), timed live with HIP events
                on the render stream during the timed steps.  The persistent path kernels are VALU-issue / divergence
                bound: bound "valu", achieved = VALU lane-instruction slots issued per second (the newest
                committed PMC summary's wave-instructions per segment x 64 x this run's segments / kernel time), peak
                78.6 T/s (2 cycles per wave-instruction per SIMD at 2.4 GHz), lane_util from the same summary; the
                SURVEY.md §8(d) HBM figure (128 B per segment + 12 B per pixel + the flat scene once per launch, vs
                8 TB/s) sits under `hbm`.  Without a PMC summary for the scene/variant the HBM figure is the roofline.
                `traffic` = FETCH_SIZE*2 + WRITE_SIZE per segment from the committed rocprofv3 PMC summary
                (profiles/, MI355X_MICROARCH.md "HBM") scaled to this run, or null.
  cpu_baseline  the reference itself (oracle/_ref/ref_harness = /root/reference/src compiled unmodified), its own
                CPU-parallel mode (engine.h:335-376: 4 row stripes, 4 threads, shared global RNG) on a bounded sample
                of the same workload (same scene, full 1920x1080, reduced spp), median of 3 runs, rank 0 at N=1 only;
                plus `all_cores`: the oracle's restatement on every host thread the job may use (median of 3).
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
    ap.add_argument("--gpus", type=int, default=1)
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
    return ap.parse_args()


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def cpu_baseline(args, repeats=3):
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
    for _ in range(repeats):
        out = subprocess.run([harness, "render", args.scene, str(args.width), str(args.height), str(args.cpu_baseline_spp),
                              "/tmp/bench_cpu_ref", "stripes", str(threads)], capture_output=True, text=True, timeout=900)
        if out.returncode != 0:
            return {"error": out.stderr.strip()[-300:]}
        last = json.loads(out.stdout.strip().splitlines()[-1])
        runs.append(last["mseg_per_s"])
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    res = {"value": round(_median(runs), 4), "unit": "Msamples/s", "cores": threads, "kind": "reference",
           "sample": f"scene {args.scene} {args.width}x{args.height}x{args.cpu_baseline_spp}spp "
                     f"({last['segments']} segments, {last['ms'] / 1e3:.1f} s per run), median of {repeats} runs, "
                     f"engine_mode::parallel_stripes semantics (4 threads, shared global mt19937); per-segment cost is spp-independent",
           "runs_Msamples_s": [round(x, 4) for x in runs], "cpu_model": model, "host_cpus": os.cpu_count()}
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


def latest_pmc(precision, scene, variant):
    """The newest committed PMC summary (tools/pmc_summary.py format: per-segment wave-instruction counts of the
    dominant kernel) for this scene and extend variant, or None."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):  # tags sort by round and letter
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        k = d.get("dominant_kernel")
        if (d.get("precision") == precision and str(d.get("scene")) == str(scene) and d.get("extend_variant") == variant and k
                and (d.get("kernels", {}).get(k, {}).get("per_segment_wave_instructions"))):
            d["_file"] = os.path.relpath(path, ROOT)
            best = d
    return best


def latest_traffic(precision, scene, variant):
    """Per-segment HBM bytes of k_extend from the newest committed PMC summary (profiles/*pmc*.json) of this extend
    variant, or None."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (d.get("precision") == precision and str(d.get("scene")) == str(scene) and d.get("extend_bytes_per_segment")
                and d.get("extend_variant", 1) == variant):
            best = d
    return best


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import another_raytracer_amd as art
    from another_raytracer_amd.distributed import band_rows_of, render_frame

    world_scene = art.scene_manager(device=dev.index).build(args.scene)
    scene_bytes = int(world_scene.info["device_bytes_f64"])
    cam = art.camera(world_scene.lookfrom, world_scene.lookat, (0, 1, 0), world_scene.vfov, args.width / args.height,
                     world_scene.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.parallel_stripes, width=args.width, height=args.height,
                     samples_per_pixel=args.spp, max_depth=args.max_depth, device=dev.index, precision=args.precision,
                     samples_per_pass=args.samples_per_pass)
    eng.set_scene(world_scene.objects, world_scene.background)
    eng.global_scene = args.global_scene
    eng.split_shade = args.split_shade
    eng.wavefront = args.wavefront
    rows = band_rows_of(args.height, args.band_rows, world, rank)
    local = torch.empty((len(rows), args.width, 3), dtype=torch.uint8, device=dev)
    profile = not args.no_profile

    def step():
        return render_frame(eng, band_rows=args.band_rows, device=dev, profile=profile, out_local=local)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs = 0
    ext_ms = shade_ms = gpu_ms = 0.0
    ext_launches = 0
    primary_segs = 0
    variant = 0
    frame = None
    for _ in range(args.steps):
        frame, st = step()
        segs += st["segments"]
        ext_ms += st["extend_ms"]
        shade_ms += st["shade_ms"]
        gpu_ms += st["ms"]
        ext_launches += st["extend_launches"]
        primary_segs += st["primary"]
        variant = st["extend_variant"]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stats = torch.tensor([elapsed, float(segs), ext_ms, shade_ms, float(ext_launches), float(primary_segs)],
                         dtype=torch.float64, device=dev)
    if world > 1:
        t_max = stats[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = stats[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed = float(t_max.item())
        segs, ext_ms, shade_ms, ext_launches, primary_segs = (float(x) for x in tot.tolist())
    if rank == 0:
        value = segs / elapsed / 1e6
        primary = args.width * args.height * args.spp * args.steps
        line = {
            "metric": "Msamples/sec (primary+secondary rays) at 1920x1080x1024spp; 1/2/4/8 GPU",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": f"scene_alias {args.scene} ('One Weekend' final random spheres)" if args.scene == "1"
                       else f"scene {args.scene}", "width": args.width, "height": args.height, "spp": args.spp,
                       "max_depth": args.max_depth, "parallelism": f"row-bands({args.band_rows}) x {world} + rccl gather",
                       "segments_per_step": int(segs / args.steps), "primary_rays_per_step": primary // args.steps,
                       "mprimary_per_s": round(primary / elapsed / 1e6, 3)},
        }
        if profile and ext_ms > 0:
            launches = max(ext_launches, 1)
            per_launch_ms = ext_ms / launches
            pixels = args.width * args.height * args.steps
            alg = survey_algorithmic_bytes(segs, pixels, scene_bytes * ext_launches)
            achieved = alg / (ext_ms * 1e-3) / 1e9
            moved = extend_moved_bytes(args.precision, variant, segs, primary_segs)
            tr = latest_traffic(args.precision, args.scene, variant)
            kernel = {3: "k_paths", 4: "k_paths_g"}.get(variant, "k_extend")
            hbm = {"achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                   "algorithmic_bytes_per_launch": round(alg / launches),
                   "algorithmic_bytes": "SURVEY 8(d): 128 B/segment + 12 B/pixel + scene bytes per launch",
                   "moved_bytes_per_segment": round(moved / max(segs, 1), 2)}
            roof = {"kernel": kernel, "traffic": (round(tr["extend_bytes_per_segment"] * segs / launches) if tr else None),
                    "extend_variant": variant, "avg_launch_ms": round(per_launch_ms, 4), "launches": int(ext_launches),
                    "extend_ms_total": round(ext_ms, 2), "shade_ms_total": round(shade_ms, 2)}
            pm = latest_pmc(args.precision, args.scene, variant) if variant in (3, 4) else None
            if pm:
                # The persistent path kernels are bound by VALU issue and lane divergence, not HBM (the
                # scene lives in LDS / L2, ~9-30 B of HBM per segment).  achieved = VALU lane-instruction slots issued
                # per second: the PMC summary's wave-instructions per segment x 64 lanes x the segments of this run /
                # the kernel time measured live; lane_util = the share of those slots doing work (SQ_THREAD_CYCLES_VALU)
                ps = pm["kernels"][pm["dominant_kernel"]]["per_segment_wave_instructions"]
                slots = ps["insts_valu"] * 64 * segs / (ext_ms * 1e-3) / 1e12
                roof.update({"bound": "valu", "achieved": round(slots, 3), "peak": round(VALU_PEAK_TLANE, 2), "unit": "Tlane-inst/s",
                             "frac": round(slots / VALU_PEAK_TLANE, 4),
                             "valu_wave_insts_per_segment": round(ps["insts_valu"], 2),
                             "lane_util": pm.get("valu_lane_util"), "useful_frac": round(slots / VALU_PEAK_TLANE * pm.get("valu_lane_util", 0), 4),
                             "issue_util_calibrated_pmc": pm.get("valu_issue_util_calibrated"),
                             "wave_frac_wait_waitcnt_pmc": pm.get("wave_frac_wait_waitcnt"),
                             "wave_frac_wait_dependency_pmc": pm.get("wave_frac_wait_inst_dependency"),
                             "pmc_summary": pm["_file"], "hbm": hbm})
            else:
                roof.update({"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm["frac"]})
                roof.update({k: v for k, v in hbm.items() if k not in roof})
            line["roofline"] = roof
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
