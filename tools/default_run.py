"""The reference's default run (main.cpp:20-50: the mesh (capsule) scene, engine_mode::adaptive, 720x540 at 100 spp,
tracer_constants.h) timed on the GPU, next to the same frame in single mode, and the reference itself on the same
box's host CPU (GPU box):

    python tools/default_run.py [--scene 9] [--reps 5] [--cpu-runs 9] [--json OUT]

The CPU line is oracle/_ref/ref_harness (the reference compiled unmodified, its ressources.h pointing at the repo's
copy of the reference's assets, oracle/Makefile ASSET_ROOT) in mode "adaptive4": `_run_adaptive` threaded as the
reference threads it (engine.h:298-313: four row stripes on a 4-thread pool sharing the global RNG), each worker pinned
to one CPU of the job's affinity set; median and best of --cpu-runs runs.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="9")
    ap.add_argument("--width", type=int, default=720)
    ap.add_argument("--height", type=int, default=540)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--cpu-runs", type=int, default=9, help="reference harness runs on the host CPU (0: none)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE", help="rt_option_set before the scene build")
    a = ap.parse_args()
    import another_raytracer_amd as art
    for o in a.option:
        name, _, value = o.partition("=")
        art.set_option(name, float(value))
    w = art.scene_manager().build(a.scene)
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, a.width / a.height, w.aperture, 10.0, 0.0, 1.0)
    rows = []
    for mode in ("adaptive", "single"):
        m = art.engine_mode.adaptive if mode == "adaptive" else art.engine_mode.single
        eng = art.engine(cam, m, width=a.width, height=a.height, samples_per_pixel=a.spp)
        eng.set_scene(w.objects, w.background)
        img = np.zeros((a.height, a.width, 3), np.uint8)
        eng.run(img)  # warm-up (upload, workspace)
        ms = []
        for _ in range(a.reps):
            t = time.perf_counter()
            r = eng.run(img)
            ms.append(((time.perf_counter() - t) * 1e3, r))
        st = eng.stats
        eng.run(img, profile=True)  # HIP events around every path-kernel launch (outside the timed reps)
        prof = eng.stats
        wall = sorted(x[0] for x in ms)[len(ms) // 2]
        rep = sorted(x[1] for x in ms)[len(ms) // 2]
        row = {"scene": a.scene, "mode": mode, "frame": [a.width, a.height, a.spp], "wall_ms": round(wall, 3),
               "engine_ms": round(rep, 3), "segments": st["segments"], "primary": st["primary"],
               "msamples_s": round(st["segments"] / wall / 1e3, 1), "passes": st["passes"], "kernel_ms_profiled": round(prof["extend_ms"], 3), "launches_profiled": prof["extend_launches"],
               "kernel": [st["extend_variant"], st["kernel_features"], st["kernel_textures"], st["kernel_lds_mode"]]}
        if a.option:
            row["options"] = {o.partition("=")[0]: float(o.partition("=")[2]) for o in a.option}
        print(json.dumps(row), flush=True)
        rows.append(row)
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if a.cpu_runs > 0 and os.path.exists(harness):
        import subprocess
        runs = []
        for i in range(a.cpu_runs + 1):  # the first is a discarded warm-up (host clock ramp)
            out = subprocess.run([harness, "render", a.scene, str(a.width), str(a.height), str(a.spp), "/tmp/default_run_cpu",
                                  "adaptive4", "4", "1"], capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                raise SystemExit("ref_harness failed: " + out.stderr.strip()[-400:])
            r = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps(r), flush=True)
            if i > 0:
                runs.append(r)
        ms = sorted(r["ms"] for r in runs)
        model = ""
        try:
            with open("/proc/cpuinfo") as f:
                model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
        except OSError:
            pass
        row = {"scene": a.scene, "mode": "adaptive", "device": "cpu", "kind": "reference", "threads": 4, "pinned": True,
               "frame": [a.width, a.height, a.spp], "runs": len(ms), "ms_median": ms[len(ms) // 2], "ms_min": ms[0],
               "ms_max": ms[-1], "spread_frac": round((ms[-1] - ms[0]) / ms[len(ms) // 2], 4),
               "segments_last": runs[-1]["segments"], "cpu_model": model,
               "note": "oracle/_ref/ref_harness render ... adaptive4 4 1: _run_adaptive's four stripes on four pinned threads "
                       "(engine.h:298-313), the reference's own code compiled unmodified"}
        gpu = next((r for r in rows if r["mode"] == "adaptive"), None)
        if gpu:
            row["gpu_speedup_vs_median"] = round(row["ms_median"] / gpu["wall_ms"], 1)
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
