"""The reference's default run (main.cpp:20-50: the mesh (capsule) scene, engine_mode::adaptive, 720x540 at 100 spp,
tracer_constants.h) timed on the GPU, next to the same frame in single mode (GPU box):

    python tools/default_run.py [--scene 9] [--reps 5] [--json OUT]
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
    a = ap.parse_args()
    import another_raytracer_amd as art
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
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
