"""Parity soak (GPU box): every builtin scene rendered with many seeds on the GPU and by the CPU restatement (pcg mode,
the same streams), compared bit for bit (RGB8, f64 sums, segment count) -- the GPU parity suite's check over more random
paths than its fixed seeds reach.  Test infrastructure: the oracle is the checker only.

    python tools/parity_soak.py [--budget-s 240] [--width 96 --height 54 --spp 16] [--variants default,wavefront,...]
                                [--out gpurun_out/soak.json]

Variants: default (the selected persistent kernel), wavefront (per-depth k_extend / k_shade), global (HBM scene),
split (per-material k_shade), depth3 (max_depth 3), codes16off (option render.codes16 = 0: 32-bit-code kernels).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCENES = ["c1", "1", "2", "3", "4", "5", "6", "7", "8", "cow", "dino", "9"]
VARIANTS = {"default": {}, "wavefront": {"wavefront": True}, "global": {"global_scene": True}, "split": {"split_shade": True},
            "depth3": {"max_depth": 3}, "codes16off": {}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget-s", type=float, default=240.0)
    ap.add_argument("--width", type=int, default=96)
    ap.add_argument("--height", type=int, default=54)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--seed0", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--variants", default="default")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from tests.oracle_lib import oracle_render
    from tests.test_gpu_parity import gpu_render
    import another_raytracer_amd as art
    variants = a.variants.split(",")
    for v in variants:
        if v not in VARIANTS:
            raise SystemExit(f"unknown variant {v}")

    def one(scene, v, seed, oracles):
        kw = VARIANTS[v]
        art.set_option("render.codes16", 0.0 if v == "codes16off" else 1.0)
        try:
            g = gpu_render(scene, a.width, a.height, a.spp, seed=seed, **kw)
        finally:
            art.set_option("render.codes16", 1.0)
        depth = kw.get("max_depth", 50)
        if depth not in oracles:
            oracles[depth] = oracle_render(scene, a.width, a.height, a.spp, mode="pcg", seed=seed, threads=a.threads, max_depth=depth)
        o = oracles[depth]
        ok = np.array_equal(g["rgb"], o["rgb"]) and np.array_equal(g["acc"], o["acc"]) and g["segments"] == o["segments"]
        case = {"scene": scene, "variant": v, "seed": seed, "ok": ok, "segments": g["segments"],
                "kernel": [g["stats"]["extend_variant"], g["stats"]["kernel_features"], g["stats"]["kernel_lds_mode"]]}
        if not ok:
            d = np.argwhere(np.any(g["acc"] != o["acc"], axis=-1))
            case.update(oracle_segments=o["segments"], pixels_differing=int(len(d)), first=d[:8].tolist())
        return case

    t0 = time.time()
    cases, bad = [], []
    seed = a.seed0
    while time.time() - t0 < a.budget_s:
        for scene in SCENES:
            oracles = {}  # the oracle's render per max_depth, shared by the variants
            for v in variants:
                case = one(scene, v, seed, oracles)
                if not case["ok"]:
                    bad.append(case)
                    print("MISMATCH", json.dumps(case), flush=True)
                cases.append(case)
        print(f"seed {seed}: {len(cases)} cases, {len(bad)} mismatches, {time.time() - t0:.0f} s", flush=True)
        seed += 1
    kernels = sorted({(c["variant"], c["scene"], *c["kernel"]) for c in cases})
    summary = {"frame": [a.width, a.height, a.spp], "variants": variants, "seeds": [a.seed0, seed - 1], "cases": len(cases),
               "mismatches": bad, "kernels": [list(k) for k in kernels],
               "segments": int(sum(c["segments"] for c in cases)), "seconds": round(time.time() - t0, 1)}
    print(json.dumps({k: v for k, v in summary.items()}), flush=True)
    if a.out:
        json.dump(summary, open(a.out, "w"), indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
