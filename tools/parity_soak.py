"""Parity soak (GPU box): every builtin scene rendered with many seeds on the GPU and by the CPU restatement (pcg mode,
the same streams), compared bit for bit (RGB8, f64 sums, segment count) -- the GPU parity suite's check over more random
paths than its fixed seeds reach.  Test infrastructure: the oracle is the checker only.

    python tools/parity_soak.py [--budget-s 240] [--width 96 --height 54 --spp 16] [--out gpurun_out/soak.json]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget-s", type=float, default=240.0)
    ap.add_argument("--width", type=int, default=96)
    ap.add_argument("--height", type=int, default=54)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--seed0", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from tests.oracle_lib import oracle_render
    from tests.test_gpu_parity import gpu_render

    t0 = time.time()
    cases, bad = [], []
    seed = a.seed0
    while time.time() - t0 < a.budget_s:
        for scene in SCENES:
            g = gpu_render(scene, a.width, a.height, a.spp, seed=seed)
            o = oracle_render(scene, a.width, a.height, a.spp, mode="pcg", seed=seed, threads=a.threads)
            ok = (np.array_equal(g["rgb"], o["rgb"]) and np.array_equal(g["acc"], o["acc"]) and g["segments"] == o["segments"])
            case = {"scene": scene, "seed": seed, "ok": ok, "segments": g["segments"]}
            if not ok:
                d = np.argwhere(np.any(g["acc"] != o["acc"], axis=-1))
                case.update(oracle_segments=o["segments"], pixels_differing=int(len(d)), first=d[:8].tolist())
                bad.append(case)
                print("MISMATCH", json.dumps(case), flush=True)
            cases.append(case)
        print(f"seed {seed}: {len(cases)} cases, {len(bad)} mismatches, {time.time() - t0:.0f} s", flush=True)
        seed += 1
    summary = {"frame": [a.width, a.height, a.spp], "seeds": [a.seed0, seed - 1], "cases": len(cases), "mismatches": bad,
               "segments": int(sum(c["segments"] for c in cases)), "seconds": round(time.time() - t0, 1)}
    print(json.dumps({k: v for k, v in summary.items()}), flush=True)
    if a.out:
        json.dump(summary, open(a.out, "w"), indent=1)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
