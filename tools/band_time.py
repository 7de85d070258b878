"""Per-rank frame time of the row-band partition on one GPU: renders rank r's bands of an N-way split (band_count N,
band_index r) of the benchmark frame and prints ms and Msamples/s, so the strong-scaling ceiling of bench.py --gpus N
(max over ranks of these times, plus the gather) can be read off a 1-GPU box.
    python tools/band_time.py [--scene 1 --spp 1024 --counts 1,2,4,8]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="1")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--counts", default="1,2,4,8")
    ap.add_argument("--band-rows", type=int, default=8)
    args = ap.parse_args()
    import torch
    import another_raytracer_amd as art
    from another_raytracer_amd.distributed import band_rows_of
    w = art.scene_manager(device=0).build(args.scene)
    cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, args.width / args.height, w.aperture, 10.0, 0.0, 1.0)
    eng = art.engine(cam, art.engine_mode.parallel_stripes, width=args.width, height=args.height,
                     samples_per_pixel=args.spp, max_depth=50, device=0)
    eng.set_scene(w.objects, w.background)
    for n in (int(x) for x in args.counts.split(",")):
        for r in sorted({0, n - 1}):
            rows = band_rows_of(args.height, args.band_rows, n, r)
            out = torch.empty((len(rows), args.width, 3), dtype=torch.uint8, device="cuda:0")
            eng.run(out, band_rows=args.band_rows, band_count=n, band_index=r)  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.run(out, band_rows=args.band_rows, band_count=n, band_index=r)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            segs = eng.stats["segments"]
            print(json.dumps({"gpus": n, "rank": r, "rows": len(rows), "ms": round(ms, 2),
                              "msamples_s": round(segs / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
