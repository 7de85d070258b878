"""Locate where the GPU and the oracle part ways on one scene's sampled rows (diagnostic, GPU box).

    python tools/diag_rows.py SCENE W H SPP STRIDE [MAX_PIXELS]

Renders the rows 0, STRIDE, 2*STRIDE, ... (band partition (1, STRIDE, 0)) on the GPU and with the oracle (pcg mode),
lists the pixels whose RGB8 or f64 sums differ, and for the first MAX_PIXELS of them bisects the sample count: the
smallest k such that the k-sample renders of that row already differ is the first diverging sample (index k - 1) of
the pixel, because samples are keyed by (pixel, sample index) and summed in order.  Prints one JSON line per pixel.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.oracle_lib import oracle_render_rows  # noqa: E402
from tests.test_gpu_parity import gpu_render  # noqa: E402


def threads():
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else min(16, os.cpu_count() or 4)


def main():
    scene, W, H, spp, stride = sys.argv[1], *map(int, sys.argv[2:6])
    maxpix = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    rows = np.arange(0, H, stride)
    g = gpu_render(scene, W, H, spp, band=(1, stride, 0))
    o = oracle_render_rows(scene, W, H, spp, rows, threads=threads())
    bad = np.argwhere(np.any(g["acc"] != o["acc"], axis=-1))
    rgb_bad = int(np.sum(np.any(g["rgb"] != o["rgb"], axis=-1)))
    print(json.dumps({"scene": scene, "rows": len(rows), "segments_gpu": g["segments"], "segments_oracle": o["segments"],
                      "acc_mismatch_pixels": len(bad), "rgb_mismatch_pixels": rgb_bad}), flush=True)
    for k, j in bad[:maxpix]:
        y = int(rows[k])
        lo, hi = 1, spp  # invariant: the spp=hi renders differ at pixel (y, j), the spp=lo-1 ones agree
        while lo < hi:
            mid = (lo + hi) // 2
            gm = gpu_render(scene, W, H, mid, band=(1, stride, 0))["acc"][k, j]
            om = oracle_render_rows(scene, W, H, mid, [y], threads=threads())["acc"][0, j]
            if np.array_equal(gm, om):
                lo = mid + 1
            else:
                hi = mid
        gk = gpu_render(scene, W, H, lo, band=(1, stride, 0))["acc"][k, j]
        ok = oracle_render_rows(scene, W, H, lo, [y], threads=threads())["acc"][0, j]
        print(json.dumps({"pixel": [y, int(j)], "first_diverging_sample": lo - 1, "gpu_sum": gk.tolist(), "oracle_sum": ok.tolist(),
                          "gpu_rgb": g["rgb"][k, j].tolist(), "oracle_rgb": o["rgb"][k, j].tolist()}), flush=True)


if __name__ == "__main__":
    main()
