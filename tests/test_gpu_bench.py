"""bench.py's output contract on a small frame (the driver parses this line at round end): one JSON line with the
metric, value, unit, n_gpus, steps, warmup, ms_per_step, higher_is_better, scaling, vs_baseline, dtype, data and
config fields, plus the roofline object of the dominant kernel; value = segments / wall time."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("scene,variant,kernel", [("1", 3, "k_paths"), ("cow", 4, "k_paths_g")])
def test_bench_line_contract(gpu, scene, variant, kernel):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--scene", scene, "--width", "96", "--height", "54",
                          "--spp", "8", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and d["unit"] == "Msamples/s" and d["value"] > 0
    c = d["config"]
    assert (c["width"], c["height"], c["spp"]) == (96, 54, 8) and c["primary_rays_per_step"] == 96 * 54 * 8
    assert c["segments_per_step"] >= c["primary_rays_per_step"]
    # value is the whole job's segments over the timed wall time
    assert d["value"] == pytest.approx(c["segments_per_step"] * d["steps"] / (d["ms_per_step"] * d["steps"] * 1e3), rel=2e-3)
    assert c["driver"] == "multi" and "rt_render_multi" in c["parallelism"]
    r = d["roofline"]
    assert r["kernel"] == kernel and r["extend_variant"] == variant and r["launches"] == 2 and r["devices"] == 1
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0 and r["avg_launch_ms"] > 0
    # achieved = the algorithmic bytes of one launch over its measured duration
    assert r["achieved"] == pytest.approx(r["algorithmic_bytes_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3, abs=1e-6)
    assert r["segments_per_launch"] == c["segments_per_step"]
