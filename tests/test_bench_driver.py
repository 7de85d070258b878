"""bench.py's choice of multi-GPU driver (CPU): `--gpus N` without torchrun drives N GPUs in one process through
rt_render_multi, under torchrun WORLD_SIZE must equal --gpus, and fewer visible GPUs than asked is an error -- the
bench never silently measures one GPU and labels it N."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plain_run_drives_n_gpus_in_one_process():
    assert bench.choose_driver(None, 1, 1) == ("multi", 1)
    assert bench.choose_driver(1, 1, 8) == ("multi", 1)
    assert bench.choose_driver(8, 1, 8) == ("multi", 8)
    assert bench.choose_driver(2, 1, 8) == ("multi", 2)


@pytest.mark.parametrize("gpus,visible", [(2, 1), (8, 4), (1, 0)])
def test_too_few_gpus_fails_loudly(gpus, visible):
    with pytest.raises(SystemExit, match=f"needs {gpus} visible GPUs, found {visible}"):
        bench.choose_driver(gpus, 1, visible)


def test_torchrun_world_must_match_gpus():
    assert bench.choose_driver(4, 4, 8) == ("procs", 4)
    assert bench.choose_driver(None, 4, 8) == ("procs", 4)
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.choose_driver(8, 4, 8)
    # one torchrun rank (WORLD_SIZE 1) is the per-process driver too: the A/B switches (--global-scene ...) need it
    assert bench.choose_driver(None, 1, 1, torchrun=True) == ("procs", 1)
    assert bench.choose_driver(1, 1, 8, torchrun=True) == ("procs", 1)


def test_bench_exits_nonzero_without_the_gpus():
    # this container has no GPU: asking for 2 must end with an error, not a 1-GPU (or 0-GPU) line
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], capture_output=True,
                       text=True, timeout=300, cwd=ROOT, env=env)
    if r.returncode == 0:
        pytest.fail("bench.py --gpus 2 succeeded on a box without 2 GPUs")
    assert "needs 2 visible GPUs" in r.stderr and not r.stdout.strip()


def test_roofline_prices_the_slowest_gpu():
    # two GPUs: the slower one's launches set the roofline (SURVEY §8(d) bytes of its own launches / its launch time)
    devs = [{"segments": 4_000_000, "primary": 1_000_000, "extend_ms": 20.0, "extend_launches": 2, "local_rows": 100, "steps": 2},
            {"segments": 6_000_000, "primary": 1_000_000, "extend_ms": 30.0, "extend_launches": 2, "local_rows": 100, "steps": 2}]
    r = bench.roofline_of(devs, 100, 1000, 3, "f64", "1", "no-such-build")
    segs, pix = 3_000_000, 100 * 100
    alg = 128 * segs + 12 * pix + 1000
    assert r["algorithmic_bytes_per_launch"] == alg and r["avg_launch_ms"] == 15.0 and r["devices"] == 2
    assert r["achieved"] == pytest.approx(alg / 15e-3 / 1e9, rel=1e-4)
    assert r["bound"] == "hbm" and r["frac"] == pytest.approx(r["achieved"] / 8000.0, rel=1e-4)
    assert r["traffic"] is None and "valu" not in r  # no summary of this build
