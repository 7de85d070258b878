"""Scene-compile restructurings switched off (ART_WORLD_MERGE=0, ART_HOIST=0: read once per process, so each case runs
in a child process): the world stays the reference's hittable_list of loose primitives, which must (a) not take the
LDS k_paths kernel -- it shades hits by LDS leaf slot, so a loose OBJ_PRIM object would be shaded with another
object's material (kernels.hip lds_scene_image) -- and (b) still equal the oracle bit for bit, as it does
with the restructurings on (tests/test_gpu_parity.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from tests.test_gpu_parity import gpu_render
from tests.oracle_lib import oracle_render
scene, W, H, spp = sys.argv[2], 64, 36, 8
g = gpu_render(scene, W, H, spp)
o = oracle_render(scene, W, H, spp, mode="pcg")
print(json.dumps({"variant": g["stats"]["extend_variant"], "rgb": bool(np.array_equal(g["rgb"], o["rgb"])),
                  "acc": bool(np.array_equal(g["acc"], o["acc"])), "segments": [g["segments"], o["segments"]]}))
"""


@pytest.mark.parametrize("scene,env", [("c1", {"ART_WORLD_MERGE": "0"}), ("2", {"ART_WORLD_MERGE": "0"}),
                                       ("1", {"ART_HOIST": "0"}), ("c1", {"ART_WORLD_MERGE": "1"})])
def test_unmerged_worlds_match_oracle(gpu, scene, env):
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, scene], capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env={**os.environ, **env})
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["rgb"] and d["acc"] and d["segments"][0] == d["segments"][1], d
    if env.get("ART_WORLD_MERGE") == "0":
        assert d["variant"] != 3, "a world of loose primitives must not take the LDS-slot-shaded k_paths"
