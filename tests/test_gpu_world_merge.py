"""Scene-compile restructurings switched off (options compile.world_merge = 0 / 1, compile.hoist = 0, which apply to
scenes compiled after they are set): the world stays the reference's hittable_list of loose primitives, which must (a)
not take the LDS k_paths kernel -- it shades hits by LDS leaf slot, so a loose OBJ_PRIM object would be shaded with
another object's material (kernels.hip lds_scene_image) -- and (b) still equal the oracle bit for bit, as it
does with the restructurings on (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from tests.oracle_lib import oracle_render
from tests.test_gpu_parity import gpu_render

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene,opts", [("c1", {"compile.world_merge": 0}), ("2", {"compile.world_merge": 0}),
                                        ("1", {"compile.hoist": 0}), ("c1", {"compile.world_merge": 1})])
def test_unmerged_worlds_match_oracle(gpu, options, scene, opts):
    for k, v in opts.items():
        options(k, v)
    W, H, spp = 64, 36, 8
    g = gpu_render(scene, W, H, spp)
    o = oracle_render(scene, W, H, spp, mode="pcg")
    assert np.array_equal(g["rgb"], o["rgb"]) and np.array_equal(g["acc"], o["acc"]) and g["segments"] == o["segments"]
    if opts.get("compile.world_merge") == 0:
        assert g["stats"]["extend_variant"] != 3, "a world of loose primitives must not take the LDS-slot-shaded k_paths"
