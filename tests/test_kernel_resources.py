"""Occupancy budgets of the persistent path kernels, read from the gfx950 code objects inside libart.so
(tools/kernel_resources.py: the offload bundles of `.hip_fatbin`, the NT_AMDGPU_METADATA note).  DESIGN.md §4's bound
analysis assumes them, so a source change that breaks one shows up here, on the CPU, before any GPU run:
  * k_paths: at most 128 VGPRs and no spills -> 4 waves per SIMD (16 waves of its one 1024-lane block per CU);
  * k_paths_g: at most 168 VGPRs -> 3 waves per SIMD (ART_PATHS_G_WAVES);
  * the mesh kernels with solid/checker textures (cow, dino: F_CODE16 | kFeatMesh, kTexBasic) spill nothing in
    LM 1 (dino) and at most a few registers elsewhere;
  * every LM 1 kernel with 16-bit codes spills nothing -- the Next-Week final's <189, 15, 1> among them (54 spilled
    VGPRs before csrc/sphere_uv.h replaced the device library's acos / atan2, whose hoisted constants were the spills);
  * SCENE_KERNELS: the persistent kernel each builtin scene runs (rt_stats.kernel_*; tests/test_gpu_parity.py checks the
    map on the GPU, tools/kernel_map.py prints it) spills no VGPR, except the capsule's textured LM 2 mesh kernel
    (10 VGPRs the allocator parks around the path start; 20 in r5's TF_ALL kernel: profiles/r5b_ab_instantiations.txt)."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernel_resources  # noqa: E402

LIB = os.path.join(ROOT, "another_raytracer_amd", "libart.so")


@pytest.fixture(scope="module")
def ks():
    if not os.path.exists(LIB):
        pytest.skip("libart.so not built")
    return kernel_resources.kernels(LIB)


def _paths_g(ks):
    out = {}
    for name, k in ks.items():
        m = re.match(r"_ZN3art9k_paths_gILj(\d+)ELj(\d+)ELi(\d)E", name)
        if m:
            out[tuple(int(x) for x in m.groups())] = k
    return out


# scene -> (features, textures, LDS mode) of the persistent kernel it runs: k_paths_g<F, TF, LM>, k_paths = (1, 0, 3)
SCENE_KERNELS = {
    "c1": (1, 0, 3), "1": (1, 0, 3), "2": (1, 0, 3), "3": (129, 15, 1), "4": (129, 15, 1), "5": (165, 15, 1), "6": (189, 15, 1),
    "7": (125, 3, 1), "8": (189, 15, 1), "cow": (167, 3, 2), "dino": (167, 3, 1), "9": (423, 19, 2),
}
# the capsule (scene 9, the reference's default; F_LEAF2 | F_CODE16 mesh kernel, barycentric-image textures): 10 VGPRs,
# path-start values only (r5's F_ALL-texture kernel spilled 20)
SPILL_ALLOWED = {(423, 19, 2): 10}


def test_every_kernel_a_builtin_scene_runs_is_spill_free(ks):
    pg = _paths_g(ks)
    for scene, key in SCENE_KERNELS.items():
        if key[2] == 3:
            continue
        assert key in pg, (scene, key)
        spilled = pg[key].get(".vgpr_spill_count", 0)
        assert spilled <= SPILL_ALLOWED.get(key, 0), (scene, key, spilled)
        assert pg[key][".vgpr_count"] + pg[key].get(".agpr_count", 0) <= 168, (scene, key)


def test_every_code_object_is_gfx950_and_has_the_path_kernels(ks):
    assert any(n.startswith("_ZN3art7k_paths") for n in ks)
    assert len(_paths_g(ks)) >= 9
    assert any("k_unpack_bands" in n for n in ks)  # multi.hip's object too


def test_k_paths_keeps_four_waves_per_simd(ks):
    k = next(v for n, v in ks.items() if n.startswith("_ZN3art7k_paths"))
    assert k[".vgpr_count"] <= 128, k[".vgpr_count"]
    assert k.get(".agpr_count", 0) == 0
    assert k.get(".vgpr_spill_count", 0) == 0
    assert k[".max_flat_workgroup_size"] == 1024


def test_k_paths_g_keeps_three_waves_per_simd(ks):
    for key, k in _paths_g(ks).items():
        assert k[".vgpr_count"] + k.get(".agpr_count", 0) <= 168, (key, k[".vgpr_count"])


def test_mesh_kernels_do_not_spill(ks):
    F_CODE16, kFeatMesh, kTexBasic = 128, 1 | 2 | 4 | 32, 1 | 2
    pg = _paths_g(ks)
    assert pg[(F_CODE16 | kFeatMesh, kTexBasic, 1)].get(".vgpr_spill_count", 0) == 0  # dino (LM 1)
    for lm in (0, 2):  # cow (LM 2), larger meshes (LM 0)
        assert pg[(F_CODE16 | kFeatMesh, kTexBasic, lm)].get(".vgpr_spill_count", 0) <= 8


def test_lm1_code16_kernels_do_not_spill(ks):
    F_CODE16 = 128
    pg = _paths_g(ks)
    assert (189, 15, 1) in pg  # the final scene's kernel (scene 8: all features, all textures, LDS BVH)
    spills = {key: k.get(".vgpr_spill_count", 0) for key, k in pg.items() if key[2] == 1 and key[0] & F_CODE16}
    assert spills and all(v <= SPILL_ALLOWED.get(key, 0) for key, v in spills.items()), spills
