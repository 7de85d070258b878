"""Ray-query parity (rt_trace_rays vs the oracle's hittable_list::hit) — the BVH traversal one ray at a time.

The renderer's box tests are conservative f32 (padded boxes, widened interval) and its leaf tests exact f64, so the
closest hit must equal the reference's bit for bit: the same t and the same hit_record normal, for every ray.  Image
parity samples paths; here the rays are chosen to stress the f32 stage: camera-like rays, rays leaving the surfaces
they were found on (path continuations), axis-parallel rays (+-0 direction components, whose slab distances are
0 * inf), rays with components below the f32 range, and a ray a full-size render exposed (tests/test_gpu_full_size.py,
scene 8: a lambertian bounce off a ground box's top face with direction x exactly +0).
"""
import numpy as np
import pytest

import another_raytracer_amd as art
from another_raytracer_amd._lib import RT_GLOBAL_SCENE, check, lib
from tests.oracle_lib import oracle_trace_rays

pytestmark = pytest.mark.gpu

SCENES = ["1", "2", "4", "5", "6", "7", "8", "cow", "dino", "9", "c1"]


def gpu_trace(scene, rays, global_scene=False):
    import ctypes
    w = art.scene_manager().build(scene)
    rays = np.ascontiguousarray(rays, dtype=np.float64)
    t = np.zeros(len(rays), np.float64)
    nrm = np.zeros((len(rays), 3), np.float64)
    check(lib.rt_trace_rays(w.objects._native, rays.ctypes.data_as(ctypes.c_void_p), len(rays), RT_GLOBAL_SCENE if global_scene else 0,
                            t.ctypes.data_as(ctypes.c_void_p), nrm.ctypes.data_as(ctypes.c_void_p)), "rt_trace_rays")
    return t, nrm, w


def ray_sets(scene, n=4096, seed=7):
    """Camera-like rays, surface continuations, axis-parallel and tiny-component rays for one scene."""
    rng = np.random.default_rng(seed)
    w = art.scene_manager().build(scene)
    eye, at = np.array(w.lookfrom, float), np.array(w.lookat, float)
    span = max(1.0, float(np.linalg.norm(at - eye)))
    tm = rng.random(n)
    # camera-like: from around the eye towards around the target
    o1 = eye + rng.normal(0, 0.02 * span, (n, 3))
    d1 = (at + rng.normal(0, 0.35 * span, (n, 3))) - o1
    cam = np.column_stack([o1, d1, tm])
    # continuations: from the oracle's hit points, in random directions (unnormalised, like scatter directions)
    t, nrm = oracle_trace_rays(scene, cam)
    ok = np.isfinite(t)
    p = o1[ok] + t[ok, None] * d1[ok]
    nrm = nrm[ok]
    d2 = rng.normal(0, 1, (len(p), 3)) + rng.normal(0, 1, (len(p), 3))
    cont = np.column_stack([p, d2, tm[ok]])
    # axis-parallel: zero out one or two direction components (+0 or -0), from the same origins -- never the component
    # along the normal of an axis-aligned face the origin lies on: such a ray lies in the rect's plane, aarect.cpp gives
    # it t = 0/0 = NaN, and the reference then keeps whichever hit its own BVH order meets last (a NaN t_max accepts
    # every later hit).  No path makes one: a scattered ray leaves its surface (d . n > 0 or refracted through it).
    d3 = d2.copy()
    k = rng.integers(0, 3, len(d3))
    on_face = np.abs(nrm) == 1.0
    for _ in range(3):  # move k off the face-normal axis
        bad = on_face[np.arange(len(k)), k]
        k[bad] = (k[bad] + 1) % 3
    d3[np.arange(len(d3)), k] = np.where(rng.random(len(d3)) < 0.5, 0.0, -0.0)
    k2 = (k + 1) % 3
    two = (rng.random(len(d3)) < 0.3) & ~on_face[np.arange(len(k2)), k2]
    d3[np.arange(len(d3))[two], k2[two]] = 0.0
    axis = np.column_stack([p, d3, tm[ok]])
    # components far below the f32 range (the f32 conversion underflows to 0 or a denormal)
    d4 = d2.copy()
    d4[np.arange(len(d4)), k] = rng.choice([1e-300, -1e-300, 1e-40, -1e-42, 5e-324], len(d4))
    tiny = np.column_stack([p, d4, tm[ok]])
    return np.concatenate([cam, cont, axis, tiny])


def assert_same_hits(scene, rays, global_scene=False):
    t_o, n_o = oracle_trace_rays(scene, rays)
    t_g, n_g, _ = gpu_trace(scene, rays, global_scene)
    # bit patterns, except that any NaN equals any NaN: the reference's rect test accepts t = 0/0 for a ray lying in the
    # rect's plane (aarect.cpp: NaN fails both range tests), and the GPU must too, but x86 and gfx950 give 0/0
    # different NaN sign bits
    def same(a, b):
        return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    bad = np.flatnonzero(~same(t_g, t_o) | ~np.all(same(n_g, n_o), axis=1))
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{scene}: {len(bad)} of {len(rays)} rays differ; first ray {rays[i].tolist()}: gpu t {t_g[i]!r} n {n_g[i]} "
                             f"oracle t {t_o[i]!r} n {n_o[i]}")


@pytest.mark.parametrize("scene", SCENES)
def test_closest_hit_matches_reference(gpu, scene):
    assert_same_hits(scene, ray_sets(scene))


def test_lds_and_hbm_traversals_agree_with_reference(gpu):
    rays = ray_sets("1", n=8192, seed=11)
    assert_same_hits("1", rays, global_scene=False)
    assert_same_hits("1", rays, global_scene=True)


def test_full_size_regression_ray(gpu):
    # scene 8, pixel (405, 1137), sample 1188 of the 1920x1080 frame, bounce 2: the ray leaves a ground box's top face
    # with direction x exactly +0 and hits the neighbouring box's +z face at t = 24.6
    bits = ["c0712581e2c7e73b", "403f2ec7727e4590", "406a0c4a697eb584", "0000000000000000", "3faea24713365ea0", "bfd5ce3471b3f835",
            "3fec46c4a0000000"]
    ray = np.array([[np.frombuffer(bytes.fromhex(b)[::-1], np.float64)[0] for b in bits]])
    assert_same_hits("8", ray)
