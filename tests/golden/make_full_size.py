"""Full-size parity fixtures aimed at the geometry: the oracle's (oracle/restate.cpp, pcg mode: the product's RNG
contract) render of rows chosen THROUGH the objects that stress the HIP path -- the mesh silhouettes (conservative f32
box tests, split-BVH duplicate references, LM 2 partial-LDS node fetches), the Next-Week box field and its media --
at each BASELINE GPU config's full width, height and spp.

    python tests/golden/make_full_size.py [1|cow|8|dino ...]      (build container; ~5 min on 8 threads)

Rows are chosen from primary-ray classification (oracle_trace_rays through pixel centres: a triangle hit is one whose
hit_record normal is not unit length, triangle.h:32,82 -- SURVEY Q1) and from the projection of the final scene's
objects (scene_manager.cpp:171-234: the fog sphere at (360,150,145) r 70, the 1000-sphere cluster, the box field).
Written per config: tests/golden/fullsize_<scene>.npz = rows, RGB8 of those rows, the SHA-256 of every row's f64
radiance sums (W x 3 little-endian doubles; the sums themselves are 24 B per pixel, too large to commit) and the
oracle's segment count over the rows.  tests/test_gpu_full_size.py compares the GPU's whole frame with them bit for bit.
Everything written is DATA produced by the committed oracle."""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# scene, W, H, spp, rows to select
CONFIGS = {"1": (1920, 1080, 1024, 24), "cow": (1920, 1080, 512, 24), "8": (1920, 1080, 4096, 16), "dino": (4096, 4096, 8192, 48)}


def view(scene):
    import another_raytracer_amd as art
    w = art.scene_manager().build(scene)
    return np.array(w.lookfrom), np.array(w.lookat), float(w.vfov)


def basis(frm, at, vfov, aspect):
    """camera.h:8-36 (pinhole: the lens offset does not move which object a pixel centre sees)."""
    h = np.tan(np.radians(vfov) / 2)
    w = (frm - at) / np.linalg.norm(frm - at)
    u = np.cross([0.0, 1.0, 0.0], w)
    u /= np.linalg.norm(u)
    v = np.cross(w, u)
    hor, ver = 10.0 * 2 * h * aspect * u, 10.0 * 2 * h * v
    llc = frm - hor / 2 - ver / 2 - 10.0 * w
    return llc, hor, ver, (u, v, w, h)


def primary_rays(scene, W, H, rows, cols):
    frm, at, vfov = view(scene)
    llc, hor, ver, _ = basis(frm, at, vfov, W / H)
    jj, ii = np.meshgrid(rows, cols, indexing="ij")
    s = (ii + 0.5) / (W - 1)
    t = ((H - 1 - jj) + 0.5) / (H - 1)
    d = llc[None, None] + s[..., None] * hor + t[..., None] * ver - frm
    rays = np.zeros(d.shape[:2] + (7,))
    rays[..., :3] = frm
    rays[..., 3:6] = d
    rays[..., 6] = 0.5
    return rays.reshape(-1, 7)


def triangle_rows(scene, W, H, n, probe_rows=512, probe_cols=256):
    """n rows spread evenly over the rows whose pixel centres hit the mesh (non-unit hit normals)."""
    from tests.oracle_lib import oracle_trace_rays
    rows = np.unique(np.linspace(0, H - 1, min(probe_rows, H)).astype(int))
    cols = np.linspace(0, W - 1, probe_cols).astype(int)
    t, nrm = oracle_trace_rays(scene, primary_rays(scene, W, H, rows, cols))
    tri = np.isfinite(t) & (np.abs(np.linalg.norm(nrm, axis=1) - 1.0) > 1e-9)
    cover = tri.reshape(len(rows), len(cols)).mean(axis=1)
    hit_rows = rows[cover > 0.02]
    lo, hi = int(hit_rows.min()), int(hit_rows.max())
    # evenly over [lo, hi] (every row in the span is probed at 1/(H/probe_rows) density; covered spans are contiguous)
    pick = np.unique(np.linspace(lo, hi, n).round().astype(int))
    return pick, (lo, hi), float(cover.max())


def project_rows(scene, W, H, centre, radius):
    """Image rows spanned by a sphere (projected centre +- projected radius, pinhole)."""
    frm, at, vfov = view(scene)
    _, _, _, (u, v, w, h) = basis(frm, at, vfov, W / H)
    d = np.asarray(centre, float) - frm
    depth = -d @ w
    tc = 0.5 + (d @ v) / depth / (2 * h)
    dt = radius / depth / (2 * h)
    r0 = int(np.clip(np.floor((H - 1) * (1 - (tc + dt))), 0, H - 1))
    r1 = int(np.clip(np.ceil((H - 1) * (1 - (tc - dt))), 0, H - 1))
    return r0, r1


def final_rows(W, H, n):
    """Next-Week final (scene_manager.cpp:171-234): rows through the box field, the r 70 fog sphere and the sphere
    cluster, n in total."""
    from tests.oracle_lib import oracle_trace_rays
    scene = "8"
    rows = np.arange(0, H, 4)
    cols = np.linspace(0, W - 1, 256).astype(int)
    rays = primary_rays(scene, W, H, rows, cols)
    t, nrm = oracle_trace_rays(scene, rays)
    p = rays[:, :3] + t[:, None] * rays[:, 3:6]
    box = np.isfinite(t) & (p[:, 1] < 101.5) & (np.abs(np.abs(nrm).max(axis=1) - 1.0) < 1e-12)
    cover = box.reshape(len(rows), len(cols)).mean(axis=1)
    field = rows[cover > 0.5]
    fog = project_rows(scene, W, H, (360, 150, 145), 70)          # constant_medium(sphere((360,150,145), 70), 0.2)
    cluster = project_rows(scene, W, H, (-100 + 82.5, 270 + 82.5, 395 + 82.5), 100)  # translate(rotate_y(bvh(1000 spheres)))
    k = n // 3
    pick = set(np.linspace(field.min(), field.max(), n - 2 * k).round().astype(int))
    pick |= set(np.linspace(fog[0], fog[1], k + 2)[1:-1].round().astype(int))
    pick |= set(np.linspace(cluster[0], cluster[1], k + 2)[1:-1].round().astype(int))
    return np.array(sorted(pick)), {"box_field": (int(field.min()), int(field.max())), "fog_sphere": fog, "sphere_cluster": cluster}


def random_rows(W, H, n):
    """The headline scene (scene_manager.cpp:13-64, alias 1): rows through the three r = 1 spheres (dielectric at
    (0,1,0), lambertian at (-4,1,0), metal at (4,1,0): the LDS image's per-slot f64 leaf tests and the dielectric
    table) and through the field of small spheres, where the static and moving (Q2 duplicate) balls stand -- the
    moving ones' per-slot dy -- n in total."""
    from tests.oracle_lib import oracle_trace_rays
    scene = "1"
    big = [project_rows(scene, W, H, c, 1.0) for c in ((0, 1, 0), (-4, 1, 0), (4, 1, 0))]
    rows = np.arange(0, H, 4)
    cols = np.linspace(0, W - 1, 256).astype(int)
    rays = primary_rays(scene, W, H, rows, cols)
    t, _ = oracle_trace_rays(scene, rays)
    p = rays[:, :3] + t[:, None] * rays[:, 3:6]
    near_big = np.zeros(len(p), bool)
    for c in ((0, 1, 0), (-4, 1, 0), (4, 1, 0)):
        near_big |= np.linalg.norm(p - np.asarray(c, float), axis=1) < 1.0 + 1e-6
    small = np.isfinite(t) & (p[:, 1] > 0.01) & ~near_big  # not the r = 1000 ground (p.y ~ 0), not the big three
    cover = small.reshape(len(rows), len(cols)).mean(axis=1)
    k = n // 6
    pick = set()
    for r0, r1 in big:
        pick |= set(np.linspace(r0, r1, k + 2)[1:-1].round().astype(int))
    field = rows[np.argsort(-cover)[: 4 * (n - len(pick))]]
    pick |= set(np.linspace(field.min(), field.max(), n - len(pick)).round().astype(int))
    return np.array(sorted(pick)), {"big_spheres": big, "small_sphere_rows": (int(field.min()), int(field.max())),
                                    "peak_small_cover": float(cover.max())}


def row_hashes(acc):
    return np.array([hashlib.sha256(np.ascontiguousarray(r, dtype="<f8").tobytes()).hexdigest() for r in acc])


def make(scene):
    from tests.oracle_lib import oracle_render_rows
    W, H, spp, n = CONFIGS[scene]
    if scene == "8":
        rows, where = final_rows(W, H, n)
    elif scene == "1":
        rows, where = random_rows(W, H, n)
    else:
        rows, span, peak = triangle_rows(scene, W, H, n)
        where = {"mesh_rows": span, "peak_row_coverage": peak}
    t0 = time.time()
    o = oracle_render_rows(scene, W, H, spp, rows, threads=os.cpu_count())
    out = os.path.join(HERE, f"fullsize_{scene}.npz")
    np.savez_compressed(out, rows=rows.astype(np.int32), rgb=o["rgb"], acc_sha256=row_hashes(o["acc"]),
                        segments=np.int64(o["segments"]), W=W, H=H, spp=spp)
    print(f"{scene}: {len(rows)} rows ({100.0 * len(rows) / H:.2f} % of the frame) {where}, {o['segments']} segments, "
          f"{time.time() - t0:.0f} s -> {out}", flush=True)


if __name__ == "__main__":
    for sc in sys.argv[1:] or list(CONFIGS):
        make(sc)
