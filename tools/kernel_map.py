"""Which persistent-path kernel each builtin scene runs (rt_stats.kernel_features / kernel_textures / kernel_lds_mode),
with that instantiation's registers and spills from libart.so's code-object metadata (tools/kernel_resources.py).

    python tools/kernel_map.py [--json OUT]      (GPU box: renders each scene once at 32x18x1)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

SCENES = ["c1", "1", "2", "3", "4", "5", "6", "7", "8", "cow", "dino", "9"]


def kernel_map():
    import numpy as np
    import another_raytracer_amd as art
    out = {}
    for s in SCENES:
        w = art.scene_manager().build(s)
        cam = art.camera(w.lookfrom, w.lookat, (0, 1, 0), w.vfov, 32 / 18, w.aperture, 10.0, 0.0, 1.0)
        e = art.engine(cam, art.engine_mode.single, width=32, height=18, samples_per_pixel=1)
        e.set_scene(w.objects, w.background)
        e.run(np.zeros((18, 32, 3), np.uint8))
        st = e.stats
        out[s] = (st["kernel_features"], st["kernel_textures"], st["kernel_lds_mode"])
    return out


def resources(lib):
    from kernel_resources import code_objects, fatbin, kernel_metadata
    res = {}
    for co in code_objects(fatbin(lib)):
        for k in kernel_metadata(co):
            res[k[".name"]] = k
    return res


def symbol(f, tf, lm):
    """Mangled name of k_paths_g<f, tf, lm> (k_paths for LDS mode 3)."""
    if lm == 3:
        return "_ZN3art7k_pathsENS_8DevSceneIdEENS_8PassGeomENS_9CameraRecIdEENS_4WorkIdEEPj"
    return f"_ZN3art9k_paths_gILj{f}ELj{tf}ELi{lm}EEEvNS_8DevSceneIdEENS_8PassGeomENS_9CameraRecIdEENS_4WorkIdEEPj"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from another_raytracer_amd._lib import LIB_PATH
    m = kernel_map()
    res = resources(LIB_PATH)
    rows = []
    for s, (f, tf, lm) in m.items():
        k = res.get(symbol(f, tf, lm), {})
        rows.append({"scene": s, "features": f, "textures": tf, "lds_mode": lm, "vgpr": k.get(".vgpr_count"),
                     "vgpr_spill": k.get(".vgpr_spill_count"), "sgpr_spill": k.get(".sgpr_spill_count")})
        print(f"{s:5s} k_paths_g<{f},{tf},{lm}>  vgpr {k.get('.vgpr_count')} spill {k.get('.vgpr_spill_count')} "
              f"sgpr_spill {k.get('.sgpr_spill_count')}" if lm != 3 else f"{s:5s} k_paths  vgpr {k.get('.vgpr_count')}")
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
