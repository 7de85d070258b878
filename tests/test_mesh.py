"""OBJ/MTL ingestion (another_raytracer_amd/csrc/objmesh.cpp, the reference's mesh class, mesh.h:29-145) against the
reference's own post-triangulation triangle lists (oracle/ref_harness `mesh`: rapidobj v1.0.1 ParseFile + Triangulate
+ mesh::build, compiled from /root/reference), committed as fixtures:
  assets/{cow,dino,capsule}.tris        the reference models (capsule: map_Kd texture coordinates too)
  tests/golden/obj/{shapes,plain}.tris  synthetic meshes covering quads on both diagonals, concave 6/7-gons (earcut),
                                        a tilted pentagon, negative and v//vn indices, g/o shapes, two MTL materials
Host-only: no GPU needed."""
import ctypes
import json
import os

import numpy as np
import pytest

import another_raytracer_amd as art
from another_raytracer_amd._lib import lib
from another_raytracer_amd.scene import _SceneHandle, scene_dump

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(ROOT, "assets")
OBJ = os.path.join(ROOT, "tests", "golden", "obj")
MESHES = {
    "cow": (os.path.join(ASSETS, "models", "cow.obj"), os.path.join(ASSETS, "cow.tris")),
    "dino": (os.path.join(ASSETS, "models", "dino.obj"), os.path.join(ASSETS, "dino.tris")),
    "capsule": (os.path.join(ASSETS, "models", "capsule", "capsule.obj"), os.path.join(ASSETS, "capsule.tris")),
    "shapes": (os.path.join(OBJ, "shapes.obj"), os.path.join(OBJ, "shapes.tris")),
    "plain": (os.path.join(OBJ, "plain.obj"), os.path.join(OBJ, "plain.tris")),
}


def read_tris(path):
    raw = open(path, "rb").read()
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    pos = np.frombuffer(raw[4:4 + 36 * n], np.float32).reshape(n, 9)
    col = np.frombuffer(raw[4 + 36 * n:4 + 60 * n], np.float64).reshape(n, 3)
    rest = raw[4 + 60 * n:]
    uv = np.frombuffer(rest, np.float64).reshape(n, 6) if rest else None
    return pos, col, uv


def mesh_as_list(obj_path):
    """mesh::build into a fresh graph, the triangles kept in order in one hittable_list, dumped."""
    g = lib.rt_graph_new()
    try:
        first = ctypes.c_int()
        n = lib.rt_mesh_build(g, obj_path.encode(), ctypes.byref(first))
        assert n > 0, lib.rt_last_error()
        ids = (ctypes.c_int * n)(*range(first.value, first.value + n))
        lst = lib.rt_obj_list(g, n, ids)
        assert lib.rt_graph_add_world(g, lst) >= 0
        out = ctypes.c_void_p()
        assert lib.rt_graph_compile(g, 0, ctypes.byref(out)) == 0, lib.rt_last_error()
        h = _SceneHandle(out)
        size = lib.rt_scene_dump(h, None, 0)
        buf = ctypes.create_string_buffer(size)
        lib.rt_scene_dump(h, buf, size)
        return json.loads(buf.value.decode())["objects"][0]["items"]
    finally:
        lib.rt_graph_free(g)


@pytest.mark.parametrize("name", list(MESHES))
def test_triangles_match_the_reference_mesh_build(name):
    obj, tris = MESHES[name]
    pos, col, uv = read_tris(tris)
    items = mesh_as_list(obj)
    assert len(items) == len(pos)
    mine = np.array([[c for p in it["p"] for c in p] for it in items])
    # f32 OBJ values widened to f64 (mesh.h:76-82): bit-exact, in the reference's triangle order
    assert np.array_equal(mine, pos.astype(np.float64))
    texs = [it["mat"]["tex"] for it in items]
    if uv is None:  # solid albedo: color::random() per triangle (no MTL) or Ka + Kd in f32 (MTL)
        assert np.array_equal(np.array([t["c"] for t in texs]), col)
    else:  # barycentric_image_texture over the map_Kd image
        assert all(t["type"] == "bary_image" for t in texs)
        got = np.array([[*t["a"], *t["b"], *t["c"]] for t in texs])
        assert np.array_equal(got, uv)


def test_counts_and_parse_like_mesh_parse():
    m = art.mesh()
    assert m.parse(MESHES["cow"][0]) and (m.triangles, m.shapes) == (5804, 172)  # 172 shapes, 5804 tris
    assert m.parse(MESHES["capsule"][0]) and m.triangles == 10200
    assert not art.mesh().parse(os.path.join(OBJ, "missing.obj"))


def test_python_mesh_build_consumes_the_reference_draws():
    """mesh::build draws one color::random() per triangle, then bvh_node its per-node draws (scene_manager.cpp:236-244):
    the Python mirror reproduces the reference's cow scene graph and its RNG state."""
    art.reset_scene_rng()
    m = art.mesh()
    assert m.parse(MESHES["cow"][0])
    world = art.hittable_list()
    world.add(art.bvh_node(m.build(), 0.0, 1.0))
    world.add(art.xz_rect(123, 423, 147, 412, 554, art.diffuse_light((7, 7, 7))))
    world.add(art.constant_medium(art.sphere((0, 0, 0), 5000, art.dielectric(1.5)), .0001, (1, 1, 1)))
    probe = [art.random_double() for _ in range(8)]
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "scenes.json")))["cow"]
    assert probe == gold["probe"]
    art.reset_scene_rng()


def test_scene_9_is_the_textured_capsule():
    w = art.scene_manager().build(art.scene_alias.mesh)
    assert w.info["triangles"] == 10200 and w.info["has_media"] == 1
    assert (w.lookfrom, w.lookat, w.vfov) == ((2.0, 2.0, 1.0), (0.0, 0.0, 0.0), 75.0)
    assert '"type":"bary_image"' in scene_dump(w)


def test_bad_obj_files_fail_loudly(tmp_path):
    cases = {
        "zero_index.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",
        "out_of_range.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n",
        "two_vertex_face.obj": "v 0 0 0\nv 1 0 0\nf 1 2\n",
        "missing_mtl.obj": "mtllib nowhere.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl x\nf 1 2 3\n",
        "unknown_material.obj": "mtllib shapes.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl blue\nf 1 2 3\n",
        "degenerate_pentagon.obj": "v 0 0 0\nv 0 0 0\nv 0 0 0\nv 0 0 0\nv 0 0 0\nf 1 2 3 4 5\n",
    }
    (tmp_path / "shapes.mtl").write_bytes(open(os.path.join(OBJ, "shapes.mtl"), "rb").read())
    for name, text in cases.items():
        p = tmp_path / name
        p.write_text(text)
        assert not art.mesh().parse(str(p)), name
        g = lib.rt_graph_new()
        try:
            assert lib.rt_mesh_build(g, str(p).encode(), None) < 0, name
        finally:
            lib.rt_graph_free(g)
