"""Scene-compile restructurings that keep every closest hit and every RNG draw, checked on the CPU through the flat-scene
file (csrc/scenefile.cpp), whose arrays are the compiled scene.

World merging (csrc/scene.cpp Compiler::world): a run of untransformed BVHs and primitives of the world list, with at
least one BVH (or >= 3 primitives, or the whole world), becomes one BVH; a constant_medium ends a run.

BVH primitive hoisting (csrc/scene.cpp Compiler::bvh_obj, device.h traverse): a primitive whose box is as large as its
whole BVH's leaves the tree and is recorded as the BVH object's hoisted leaf (layout.h ObjRec::b), which every
traversal tests first.  Checked on the CPU through the flat-scene file (csrc/scenefile.cpp), whose arrays are the
compiled scene: the random scene's r = 1000 ground sphere (scene_manager.cpp:18) is hoisted and in no BVH leaf, the
other scenes hoist nothing, and a file whose hoisted leaf points outside the primitive references is refused.  Image
parity of the hoisted traversal is the GPU suite's (tests/test_gpu_parity.py, tests/test_gpu_full_size.py: scene 1)."""
import struct

import numpy as np
import pytest

import another_raytracer_amd as art

# scenefile.cpp FileHeader: magic, version, header_bytes, record_bytes[13], features, has_media, max_bvh_depth,
# max_stack, (pad), background[3], lookfrom[3], lookat[3], vfov, aperture, offset[13], count[13], payload, checksum
A_SPHERES, A_PRIMREFS, A_NODES, A_OBJS, A_WORLD = 0, 4, 5, 6, 7
OFF_OFFSET = 176
OBJ_BVH = 1
NODE_EMPTY = -1


def _arrays(blob):
    assert struct.unpack_from("<I", blob, 12)[0] == OFF_OFFSET + 13 * 16 + 16  # header_bytes: the layout above
    off = struct.unpack_from("<13Q", blob, OFF_OFFSET)
    cnt = struct.unpack_from("<13Q", blob, OFF_OFFSET + 13 * 8)
    return off, cnt


def _objs(blob):
    off, cnt = _arrays(blob)
    dt = np.dtype([("kind", "<i4"), ("a", "<i4"), ("b", "<i4"), ("pad", "<i4"), ("p", "<f8", 4)])
    return np.frombuffer(blob, dt, int(cnt[A_OBJS]), int(off[A_OBJS])), off[A_OBJS]


def _leaf(code):
    x = (~int(code)) & 0xFFFFFFFF
    return x & 0xFFFFFF, (x >> 24) & 0x7F


def _saved(name, tmp_path):
    p = tmp_path / f"{name}.artscene"
    art.save_scene(art.scene_manager().build(name), p)
    return bytearray(p.read_bytes())


def test_random_scene_hoists_the_ground_sphere(tmp_path):
    blob = _saved("1", tmp_path)
    off, cnt = _arrays(blob)
    objs, _ = _objs(blob)
    bvhs = objs[objs["kind"] == OBJ_BVH]
    assert len(bvhs) == 1 and bvhs[0]["b"] != NODE_EMPTY
    first, count = _leaf(bvhs[0]["b"])
    assert count == 1
    refs = np.frombuffer(blob, "<u4", int(cnt[A_PRIMREFS]), int(off[A_PRIMREFS]))
    ref = int(refs[first])
    assert ref >> 30 == 0  # PRIM_SPHERE
    sph = np.frombuffer(blob, "<f8", int(cnt[A_SPHERES]) * 10, int(off[A_SPHERES])).reshape(-1, 10)
    c, r = sph[ref & ((1 << 30) - 1), :3], sph[ref & ((1 << 30) - 1), 3]
    assert r == 1000.0 and tuple(c) == (0.0, -1000.0, 0.0)
    # no BVH leaf covers the hoisted primitive reference, and every other reference is in exactly one leaf
    nodes = np.frombuffer(blob, "<i4", int(cnt[A_NODES]) * 32, int(off[A_NODES])).reshape(-1, 32)
    covered = np.zeros(len(refs), np.int32)
    for ch in nodes[:, 24:28].ravel():
        if ch < NODE_EMPTY:
            f, n = _leaf(ch)
            covered[f:f + n] += 1
    assert covered[first] == 0
    assert np.all(np.delete(covered, first) == 1)


@pytest.mark.parametrize("name", ["8", "cow", "dino"])
def test_other_scenes_hoist_nothing(name, tmp_path):
    objs, _ = _objs(_saved(name, tmp_path))
    assert np.all(objs[objs["kind"] == OBJ_BVH]["b"] == NODE_EMPTY)


def _fnv1a(data):
    h = 1469598103934665603
    for b in data:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_out_of_range_hoisted_leaf_is_refused(tmp_path):
    blob = _saved("1", tmp_path)
    objs, base = _objs(blob)
    i = int(np.nonzero(objs["kind"] == OBJ_BVH)[0][0])
    _, cnt = _arrays(blob)
    bad = ~((1 << 24) | int(cnt[A_PRIMREFS]))  # one reference past the end
    struct.pack_into("<i", blob, int(base) + 48 * i + 8, bad)
    header = struct.unpack_from("<I", blob, 12)[0]
    start = (header + 63) & ~63
    struct.pack_into("<Q", blob, header - 8, _fnv1a(bytes(blob[start:])))
    p = tmp_path / "bad.artscene"
    p.write_bytes(bytes(blob))
    with pytest.raises(art.RTError) as e:
        art.scene_manager().load(p)
    assert "BVH object out of range" in str(e.value)


OBJ_PRIM, OBJ_TRANSLATE, OBJ_MEDIUM = 0, 2, 4


@pytest.mark.parametrize("name,kinds", [
    # Next-Week final (scene_manager.cpp:169-235): [box BVH, light, moving sphere, 3 spheres] merge; the two media,
    # earth, perlin sphere and the translated BVH stay in order
    ("8", [OBJ_BVH, OBJ_MEDIUM, OBJ_MEDIUM, OBJ_PRIM, OBJ_PRIM, OBJ_TRANSLATE]),
    ("cow", [OBJ_BVH, OBJ_MEDIUM]),  # mesh BVH + light merge, the mist medium stays
    ("1", [OBJ_BVH]),
    ("c1", [OBJ_BVH]),  # three spheres, the whole world: merged
    ("4", [OBJ_PRIM]),  # a single object: unchanged
    ("7", [OBJ_BVH, OBJ_MEDIUM, OBJ_MEDIUM]),  # Cornell smoke: six rects merged, the two box media stay
])
def test_world_merging(name, kinds, tmp_path):
    blob = _saved(name, tmp_path)
    off, cnt = _arrays(blob)
    objs, _ = _objs(blob)
    world = np.frombuffer(blob, "<i4", int(cnt[A_WORLD]), int(off[A_WORLD]))
    assert [int(objs[w]["kind"]) for w in world] == kinds


def test_split_bvh_references_every_triangle(tmp_path):
    # dino (394 triangles + the merged light rect): spatial splits reference straddling triangles from both sides, so
    # there are more references than primitives, and every primitive keeps at least one
    blob = _saved("dino", tmp_path)
    off, cnt = _arrays(blob)
    refs = np.frombuffer(blob, "<u4", int(cnt[A_PRIMREFS]), int(off[A_PRIMREFS]))
    tris = refs[refs >> 30 == 1] & ((1 << 30) - 1)
    assert len(refs) > 395
    assert set(tris.tolist()) == set(range(394))


def _leaf_cover(blob):
    off, cnt = _arrays(blob)
    nodes = np.frombuffer(blob, "<i4", int(cnt[A_NODES]) * 32, int(off[A_NODES])).reshape(-1, 32)
    covered = np.zeros(int(cnt[A_PRIMREFS]), np.int32)
    sizes = []
    for ch in nodes[:, 24:28].ravel():
        if ch < NODE_EMPTY:
            f, n = _leaf(ch)
            covered[f:f + n] += 1
            sizes.append(n)
    return len(nodes), covered, sizes


@pytest.mark.parametrize("mode", [0, 1])
def test_bvh_collapse_covers_every_reference_once(mode, tmp_path):
    # bvh.cpp collapse: greedy (option bvh.collapse = 0, the default) and SAH-optimal dynamic programming (1, which also
    # merges binary leaves into one wide-tree leaf): every primitive reference sits in exactly one leaf of at most
    # kMaxLeafPrims (4), except the random scene's hoisted ground sphere (no leaf); the option applies to scenes
    # compiled after it is set
    import pathlib
    art.set_option("bvh.collapse", mode)
    try:
        res = []
        for name in ("1", "8", "cow", "dino"):
            p = pathlib.Path(tmp_path) / f"s{name}.artscene"
            art.save_scene(art.scene_manager().build(name), p)
            art.scene_manager().load(p)  # the loader recomputes max_stack / depth and checks every index
            n, covered, sizes = _leaf_cover(bytearray(p.read_bytes()))
            res.append((name, n, int(covered.min()), int(covered.max()), max(sizes)))
    finally:
        art.set_option("bvh.collapse", 0)
    for name, n, lo, hi, biggest in res:
        assert hi == 1 and biggest <= 4, (name, hi, biggest)
        assert lo == (0 if name == "1" else 1), name
    nodes = {name: n for name, n, *_ in res}
    if mode == 1:  # the optimal collapse fills the 4-wide nodes: fewer nodes than the greedy one's 259 / 566 / 1884 / 159
        assert nodes["1"] < 259 and nodes["8"] < 566 and nodes["cow"] < 1884 and nodes["dino"] < 159
