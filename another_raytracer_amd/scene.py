"""Scene surface of the reference, mirrored on the native scene graph (include/art.h rt_graph_*).

* `scene_manager().build(alias)` == scene_manager::build (src/scene_manager.cpp:260-355), plus the build-defined
  scenes "c1"  and "cow"/"dino" (SURVEY Q8).
* `mesh().parse(path)` / `.build()` == the reference's OBJ/MTL mesh class (src/primitives/mesh.h:29-145).
* The hittable / material / texture classes take the reference constructors' arguments.  Like the reference,
  which draws from ONE process-wide std::mt19937 (src/utils/tracer_utils.h:27-31), they all record into one
  process-wide native graph whose generator draws in construction order: `noise_texture` (perlin tables,
  perlin.h:10-19) and `bvh_node` (one random_int per node, bvh.cpp:9) consume it, and `random_double()` reads it,
  so a scene recipe written against these classes reproduces the reference's geometry bit for bit.
"""
import ctypes
import enum
import os

import numpy as np

from ._lib import check, dvec, lib, rt_scene_info

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")

_graph = None


def _g():
    global _graph
    if _graph is None:
        _graph = lib.rt_graph_new()
        if not _graph:
            raise MemoryError("rt_graph_new failed")
    return _graph


def reset_scene_rng():
    """Start a fresh graph (fresh mt19937, seed 5489), as a fresh reference process would."""
    global _graph
    if _graph is not None:
        lib.rt_graph_free(_graph)
    _graph = None


def random_double(lo=None, hi=None):
    """tracer_utils.h:27-36 random_double() / random_double(min, max) on the shared scene generator."""
    out = ctypes.c_double()
    check(lib.rt_graph_random_double(_g(), ctypes.byref(out)), "rt_graph_random_double")
    return out.value if lo is None else lo + (hi - lo) * out.value


def _color(c):
    return tuple(float(x) for x in c)


# ------------------------------------------------------------------------------------------------ textures
class texture:
    id = -1


class solid_color(texture):  # texture.h:16-29
    def __init__(self, r, g=None, b=None):
        c = _color(r) if g is None else (float(r), float(g), float(b))
        self.color = c
        self.id = check(lib.rt_tex_solid(_g(), *c), "solid_color")


def _as_texture(t):
    return t if isinstance(t, texture) else solid_color(t)


class checker_texture(texture):  # texture.h:31-50
    def __init__(self, even, odd):
        self.even, self.odd = _as_texture(even), _as_texture(odd)
        self.id = check(lib.rt_tex_checker(_g(), self.even.id, self.odd.id), "checker_texture")


class noise_texture(texture):  # texture.h:52-65
    def __init__(self, scale):
        self.scale = float(scale)
        self.id = check(lib.rt_tex_noise(_g(), self.scale), "noise_texture")


class image_texture(texture):  # texture.h:67-118
    """From an (H, W, C>=3) uint8 array, or from a raw asset file (int32 w, h, bpp header + bytes)."""

    def __init__(self, source):
        if isinstance(source, (str, os.PathLike)):
            with open(source, "rb") as f:
                w, h, c = np.frombuffer(f.read(12), np.int32)
                data = np.frombuffer(f.read(), np.uint8)[: w * h * c].reshape(h, w, c)
        else:
            data = np.asarray(source, np.uint8)
        data = np.ascontiguousarray(data)
        h, w, c = data.shape
        self.id = check(lib.rt_tex_image(_g(), w, h, c, data.ctypes.data_as(ctypes.c_void_p)), "image_texture")


class barycentric_image_texture(texture):  # texture.h:135-154
    def __init__(self, a, b, c, tex):
        if not isinstance(tex, image_texture):
            raise TypeError("barycentric_image_texture samples an image_texture")
        uv = (ctypes.c_double * 6)(*[float(x) for x in (*a, *b, *c)])
        self.id = check(lib.rt_tex_bary_image(_g(), uv, tex.id), "barycentric_image_texture")


# ------------------------------------------------------------------------------------------------ materials
class material:
    id = -1


class lambertian(material):  # material.h:20-43
    def __init__(self, albedo):
        self.albedo = _as_texture(albedo)
        self.id = check(lib.rt_mat_lambertian(_g(), self.albedo.id), "lambertian")


class metal(material):  # material.h:45-61
    def __init__(self, albedo, fuzz):
        self.id = check(lib.rt_mat_metal(_g(), *_color(albedo), float(fuzz)), "metal")


class dielectric(material):  # material.h:63-99
    def __init__(self, index_of_refraction):
        self.id = check(lib.rt_mat_dielectric(_g(), float(index_of_refraction)), "dielectric")


class diffuse_light(material):  # material.h:101-118
    def __init__(self, emit):
        self.emit = _as_texture(emit)
        self.id = check(lib.rt_mat_diffuse_light(_g(), self.emit.id), "diffuse_light")


# ------------------------------------------------------------------------------------------------ hittables
class hittable:
    id = -1


class sphere(hittable):  # sphere.h
    def __init__(self, center, radius, mat):
        self.id = check(lib.rt_obj_sphere(_g(), dvec(center), float(radius), mat.id), "sphere")


class moving_sphere(hittable):  # moving_sphere.h
    def __init__(self, center0, center1, time0, time1, radius, mat):
        self.id = check(lib.rt_obj_moving_sphere(_g(), dvec(center0), dvec(center1), float(time0), float(time1),
                                                 float(radius), mat.id), "moving_sphere")


class triangle(hittable):  # triangle.h
    def __init__(self, p1, p2, p3, mat):
        self.id = check(lib.rt_obj_triangle(_g(), dvec(p1), dvec(p2), dvec(p3), mat.id), "triangle")


class _rect(hittable):
    AXIS = 0

    def __init__(self, a0, a1, b0, b1, k, mat):
        self.id = check(lib.rt_obj_rect(_g(), self.AXIS, float(a0), float(a1), float(b0), float(b1), float(k), mat.id),
                        type(self).__name__)


class xy_rect(_rect):  # aarect.h
    AXIS = 0


class xz_rect(_rect):
    AXIS = 1


class yz_rect(_rect):
    AXIS = 2


class box(hittable):  # box.cpp
    def __init__(self, p0, p1, mat):
        self.id = check(lib.rt_obj_box(_g(), dvec(p0), dvec(p1), mat.id), "box")


def _ids(objs):
    return (ctypes.c_int * len(objs))(*[o.id for o in objs])


class hittable_list(hittable):  # hittable_list.h
    def __init__(self, obj=None, native=None):
        self.objects = []
        self._native = native  # an rt_scene built by scene_manager (builtin scenes)
        if obj is not None:
            self.add(obj)

    def add(self, obj):
        if self._native is not None:
            raise TypeError("a builtin scene's object list is compiled; build a new hittable_list instead")
        self.objects.append(obj)

    def empty(self):
        return self._native is None and not self.objects

    def size(self):
        return len(self.objects)

    def clear(self):
        self.objects.clear()

    @property
    def id(self):  # used as a child object: materialise the list node in the graph
        if self._native is not None:
            raise TypeError("a builtin scene cannot be nested in another scene")
        return check(lib.rt_obj_list(_g(), len(self.objects), _ids(self.objects)), "hittable_list")


class bvh_node(hittable):  # bvh.h / bvh.cpp (draws its random_int(0,2) per node now, in call order)
    def __init__(self, objects, time0=0.0, time1=1.0):
        items = objects.objects if isinstance(objects, hittable_list) else list(objects)
        self.id = check(lib.rt_obj_bvh(_g(), len(items), _ids(items)), "bvh_node")


class mesh:  # primitives/mesh.h:29-145
    """Wavefront OBJ (+ MTL) triangle mesh.  parse() validates and counts like mesh::parse; build() adds one triangle per
    post-triangulation face to the shared graph (drawing color::random() per triangle when the OBJ has no material
    library, exactly as mesh::build) and returns them as a hittable_list."""

    def __init__(self):
        self.path = None
        self.triangles = self.shapes = 0

    def parse(self, mesh_path):
        t, sh = ctypes.c_int64(), ctypes.c_int64()
        if lib.rt_mesh_parse(os.fspath(mesh_path).encode(), ctypes.byref(t), ctypes.byref(sh)) < 0:
            return False  # mesh.h:33-40 reports the error and returns false
        self.path, self.triangles, self.shapes = os.fspath(mesh_path), t.value, sh.value
        return True

    def build(self):
        if self.path is None:
            raise RuntimeError("mesh::build before a successful parse")
        first = ctypes.c_int()
        n = check(lib.rt_mesh_build(_g(), self.path.encode(), ctypes.byref(first)), "mesh.build")
        out = hittable_list()
        for i in range(n):
            h = hittable()
            h.id = first.value + i
            out.add(h)
        return out


class translate(hittable):  # hittable.cpp:3-23
    def __init__(self, p, displacement):
        self.id = check(lib.rt_obj_translate(_g(), p.id, dvec(displacement)), "translate")


class rotate_y(hittable):  # hittable.cpp:25-85
    def __init__(self, p, angle):
        self.id = check(lib.rt_obj_rotate_y(_g(), p.id, float(angle)), "rotate_y")


class constant_medium(hittable):  # constant_medium.h
    def __init__(self, boundary, density, albedo):
        tex = _as_texture(albedo)
        self.id = check(lib.rt_obj_constant_medium(_g(), boundary.id, float(density), tex.id), "constant_medium")


def compile_world(world, device):
    """hittable_list -> native rt_scene handle (c_void_p) on `device`.  A builtin scene's list is already compiled
    for the device its scene_manager named: using it on another device is an error (rendering it there would run on
    the scene's device and copy the frame across)."""
    if world._native is not None:
        if world._native.device != int(device):
            raise ValueError(f"this scene was built for device {world._native.device}, not {int(device)}: "
                             f"build it with scene_manager(device={int(device)})")
        return world._native
    g = _g()
    check(lib.rt_graph_clear_world(g), "rt_graph_clear_world")
    for o in world.objects:
        check(lib.rt_graph_add_world(g, o.id), "rt_graph_add_world")
    out = ctypes.c_void_p()
    check(lib.rt_graph_compile(g, int(device), ctypes.byref(out)), "rt_graph_compile")
    return _SceneHandle(out, device)


class _SceneHandle(ctypes.c_void_p):
    """Owns an rt_scene* (and remembers the device it was built for)."""

    def __init__(self, ptr, device=0):
        super().__init__(ptr.value if isinstance(ptr, ctypes.c_void_p) else ptr)
        self.device = int(device)

    def __del__(self):
        if self.value and lib is not None:
            lib.rt_scene_destroy(self)
            self.value = None


# ------------------------------------------------------------------------------------------------ scene_manager
class scene_alias(enum.IntEnum):  # scene_manager.h:16-27
    random = 1
    two_spheres = 2
    two_perlin_spheres = 3
    earth = 4
    simple_light = 5
    cornell_box = 6
    cornell_smoke = 7
    final = 8
    mesh = 9


class scene:  # scene_manager.h:6-14
    def __init__(self, lookfrom=(0, 0, 0), lookat=(0, 0, -1), vfov=40.0, aperture=0.0, background=(0, 0, 0),
                 objects=None):
        self.lookfrom, self.lookat, self.vfov, self.aperture = tuple(lookfrom), tuple(lookat), vfov, aperture
        self.background = tuple(background)
        self.objects = objects if objects is not None else hittable_list()


class scene_manager:
    def __init__(self, asset_dir=None, device=0):
        self.asset_dir = asset_dir or ASSET_DIR
        self.device = device

    def build(self, alias):
        name = str(int(alias)) if isinstance(alias, (scene_alias, int)) else str(alias)
        out = ctypes.c_void_p()
        check(lib.rt_scene_build(name.encode(), self.asset_dir.encode(), int(self.device), ctypes.byref(out)),
              f"scene_manager.build({alias})")
        return self._wrap(_SceneHandle(out, self.device))

    def load(self, path):
        """A scene saved by save_scene (rt_scene_load: the flat-scene file, no rebuild)."""
        out = ctypes.c_void_p()
        check(lib.rt_scene_load(os.fspath(path).encode(), int(self.device), ctypes.byref(out)), f"scene_manager.load({path})")
        return self._wrap(_SceneHandle(out, self.device))

    def _wrap(self, handle):
        info = rt_scene_info()
        check(lib.rt_scene_info_get(handle, ctypes.byref(info)), "rt_scene_info_get")
        s = scene(tuple(info.lookfrom), tuple(info.lookat), info.vfov, info.aperture, tuple(info.background),
                  hittable_list(native=handle))
        s.info = {f: (tuple(getattr(info, f)) if isinstance(getattr(info, f), ctypes.Array) else getattr(info, f))
                  for f, _ in info._fields_}
        return s


def save_scene(world, path):
    """Writes a builtin / loaded scene (scene_manager result) as a versioned flat-scene file (rt_scene_save)."""
    h = world.objects._native if isinstance(world, scene) else world._native
    if h is None:
        raise TypeError("save_scene takes a scene from scene_manager.build / load")
    check(lib.rt_scene_save(h, os.fspath(path).encode()), "save_scene")


def scene_dump(world):
    """Canonical JSON of a builtin scene (schema of oracle/ref_harness `dump`)."""
    h = world.objects._native if isinstance(world, scene) else world._native
    n = lib.rt_scene_dump(h, None, 0)
    buf = ctypes.create_string_buffer(n)
    lib.rt_scene_dump(h, buf, n)
    return buf.value.decode()
