"""another_raytracer_amd — MI355X-native drop-in for the ray_color / BVH / scatter hot path of
blackccpie/another_raytracer.

The Python surface mirrors the reference's own classes so a user of `src/main.cpp` finds the same calls:

    from another_raytracer_amd import scene_manager, scene_alias, camera, engine, engine_mode, imageio
    world = scene_manager().build(scene_alias.random)          # scene_manager.cpp:260-355
    cam = camera(world.lookfrom, world.lookat, (0, 1, 0), world.vfov, W / H, world.aperture, 10.0, 0.0, 1.0)
    eng = engine(cam, engine_mode.parallel_stripes, width=W, height=H, samples_per_pixel=100)  # engine.h:22
    eng.set_scene(world.objects, world.background)               # engine.h:24-28
    ms = eng.run(image)                                          # engine.h:30-54, image: uint8 (H, W, 3)
    imageio.save_image("output.png", W, H, 3, image)             # imageio.cpp:17-20

Scenes can also be assembled object by object with the reference's constructors (sphere, moving_sphere, triangle,
xy_rect, xz_rect, yz_rect, box, hittable_list, bvh_node, translate, rotate_y, constant_medium; lambertian, metal,
dielectric, diffuse_light; solid_color, checker_texture, noise_texture, image_texture, barycentric_image_texture) and
OBJ/MTL meshes (mesh().parse(path) / .build(), mesh.h) — see scene.py.
All compute runs in libart.so (HIP, gfx950) behind include/art.h.
"""
from ._lib import RTError, get_option, lib, set_option  # noqa: F401  (fails loudly when libart.so is missing)
from .engine import camera, engine, engine_mode, tracer_constants  # noqa: F401
from .scene import (  # noqa: F401
    barycentric_image_texture, box, bvh_node, checker_texture, constant_medium, dielectric, diffuse_light, hittable_list, image_texture,
    lambertian, mesh, metal, moving_sphere, noise_texture, random_double, rotate_y, scene, scene_alias, scene_manager,
    solid_color, sphere, translate, triangle, xy_rect, xz_rect, yz_rect, reset_scene_rng, save_scene,
)
from . import imageio  # noqa: F401

__all__ = [
    "RTError", "set_option", "get_option", "camera", "engine", "engine_mode", "tracer_constants", "scene", "scene_alias", "scene_manager",
    "hittable_list", "bvh_node", "sphere", "moving_sphere", "triangle", "xy_rect", "xz_rect", "yz_rect", "box",
    "translate", "rotate_y", "constant_medium", "lambertian", "metal", "dielectric", "diffuse_light", "solid_color",
    "checker_texture", "noise_texture", "image_texture", "barycentric_image_texture", "mesh", "random_double", "reset_scene_rng", "imageio", "save_scene",
]
