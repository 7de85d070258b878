"""The C++ host surface (include/art_engine.hpp + another_raytracer_amd/host/art_render.cpp): the reference's
src/main.cpp path -- scene_manager::build -> camera -> engine<W,H,C>::run -> imageio::save_image -- as C++ over the C
ABI.  CPU tests cover the scene side and the header's compile surface; the GPU test checks the C++ host renders the
same image as the Python mirror."""
import json
import os
import subprocess

import numpy as np
import pytest

import another_raytracer_amd as art
from another_raytracer_amd import imageio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "another_raytracer_amd", "art_render")


def run(*args, check=True):
    out = subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=300)
    if check:
        assert out.returncode == 0, out.stderr
    return out


@pytest.mark.parametrize("scene", ["1", "c1", "8", "cow", "9"])
def test_info_matches_the_python_scene_manager(scene):
    info = json.loads(run("--info", scene).stdout)
    py = art.scene_manager().build(scene).info
    assert (info["objects"], info["spheres"], info["triangles"], info["bvh_nodes"]) == (
        py["objects"], py["spheres"], py["triangles"], py["bvh_nodes"])
    assert info["vfov"] == py["vfov"] and info["lookfrom"] == list(py["lookfrom"])


def test_unknown_scene_is_the_references_error():
    out = run("--info", "42", check=False)
    assert out.returncode == 1 and "unkwnown scene requested" in out.stderr


def test_option_flag_reaches_the_library():
    # --option NAME=VALUE is rt_option_set before the build: the final scene without world merging keeps its 11 world
    # objects (6 merged); an unknown option is refused
    assert json.loads(run("--info", "8").stdout)["objects"] == 6
    assert json.loads(run("--info", "8", "--option", "compile.world_merge=0").stdout)["objects"] == 11
    out = run("--info", "8", "--option", "no.such.option=1", check=False)
    assert out.returncode == 1 and "unknown option" in out.stderr


def test_reference_style_main_compiles(tmp_path):
    """main.cpp:25-60 written against the header with the compile-time engine<W,H,C>."""
    src = tmp_path / "main.cpp"
    src.write_text("""
#include "art_engine.hpp"
int main() {
    constexpr int W = 400, H = 225;
    art::scene_manager sm("assets");
    art::scene world = sm.build("random");
    art::camera cam(world.lookfrom, world.lookat, art::vec3{{0, 1, 0}}, world.vfov, double(W) / H, world.aperture, 10.0, 0.0, 1.0);
    art::engine<W, H, 3> eng(cam, art::engine_mode::parallel_stripes);
    eng.set_scene(world, world.background);
    std::vector<std::uint8_t> image(W * H * 3);
    if (eng.run(image.data()) < 0) return 1;
    return art::imageio::save_image("output.png", W, H, 3, image.data()) ? 0 : 1;
}
""")
    out = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                          "-I" + os.path.join(ROOT, "include"), str(src)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stripes", "adaptive"])
def test_cpp_host_renders_the_python_image(tmp_path, mode):
    W, H, spp = 96, 48, 8
    png = tmp_path / "out.png"
    info = json.loads(run("1", W, H, spp, png, "--mode", mode).stdout)
    got = imageio.load_image(str(png))
    world = art.scene_manager().build("1")
    cam = art.camera(world.lookfrom, world.lookat, (0, 1, 0), world.vfov, W / H, world.aperture, 10.0, 0.0, 1.0)
    m = art.engine_mode.adaptive if mode == "adaptive" else art.engine_mode.parallel_stripes
    eng = art.engine(cam, m, width=W, height=H, samples_per_pixel=spp)
    eng.set_scene(world.objects, world.background)
    img = np.zeros((H, W, 3), np.uint8)
    eng.run(img)
    assert np.array_equal(got, img)
    assert info["segments"] == eng.stats["segments"]


def test_header_surface_beyond_main_compiles(tmp_path):
    """The rest of the C++ surface: multi_engine (rt_render_multi), run_progressive, save_scene / scene_manager::load,
    imageio::load_image."""
    src = tmp_path / "more.cpp"
    src.write_text("""
#include "art_engine.hpp"
int main() {
    art::scene_manager sm("assets");
    art::scene world = sm.build("cow");
    art::save_scene(world, "cow.artscn");
    art::scene again = sm.load("cow.artscn");
    art::camera cam(again.lookfrom, again.lookat, art::vec3{{0, 1, 0}}, again.vfov, 16.0 / 9, again.aperture, 10.0, 0.0, 1.0);
    art::render_engine eng(320, 180, cam, art::engine_mode::parallel_stripes, 16);
    eng.set_scene(again, again.background);
    std::vector<std::uint8_t> image(320 * 180 * 3);
    int passes = 0;
    eng.run_progressive(image.data(), [&](int, const std::uint8_t*) { return ++passes < 3; }, 4);
    art::multi_engine multi("cow", "assets", {0, 1}, 320, 180, cam, 16);
    multi.set_background(world.background);
    multi.run(image.data());
    int w = 0, h = 0, c = 0;
    std::vector<std::uint8_t> tex = art::imageio::load_image("assets/earthmap.jpg", w, h, c);
    return tex.size() == static_cast<size_t>(w) * h * c ? 0 : 1;
}
""")
    out = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror",
                          "-I" + os.path.join(ROOT, "include"), str(src)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


@pytest.mark.gpu
def test_cpp_host_multi_progressive_and_scene_file(tmp_path):
    """--gpus 1 (multi_engine: RCCL gather path), --progressive (last snapshot) and a saved-then-loaded scene file all
    give the plain run's image bit for bit."""
    W, H, spp = 96, 54, 8
    base = tmp_path / "base.png"
    scn = tmp_path / "cow.artscn"
    info = json.loads(run("cow", W, H, spp, base, "--save-scene", scn).stdout)
    ref = imageio.load_image(str(base))
    multi = tmp_path / "multi.png"
    run("cow", W, H, spp, multi, "--gpus", 1)
    assert np.array_equal(imageio.load_image(str(multi)), ref)
    prog = tmp_path / "prog.png"
    out = run("cow", W, H, spp, prog, "--progressive", 3).stdout.strip().splitlines()
    assert [json.loads(x)["pass_samples_done"] for x in out[:-1]] == [3, 6, 8]
    assert np.array_equal(imageio.load_image(str(prog)), ref)
    loaded = tmp_path / "loaded.png"
    info2 = json.loads(run(f"file:{scn}", W, H, spp, loaded).stdout)
    assert np.array_equal(imageio.load_image(str(loaded)), ref)
    assert info2["segments"] == info["segments"]
