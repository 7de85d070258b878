// art_render.cpp — the reference's src/main.cpp (main.cpp:25-60) as a headless C++ host of libart.so:
// scene_manager::build -> camera (aspect W/H, focus distance 10, shutter [0, 1]) -> engine::run -> imageio::save_image.
//
//   art_render SCENE W H SPP OUT.png [--mode single|stripes|images|adaptive] [--seed N] [--max-depth D] [--device I]
//                                    [--assets DIR] [--gpus N] [--progressive K] [--save-scene FILE] [--option NAME=VALUE]
//   art_render --info SCENE [--assets DIR]     scene_manager::build only (no GPU needed): prints the scene summary
//
// SCENE is a scene_manager alias, or file:PATH for a flat-scene file written by --save-scene.  --gpus N renders on
// devices 0..N-1 through multi_engine (RCCL); --progressive K traces K samples per pass and prints one JSON line per
// pass (the headless live preview); --option sets a library option (rt_option_set, include/art.h) before the scene is
// built, e.g. --option bvh.sah_ci=1.0 (repeatable).  Prints one JSON line: {"scene", "W", "H", "spp", "ms", "segments",
// "msamples_per_s", "extend_variant"}.
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "art_engine.hpp"

namespace {

std::string default_assets(const char* argv0) {  // <repo>/assets next to <repo>/another_raytracer_amd/art_render
    std::string p(argv0);
    const size_t s = p.find_last_of('/');
    const std::string dir = s == std::string::npos ? std::string(".") : p.substr(0, s);
    return dir + "/../assets";
}

int usage() {
    std::cerr << "usage: art_render SCENE W H SPP OUT.png [--mode single|stripes|images|adaptive] [--seed N] [--max-depth D]"
                 " [--device I] [--assets DIR] [--gpus N] [--progressive K] [--save-scene FILE] [--option NAME=VALUE]\n"
                 "       art_render --info SCENE [--assets DIR]\n";
    return 2;
}

}  // namespace

int main(int argc, char** argv) try {
    std::vector<std::string> pos;
    std::string assets = default_assets(argv[0]), mode = "stripes";
    uint64_t seed = 0;
    int max_depth = 50, device = 0, gpus = 0, progressive = -1;
    std::string save_path;
    bool info = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) throw std::invalid_argument("missing value after " + a);
            return argv[++i];
        };
        if (a == "--info") info = true;
        else if (a == "--assets") assets = next();
        else if (a == "--mode") mode = next();
        else if (a == "--seed") seed = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--max-depth") max_depth = std::atoi(next().c_str());
        else if (a == "--device") device = std::atoi(next().c_str());
        else if (a == "--gpus") gpus = std::atoi(next().c_str());
        else if (a == "--progressive") progressive = std::atoi(next().c_str());
        else if (a == "--save-scene") save_path = next();
        else if (a == "--option") {
            const std::string kv = next();
            const size_t eq = kv.find('=');
            if (eq == std::string::npos) throw std::invalid_argument("--option wants NAME=VALUE, got " + kv);
            // the whole value must be a number: "" or "abc" would parse as 0, which is inside most ranges
            const char* v = kv.c_str() + eq + 1;
            char* stop = nullptr;
            const double x = std::strtod(v, &stop);
            if (stop == v || *stop != '\0') throw std::invalid_argument("--option " + kv.substr(0, eq) + ": not a number: '" + std::string(v) + "'");
            art::set_option(kv.substr(0, eq), x);
        } else pos.push_back(a);
    }
    art::scene_manager sm(assets, device);  // main.cpp:29-30
    if (info) {
        if (pos.size() != 1) return usage();
        const art::scene w = sm.build(pos[0]);
        std::cout << "{\"scene\":\"" << pos[0] << "\",\"objects\":" << w.info.objects << ",\"spheres\":" << w.info.spheres
                  << ",\"triangles\":" << w.info.triangles << ",\"bvh_nodes\":" << w.info.bvh_nodes << ",\"vfov\":" << w.vfov
                  << ",\"aperture\":" << w.aperture << ",\"lookfrom\":[" << w.lookfrom.x() << "," << w.lookfrom.y() << ","
                  << w.lookfrom.z() << "]}" << std::endl;
        return 0;
    }
    if (pos.size() != 5) return usage();
    const int W = std::atoi(pos[1].c_str()), H = std::atoi(pos[2].c_str()), spp = std::atoi(pos[3].c_str());
    const art::engine_mode m = mode == "single" ? art::engine_mode::single
                               : mode == "adaptive" ? art::engine_mode::adaptive
                               : mode == "images"   ? art::engine_mode::parallel_images
                                                    : art::engine_mode::parallel_stripes;
    const bool from_file = pos[0].rfind("file:", 0) == 0;
    const art::scene world = from_file ? sm.load(pos[0].substr(5)) : sm.build(pos[0]);
    if (!save_path.empty()) art::save_scene(world, save_path);
    const double dist_to_focus = 10.0;  // main.cpp:34
    art::camera cam(world.lookfrom, world.lookat, art::vec3{{0, 1, 0}}, world.vfov, double(W) / H, world.aperture, dist_to_focus, 0.0,
                    1.0);  // main.cpp:35 (aspect W/H: SURVEY Q6)
    std::vector<std::uint8_t> image(static_cast<size_t>(W) * H * 3);
    rt_stats st{};
    if (gpus > 0) {  // engine.h:335-376's parallel drivers over GPUs
        if (from_file) throw std::invalid_argument("--gpus builds the scene on every device: give a scene alias");
        std::vector<int> devs;
        for (int k = 0; k < gpus; ++k) devs.push_back(k);
        art::multi_engine eng(pos[0], assets, devs, W, H, cam, spp, max_depth, seed);
        eng.set_background(world.background);
        eng.run(image.data());
        st = eng.stats();
    } else {
        art::render_engine eng(W, H, cam, m, spp, max_depth, seed);
        eng.set_scene(world, world.background);  // main.cpp:44
        int ms;
        if (progressive >= 0) {
            ms = eng.run_progressive(image.data(), [&](int done, const std::uint8_t*) {
                std::cout << "{\"pass_samples_done\":" << done << "}" << std::endl;
                return true;
            }, progressive);
        } else {
            ms = eng.run(image.data());  // main.cpp:45
        }
        if (ms < 0) return 1;
        st = eng.stats();
    }
    if (!art::imageio::save_image(pos[4], W, H, 3, image.data())) throw std::runtime_error("cannot write " + pos[4]);
    std::cout << "{\"scene\":\"" << pos[0] << "\",\"W\":" << W << ",\"H\":" << H << ",\"spp\":" << spp << ",\"ms\":" << st.ms
              << ",\"segments\":" << st.segments << ",\"msamples_per_s\":" << (st.ms > 0 ? st.segments / st.ms / 1e3 : 0.0)
              << ",\"extend_variant\":" << st.extend_variant << "}" << std::endl;
    return 0;
} catch (const std::exception& e) {
    std::cerr << "art_render: " << e.what() << std::endl;
    return 1;
}
