// scenefile.h — versioned flat-scene files: a compiled scene (FlatScene: primitive records, the SAH BVH4, objects,
// materials, textures, texels) written once and loaded without re-parsing OBJ/MTL, re-decoding textures,
// re-triangulating or rebuilding the BVH.  Replaces the reference's per-run scene construction (scene_manager::build,
// scene_manager.cpp:260-355; mesh::parse/build, mesh.h:31-145; the O(N^2) bvh_node build, bvh.cpp:3-42).
//
// Layout (little-endian; every array 64-B aligned, so a file mapped into memory is used in place):
//   FileHeader (magic "ARTSCN\0\1", version, sizeof of every record type, the view of scene_manager::build, flags,
//   one {offset, count} per array, FNV-1a 64 of everything after the header) then the arrays in FileHeader order.
#pragma once
#include <string>

#include "scene.h"

namespace art {

constexpr uint32_t kSceneFileVersion = 3;  // 2: feature bit F_MEDIA_G; 3: hoisted BVH primitives (ObjRec::b)

struct SceneView {  // what scene_manager::build returns besides the objects (scene_manager.h:6-14)
    double lookfrom[3] = {0, 0, 0}, lookat[3] = {0, 0, 0}, vfov = 40.0, aperture = 0.0;
};

void save_scene_file(const std::string& path, const FlatScene& flat, const SceneView& view);
// Throws std::runtime_error naming what is wrong (not a scene file, another version or record layout, truncated,
// checksum mismatch).
void load_scene_file(const std::string& path, FlatScene& flat, SceneView& view);

}  // namespace art
