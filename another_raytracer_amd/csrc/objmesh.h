// objmesh.h — Wavefront OBJ/MTL ingestion: the reference's `mesh` class (src/primitives/mesh.h:29-145).
//
// The reference parses with rapidobj v1.0.1 (vendored, 3rd_parties/rapidobj/rapidobj.hpp) and triangulates with
// rapidobj::Triangulate (rapidobj.hpp:7137-7302), whose >4-vertex faces go through the vendored mapbox earcut v2.2.4
// (rapidobj.hpp:352-1175).  The triangle list, its order and its f32 vertex values decide both the geometry and the
// order of the scene RNG draws (one color::random() per triangle when the OBJ has no material library), so this
// loader restates exactly the parts of that pipeline the reference's meshes exercise:
//   * `v` / `vt` / `f` / `g` / `o` / `usemtl` / `mtllib` records; f32 values parsed correctly rounded (fast_float);
//     1-based, negative (relative) and v/vt/vn, v//vn face indices;
//   * triangles pass through, quads split along the shorter diagonal, larger faces are projected on the plane of
//     their largest f32 shoelace area and ear-clipped by an earcut restatement (passes 0-3, no holes);
//   * MTL `newmtl`, `Ka`, `Kd`, `map_Kd` (the only fields mesh.h:98-135 reads).
// Pinned by tests/test_mesh.py against the reference's own post-triangulation triangle lists (assets/*.tris,
// exported by oracle/ref_harness `mesh`).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "scene.h"

namespace art {

struct ObjIndex {
    int32_t p = -1, t = -1, n = -1;  // 0-based position / texcoord / normal index (-1 = absent)
};

struct ObjMaterial {  // rapidobj::Material (rapidobj.hpp:260-290), the fields mesh.h reads
    std::string name;
    float ka[3] = {0, 0, 0};
    float kd[3] = {0, 0, 0};
    std::string map_kd;
};

struct ObjMesh {
    std::string dir;                      // model_work_path (mesh.h:60): textures resolve against it
    std::vector<float> positions;         // xyz per vertex
    std::vector<float> texcoords;         // uv per texture vertex
    std::vector<ObjIndex> tri;            // 3 per triangle, in rapidobj's post-Triangulate order
    std::vector<int32_t> tri_mat;         // material id per triangle (-1: none)
    std::vector<ObjMaterial> materials;   // in `newmtl` order
    size_t shapes = 0, faces = 0;         // non-empty shapes, faces before triangulation
};

// mesh::parse (mesh.h:31-65): rapidobj::ParseFile + rapidobj::Triangulate.  Throws std::runtime_error.
ObjMesh load_obj(const std::string& path);

// mesh::build (mesh.h:67-145): one triangle per entry of m.tri, with
//   * lambertian(barycentric_image_texture(uv1, uv2, uv3, image)) when its material has a map_Kd (one image per
//     distinct map name, material_map_handler mesh.h:9-27),
//   * lambertian(Ka + Kd) (f32 sums) for other materials,
//   * lambertian(color::random()) when the OBJ has no materials (draws from g.rng).
// Returns the triangle node ids (consecutive, in order).  A map_Kd image is decoded from its file next to the MTL
// (SceneGraph::image_file: imagedec.cpp, stb_image v2.27's bytes, as material_map_handler's image_texture loads it).
std::vector<int> build_mesh(SceneGraph& g, const ObjMesh& m);

// mapbox earcut (rapidobj.hpp:497-1166) over one ring of 2-D points (x0, y0, x1, y1, ...): vertex indices, 3 per
// triangle, before rapidobj's swap of each triangle's first two.  Empty on failure.
std::vector<uint32_t> earcut_ring(const std::vector<double>& xy);

}  // namespace art
