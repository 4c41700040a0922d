// Host scene preparation: the reference's startup path, restated in C++.
//   SceneSpec::to_scene      scene.rs:357-441
//   Mesh::load / prism/cube  geometry.rs:753-866
//   Geometry transforms      geometry.rs:426-510
//   Octree::build            geometry.rs:1145-1216 (+ BoundingBox::overlaps_triangle :1038-1061)
// All f64 arithmetic is compiled with -ffp-contract=off so mesh vertices, boxes and the octree
// are bit-identical to the reference's (the octree shape decides which triangles a ray sees,
// geometry.rs:1245-1295).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/rt_ffi.h"

namespace rt::host {

struct D3 {
    double x, y, z;
};
struct Box {
    D3 min, max;
};

struct Octree {
    // DFS pre-order, node i == reference node i
    std::vector<int32_t> kind;      // 0 parent, 1 leaf
    std::vector<int32_t> child;     // 8 per node, -1 empty
    std::vector<int32_t> leaf_off;  // -1 for parents
    std::vector<int32_t> leaf_cnt;
    std::vector<int32_t> parent;    // -1 root
    std::vector<int32_t> slot;      // octant index in parent
    std::vector<Box> box;           // the box the node was built for
    std::vector<int32_t> refs;      // leaf triangle lists (mesh-local triangle indices)
    Box root;
    int64_t parents = 0, leaves = 0, max_leaf = 0, max_depth = 0;
    size_t size() const { return kind.size(); }
};

struct Mesh {
    std::vector<D3> vertices;
    std::vector<uint32_t> indices;
    Box bbox;
    double surface_area = 0.0;
    std::vector<double> areas;  // WeightedIndex weights (Mesh::new, pre-transform)
    Octree octree;
    size_t num_triangles() const { return indices.size() / 3; }
};

struct Object {
    D3 emitted{0, 0, 0};
    int32_t brdf = RT_BRDF_DIFFUSE;
    D3 k{0, 0, 0};
    double ph_kd = 0, ph_ks = 0;
    int32_t ph_power = 0;
    D3 color_d{0, 0, 0}, color_s{0, 0, 0};
    int32_t geom = RT_GEOM_SPHERE;
    D3 pos{0, 0, 0};
    double r = 0;
    D3 n{0, 0, 0};
    int32_t mesh = -1;
};

struct Scene {
    D3 cam_pos{0, 0, 0}, cam_dir{0, 0, 1};
    std::vector<Object> objects;
    std::vector<Mesh> meshes;
    int32_t light = -1;
};

// Each returns RT_OK or an RT_E_* code with a message in *err.
int load_scene_toml(const std::string& toml_path, const std::string& assets_dir, Scene* out, std::string* err);
int scene_from_desc(const rt_scene_desc* desc, Scene* out, std::string* err);
int load_obj(const std::string& path, Mesh* out, std::string* err);
Mesh make_prism(D3 p, double w, double h, double d);
Mesh make_mesh(std::vector<D3> vertices, std::vector<uint32_t> indices);
void build_octree(Mesh& m);
// scene.rs:126-141 — light = first object whose emission is not within 1e-5 of zero.
int pick_light(Scene* s, std::string* err);
// camera frame of sample_pixel (server.rs:328-331)
void camera_frame(const Scene& s, int width, int height, double cx[3], double cy[3]);

}  // namespace rt::host
