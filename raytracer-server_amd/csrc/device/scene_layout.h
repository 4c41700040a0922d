// Device-resident scene layout (shared by the host packer and the HIP kernels).
//
// Everything is flat, read-only, and lives in HBM for the lifetime of an rt_scene; per-render
// state (path slots, queues, accumulators) is allocated separately. f64 throughout, because the
// reference is f64 (geometry.rs:21-26) and the default render mode is bit-faithful to it.
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

#define RT_LAYOUT_FN __host__ __device__ inline

namespace rt {

enum : int32_t { GEOM_SPHERE = 0, GEOM_PLANE = 1, GEOM_MESH = 2 };
enum : int32_t { BRDF_DIFFUSE = 0, BRDF_SPECULAR = 1, BRDF_PHONG = 2 };

// One scene object (scene.rs:10-15). 16-byte aligned so the uniform object loop reads it with
// scalar (s_load) instructions.
struct alignas(16) DevObject {
    int32_t geom, brdf, mesh, ph_power;
    double emitted[3];
    double k[3];          // Diffuse kd / Specular ks
    double pos[3];        // sphere centre / plane point
    double r;             // sphere radius
    double n[3];          // plane normal
    double ph_kd, ph_ks;
    double color_d[3], color_s[3];
    int32_t emissive;     // emitted != 0 (any component)
    int32_t axis;         // plane with n == +-e_axis exactly (0,1,2), else -1
    int32_t pad0, pad1;
    double kpi[3];        // diffuse: kd * FRAC_1_PI (Diffuse::eval, scene.rs:41-43), host-evaluated
    double lef[3];        // diffuse: light's emitted * kpi (the NEE term's Le * f), host-evaluated
};

// Octree of one mesh, flattened in the reference's DFS pre-order (geometry.rs:1164-1216) so node
// i here is node i of the reference's Vec<Node> (plus node_base). Node boxes are NOT stored: a
// child's box is the octant of its parent's box (geometry.rs:1067-1099), recomputed in registers
// with the build's own arithmetic, so the traversal reads only the child table (32 B per node).
// All indices are GLOBAL (mesh bases already added).
struct alignas(16) DevMesh {
    int32_t node_base, n_nodes, root_leaf, max_depth;  // root_leaf: leaf id when the root is a leaf, else -1
    int32_t tri_base, n_tris, bvh_base, bvh_n;  // bvh: this mesh's nodes in DevScene::bvh
    double root_box[6];       // Octree.bounding_box (min xyz, max xyz): octant arithmetic of the walk
    double cull_box[6];       // root_box united with the vertex bounds: the early-out culls (near_box).
                              // The `scale` transform grows the stored box wrongly (geometry.rs:503-506),
                              // so root_box alone need not enclose the triangles a leaf root or the
                              // nearest-triangle loop tests without any box test (geometry.rs:886-903, 1276)
    double oct_center[8][3];  // centres of the ROOT box's octants: traversal order key (geometry.rs:1249-1260)
    double surface_area;      // Mesh.surface_area (mesh-light pdf, geometry.rs:591)
    double total_weight;      // sum of triangle areas (WeightedIndex total)
    double cull_pad;          // near_box padding: 1e-7 * max(1, |box coordinates|)
    int32_t btri_base;        // first of this mesh's n_tris BVH-order triangles (DevScene::btris)
    int32_t root_pid;         // the root's row in DevScene::node_slot / node_box (parent ordinal), -1 for a
                              // root leaf
    int32_t root_exist;       // the root's existence mask (KidSlot): the slot walk's first walk_enter
    int32_t pad2;
    double tight_base[3], tight_step;  // KidSlot bounds: base[k] + q * step (cull box min - E, 3 E / 65535)
    float cull32[6];          // cull_box rounded outward to f32 (near_mesh32's single-precision cull)
    float cull32_s;           // max(1, |cull box coordinates|): the scale of near_mesh32's padding
    int32_t pad4;
    // Flat octree (the cubes): the root is a leaf, or a parent whose children are all leaves, with at
    // most kFlatMaxTris triangles and every leaf list in triangle order. flat_leaf[j / 4] byte j % 4 =
    // the leaves (octant bits; bit 0 for a root leaf) that hold triangle j; flat_kids = octants with a
    // leaf. render_flat_f64.hip evaluates the reference's walk on these tables (flat_query).
    int32_t flat, flat_kids, flat_root_leaf, pad3;
    uint32_t flat_leaf[8];
};
constexpr int kFlatMaxTris = 32;
constexpr int kFlatMeshes = 2;  // meshes of a flat scene: the flat kernels' LDS queues and result columns
                                // (render_flat_f64.hip) and rt_api.cpp's RenderArgs::all_flat

// BVH over a mesh's triangles for the nearest-triangle mode (RT_FLAG_MESH_NEAREST), nodes in DFS
// pre-order: an inner node's left child is the next node, `a` its right child, `axis` the split
// axis (left = smaller centroids); a leaf (count > 0) holds btris[a .. a + count).
constexpr int kBvhMaxDepth = 20;  // the traversal's per-lane stack (LDS; 20 entries fit the mesh kernel's park)
struct alignas(16) DevBvhNode {
    double bmin[3], bmax[3];
    int32_t a, count, axis, pad;
};

// node_kids[node][8] entries: -1 empty octant, >= 0 parent node, <= -2 a leaf: e = -2 - entry holds
// the leaf's triangle range inline, first list entry (e >> 6) and count (e & 63), so opening a leaf
// needs no further load; a leaf of >= 63 triangles or a first entry >= 2^25 stores count 63 and its
// leaf id in e >> 6 instead (its range is then read from leaf_span).
constexpr int32_t kKidEmpty = -1;
constexpr int32_t kKidCountEscape = 63;
RT_LAYOUT_FN int32_t kid_leaf(int32_t leaf, int32_t first, int32_t count) {
    const bool inl = count < kKidCountEscape && first < (1 << 25);
    return -2 - ((inl ? first : leaf) << 6 | (inl ? count : kKidCountEscape));
}
// A walk's child pick reads one 16-byte slot: node_slot[pid][8] = the child entry (as node_kids,
// with the parent encoding below) and the child subtree's triangle
// bounds ("tight box": the vertices of every triangle in the subtree's leaves, padded by
// DevMesh::cull_pad), rounded OUTWARD to 16-bit codes over the mesh's range (DevMesh::tight_base /
// tight_step: bound = base + q * step, one extra step each way (rt_api.cpp make_slot: no code is clamped, or the
// scene has no slot tables; before round 5 a low code 0 meant -inf, a high code
// 65535 +inf). Triangles may reach far outside their octant (geometry.rs:1038-1060 assigns any
// triangle that touches it), so the bounds are not the octant box. A ray that passes farther than the
// padding from them cannot get tri_intersect == true from any triangle below, so the reference's walk
// would find nothing there: skipping the child changes no result (Octree).
// A parent child's entry in a slot also carries that child's own existence mask (bit k: its octant k
// holds a node), so entering it needs no load: entry = pid | mask << 23 (pids < 2^23); leaf and
// empty entries as in node_kids. The slot walk refers to parents only (leaves are inline in the
// entries), so node_slot and node_box are indexed by the parent ordinal `pid` (parents numbered in the
// octree's DFS order, over all meshes): 9,540 rows for the unicorn instead of one per node (47,183), and
// a pop's box load no longer shares its cache lines with the boxes of leaves.
struct alignas(16) KidSlot {
    int32_t kid;
    uint16_t lo[3], hi[3];
};
constexpr int kTightTop = 65535;
constexpr int32_t kSlotMaxNode = 1 << 23;
RT_LAYOUT_FN int32_t slot_parent(int32_t node, uint32_t exist) { return node | (int32_t)(exist << 23); }
RT_LAYOUT_FN int32_t slot_node(int32_t e) { return e & (kSlotMaxNode - 1); }
RT_LAYOUT_FN uint32_t slot_exist(int32_t e) { return (uint32_t)e >> 23; }
// node_up[node] = {parent node (-1 at the root), octant slot in the parent}
// leaf_span[leaf] = {first entry of the leaf in ltri_id (ltris in RT_LTRI_INDEX=0 builds), count}

// Triangle, precomputed exactly as Triangle::intersect derives it per call (geometry.rs:637-653):
// a, ab = b - a, ac = c - a, n = ((c - a) x (b - a)).norm(). 12 doubles = 96 B.
struct DevTri {
    double a[3], ab[3], ac[3], n[3];
};
// The octree leaves' triangle copies (DevScene::ltris): DevTri, or in RT_LTRI72 builds 72 B without the
// normal, which the walk's test recomputes with the host's operations (tri_normal, path_f64.h).
#ifndef RT_LTRI72
#define RT_LTRI72 0
#endif
struct DevTri72 {
    double a[3], ab[3], ac[3];
};
#if RT_LTRI72
typedef DevTri72 LeafTri;
#else
typedef DevTri LeafTri;
#endif

// Compact per-type object tables, passed in the kernel arguments so the trace loops are unrolled
// and their operands live in scalar registers (no per-object loads or type branches). Objects keep
// their scene index for the reference's tie rule (scene.rs:278: ties go to the lower index).
constexpr int kMaxAxisPlanes = 4;  // per axis
constexpr int kMaxSpheres = 4;
constexpr int kMaxGeneric = 8;     // meshes and non-axis planes
constexpr int kMaxCompactObjects = 16;  // compact scenes also hold their object table in LDS (3.3 KB)
// The compact tables live in device memory (part of the scene blob) and are read through a
// constant-address-space pointer: scalar loads at each use, so they never occupy SGPRs across the
// path loop (as kernel arguments they did, and the spilled SGPRs were reloaded with ~900 static
// v_readlane instructions in the cornell megakernel).
struct CompactTab {
    int32_t n_ax[3];                         // planes with n = +-e_k, per axis k
    int32_t n_sph, n_gen;
    int32_t last_mesh_g;                     // the last gen_idx slot holding a mesh (-1 none): a walk pool
                                             // query whose walk of that mesh ended has its result
    int32_t ax_idx[3][kMaxAxisPlanes];
    double ax_pos[3][kMaxAxisPlanes];        // plane point coordinate along its axis
    int32_t sph_idx[kMaxSpheres];
    double sph[kMaxSpheres][4];              // centre xyz, r*r
    int32_t gen_idx[kMaxGeneric];            // everything else, through the generic intersector
    // per gen slot, so the per-ray loops over the gen slots read only this table (scalar loads issued
    // together) instead of the object and then its mesh (a chain of dependent loads):
    uint32_t gen_analytic;                   // bit g: slot g is a sphere or plane (analytic_t can hit it)
    int32_t gen_mesh[kMaxGeneric];           // slot g's mesh when it is a mesh with a non-empty octree, else -1
    float gen_cull32[kMaxGeneric][8];        // that mesh's cull32[0..5] and cull32_s (near_mesh32's operands)
};
typedef const __attribute__((address_space(4))) CompactTab CTab;

// f32 perf mode (RT_FLAG_FP32, kernels/render_f32.hip): the same scene rounded to f32, statistical
// parity only. Objects 64 B; BVH nodes 32 B with boxes rounded outward (conservative); triangles 48 B.
struct alignas(16) Obj32 {
    int32_t geom, brdf, mesh, emissive;
    float emitted[3], r;
    float k[3], r2;       // kd / ks; sphere radius squared
    float pos[3];
    int32_t axis;         // plane with n = +-e_axis (0, 1, 2), else -1
    float n[3], pad1;
};
struct alignas(16) Bvh32 {
    float bmin[3];
    int32_t a;            // right child (inner) / first btri (leaf)
    float bmax[3];
    int32_t cnt_axis;     // count * 4 + axis (count 0: inner node)
};
struct Tri32 {
    float a[3], ab[3], ac[3], n[3];
};

// CompactTab in f32 (built from it): the trace loops' operands in one scalar-loadable block.
struct Compact32 {
    int32_t n_ax[3], n_sph, n_gen, ok;
    int32_t ax_idx[3][kMaxAxisPlanes];
    float ax_pos[3][kMaxAxisPlanes];
    int32_t sph_idx[kMaxSpheres];
    float sph[kMaxSpheres][4];  // centre xyz, r*r
    int32_t gen_idx[kMaxGeneric];
};

struct DevScene {
    const DevObject* objects;
    const DevMesh* meshes;
    const int32_t* node_kids;   // [node][8], see kid_leaf (leaf triangle ranges inline)
    const int2* node_up;        // [node] {parent, slot}
    const int2* leaf_span;      // [leaf] {first ltri, count}
    const LeafTri* ltris;       // RT_LTRI_INDEX=0 builds only: leaf triangle lists as copies, in leaf order
                                // (the reference's leaves hold (index, Triangle) copies, geometry.rs:1131-1137)
    const int32_t* ltri_id;     // [ltri] leaf triangle lists as global triangle indices into `tris`, in leaf
                                // order (the walk's triangles and the hit's `prim`)
    const DevTri* tris;         // per triangle (surface normal, mesh-light sampling)
    const double* tri_cum_area;  // per triangle, cumulative area within its mesh (mesh-light pick)
    const CompactTab* ctab;     // compact tables (valid when `compact`; see Cfg::compact)
    const DevBvhNode* bvh;      // nearest-triangle mode: BVH nodes (DevMesh::bvh_base)
    const DevTri* btris;        // BVH leaf triangles, in leaf order
    const int32_t* btri_id;     // [btri] global triangle index
    const Obj32* obj32;         // f32 perf mode tables (Obj32 / Bvh32 / Tri32 above)
    const Bvh32* bvh32;
    const Tri32* btris32;
    const Compact32* ctab32;    // f32 compact tables (ok == 0: the generic object loop)
    const KidSlot* node_slot;   // [pid][8] child entry + subtree triangle bounds (KidSlot above); null
                                // when a node id does not fit a slot entry (>= kSlotMaxNode): the walks
                                // then read node_kids (walk_step<false>)
    const double* node_box;     // [pid][6] the parent's octant box (min xyz, max xyz) with the walk's own
                                // arithmetic: a pop of the slot walk reloads the ancestor's box from here
    const int32_t* pid_up;      // [pid] the parent's parent as a pid (-1 at a root): the pops of slot walks
                                // without an LDS ancestor column (node_up is indexed by node id)
    int32_t n_pid;              // rows of node_slot / node_box / pid_up (parents of all octrees)
    int32_t pad7;
    float off32;                // f32 mode: hit points are offset by off32 * n (scene-scaled epsilon)
    int32_t n_objects, light, n_meshes, compact;
    double cam_pos[3], cam_dir[3];
    double light_pdf;           // area pdf of the light: 1 / (4 pi r^2) (geometry.rs:583) or
                                // 1 / surface_area (:591), evaluated once on the host
};

}  // namespace rt
