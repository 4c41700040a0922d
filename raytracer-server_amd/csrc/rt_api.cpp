// C ABI (include/rt_ffi.h): scene packing + per-device upload, render dispatch, error reporting.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_ffi.h"
#include "ab_knobs.h"
#include "device/scene_layout.h"
#include "host/scene_host.hpp"
#include "kernels/kernels.h"
#include "kernels/wavefront.h"

#ifndef RT_LTRI_INDEX
#define RT_LTRI_INDEX 0  // as path_f64.h (1: leaf triangle lists as indices, no per-leaf copies uploaded)
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(e_ == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP,                        \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                    \
    } while (0)

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Host image of the device scene, packed once per scene.
struct Packed {
    std::vector<rt::DevObject> objects;
    std::vector<rt::DevMesh> meshes;
    std::vector<int32_t> kids;   // [node][8]
    std::vector<int2> up;        // [node]
    std::vector<int2> leaves;    // [leaf] {first ltri, count}
    std::vector<rt::LeafTri> ltris;
    std::vector<int32_t> ltri_id;
    std::vector<rt::DevTri> tris;
    std::vector<double> cum_area;
    std::vector<rt::DevBvhNode> bvh;  // nearest-triangle mode (RT_FLAG_MESH_NEAREST)
    std::vector<rt::DevTri> btris;
    std::vector<int32_t> btri_id;
    std::vector<rt::KidSlot> slots;      // [pid][8] child entry + subtree triangle bounds (scene_layout.h KidSlot);
                                         // empty when a node id does not fit a slot entry (the node_kids walk)
    std::vector<double> node_box;        // [pid][6] parents' octant boxes, the walk's arithmetic (DevScene::node_box)
    std::vector<int32_t> pid_up;         // [pid] the parent's parent as a pid, -1 at the root (DevScene::pid_up)
};

// A child slot (scene_layout.h KidSlot): the child entry and its subtree's triangle bounds b (lo xyz,
// hi xyz, already padded), rounded OUTWARD to 16-bit codes over the mesh's range (base + q * step), one
// extra step each way so that device-side rounding of the dequantised bounds cannot move them inward.
// The device decodes every code as base + q * step (path_f64.h kid_tight_hit), so a bound is conservative
// only if its code was not clamped to the range: for a mesh of extent E > 0 the codes of its padded
// triangle bounds lie in about [E / step, 2 E / step] = [21845, 43690], but a mesh whose cull padding
// exceeds E (a sub-1e-7 mesh far from the origin) would clamp. *exact turns false then, and the scene
// walks without slot tables (node_kids: the same result without the subtree culls).
rt::KidSlot make_slot(int32_t kid, const rt::DevMesh& dm, const double* b, bool* exact) {
    rt::KidSlot s{};
    s.kid = kid;
    for (int k = 0; k < 3; ++k) {
        s.lo[k] = 0;
        s.hi[k] = (uint16_t)rt::kTightTop;
        if (kid == rt::kKidEmpty) continue;  // never picked: its slot is not read
        if (!(dm.tight_step > 0.0) || !std::isfinite(dm.tight_step)) {
            *exact = false;
            continue;
        }
        const double ql = std::floor((b[k] - dm.tight_base[k]) / dm.tight_step) - 1.0;
        const double qh = std::ceil((b[3 + k] - dm.tight_base[k]) / dm.tight_step) + 1.0;
        if (!(ql >= 1.0 && qh <= (double)(rt::kTightTop - 1))) *exact = false;
        s.lo[k] = ql >= 1.0 ? (uint16_t)std::min(ql, (double)(rt::kTightTop - 1)) : (uint16_t)0;
        s.hi[k] = qh <= (double)(rt::kTightTop - 1) ? (uint16_t)std::max(qh, 1.0) : (uint16_t)rt::kTightTop;
    }
    return s;
}

struct DeviceCopy {
    bool ready = false;
    void* blob = nullptr;
    rt::DevScene ds{};
};

}  // namespace

struct rt_scene {
    rt::host::Scene host;
    Packed packed;
    std::mutex mu;
    std::vector<DeviceCopy> dev;
    std::vector<std::unique_ptr<rt::Workspace>> pool;  // free wavefront workspaces, per device tagged
    ~rt_scene() {
        for (auto& d : dev)
            if (d.blob) (void)hipFree(d.blob);
        pool.clear();
    }
};

namespace {

void cp3(double* dst, const rt::host::D3& v) {
    dst[0] = v.x;
    dst[1] = v.y;
    dst[2] = v.z;
}

// BVH over one mesh's triangles for the nearest-triangle mode: median split of the triangle
// centroids along the longest axis, leaves of <= 4 triangles (or at depth kBvhMaxDepth - 1), nodes
// in DFS pre-order (DevBvhNode). Node boxes are the triangles' vertex bounds; the traversal's slab test pads
// them (near_box, DevMesh::cull_pad), so a triangle the ray hits is never culled.
// RT_BVH_SAH=0 selects the median-split build (A/B); default: binned SAH.
constexpr int kBins = 16;      // SAH bins per axis
constexpr int kSahDepth = 16;  // deeper BVH nodes split at the median (depth stays <= kBvhMaxDepth)
bool bvh_sah_enabled() { return rt::ab_knob("RT_BVH_SAH", 1) != 0; }

void build_bvh(Packed& p, const rt::host::Mesh& m, int32_t tri_base) {
    using rt::host::D3;
    struct Item { double lo[3], hi[3], c[3]; int32_t id; };
    const size_t n = m.num_triangles();
    std::vector<Item> it(n);
    for (size_t t = 0; t < n; ++t) {
        const D3 v[3] = {m.vertices[m.indices[3 * t]], m.vertices[m.indices[3 * t + 1]], m.vertices[m.indices[3 * t + 2]]};
        Item& x = it[t];
        x.id = (int32_t)t;
        for (int k = 0; k < 3; ++k) {
            const double a = k == 0 ? v[0].x : k == 1 ? v[0].y : v[0].z;
            const double b = k == 0 ? v[1].x : k == 1 ? v[1].y : v[1].z;
            const double c = k == 0 ? v[2].x : k == 1 ? v[2].y : v[2].z;
            x.lo[k] = std::min({a, b, c});
            x.hi[k] = std::max({a, b, c});
            x.c[k] = 0.5 * (x.lo[k] + x.hi[k]);
        }
    }
    struct Rec {
        Packed& p;
        std::vector<Item>& it;
        int32_t tri_base;
        bool sah;
        // Binned surface-area heuristic (16 bins per axis over the centroid bounds): the split
        // minimising area(L) * n(L) + area(R) * n(R); items are partitioned in place (left = lower
        // centroids along *ax). *mid = b when no split separates the items.
        static double half_area(const double* lo, const double* hi) {
            const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
            return dx * dy + dy * dz + dz * dx;
        }
        void sah_split(size_t b, size_t e, const double* clo, const double* chi, int* ax_out, size_t* mid) {
            double best = INFINITY;
            int best_ax = -1, best_bin = -1;
            for (int ax = 0; ax < 3; ++ax) {
                const double ext = chi[ax] - clo[ax];
                if (!(ext > 0.0)) continue;
                double lo[kBins][3], hi[kBins][3];
                size_t cnt[kBins] = {0};
                for (int q = 0; q < kBins; ++q)
                    for (int k = 0; k < 3; ++k) { lo[q][k] = INFINITY; hi[q][k] = -INFINITY; }
                for (size_t i = b; i < e; ++i) {
                    int q = (int)((it[i].c[ax] - clo[ax]) / ext * kBins);
                    q = std::min(kBins - 1, std::max(0, q));
                    ++cnt[q];
                    for (int k = 0; k < 3; ++k) {
                        lo[q][k] = std::min(lo[q][k], it[i].lo[k]);
                        hi[q][k] = std::max(hi[q][k], it[i].hi[k]);
                    }
                }
                double ra[kBins];
                size_t rc[kBins];
                double al[3] = {INFINITY, INFINITY, INFINITY}, ah[3] = {-INFINITY, -INFINITY, -INFINITY};
                size_t ac = 0;
                for (int q = kBins - 1; q > 0; --q) {  // suffix boxes: bins q..15
                    for (int k = 0; k < 3; ++k) { al[k] = std::min(al[k], lo[q][k]); ah[k] = std::max(ah[k], hi[q][k]); }
                    ac += cnt[q];
                    rc[q] = ac;
                    ra[q] = ac ? half_area(al, ah) : 0.0;
                }
                double pl[3] = {INFINITY, INFINITY, INFINITY}, ph[3] = {-INFINITY, -INFINITY, -INFINITY};
                size_t pc = 0;
                for (int q = 1; q < kBins; ++q) {  // split between bins q-1 and q
                    for (int k = 0; k < 3; ++k) { pl[k] = std::min(pl[k], lo[q - 1][k]); ph[k] = std::max(ph[k], hi[q - 1][k]); }
                    pc += cnt[q - 1];
                    if (pc == 0 || rc[q] == 0) continue;
                    const double cost = half_area(pl, ph) * (double)pc + ra[q] * (double)rc[q];
                    if (cost < best) { best = cost; best_ax = ax; best_bin = q; }
                }
            }
            *mid = b;
            if (best_ax < 0) return;
            const int ax = best_ax;
            const double ext = chi[ax] - clo[ax];
            auto left = [&](const Item& x) {
                int q = (int)((x.c[ax] - clo[ax]) / ext * kBins);
                return std::min(kBins - 1, std::max(0, q)) < best_bin;
            };
            *mid = (size_t)(std::stable_partition(it.begin() + b, it.begin() + e, left) - it.begin());
            *ax_out = ax;
        }
        void build(size_t b, size_t e, int depth) {
            const size_t node = p.bvh.size();
            p.bvh.push_back(rt::DevBvhNode{});
            rt::DevBvhNode nd{};
            double clo[3], chi[3];
            for (int k = 0; k < 3; ++k) {
                nd.bmin[k] = clo[k] = INFINITY;
                nd.bmax[k] = chi[k] = -INFINITY;
            }
            for (size_t i = b; i < e; ++i)
                for (int k = 0; k < 3; ++k) {
                    nd.bmin[k] = std::min(nd.bmin[k], it[i].lo[k]);
                    nd.bmax[k] = std::max(nd.bmax[k], it[i].hi[k]);
                    clo[k] = std::min(clo[k], it[i].c[k]);
                    chi[k] = std::max(chi[k], it[i].c[k]);
                }
            if (e - b <= 4 || depth + 1 >= rt::kBvhMaxDepth) {
                nd.a = (int32_t)p.btris.size();
                nd.count = (int32_t)(e - b);
                std::sort(it.begin() + b, it.begin() + e, [](const Item& x, const Item& y) { return x.id < y.id; });
                for (size_t i = b; i < e; ++i) {
                    p.btris.push_back(p.tris[tri_base + it[i].id]);
                    p.btri_id.push_back(tri_base + it[i].id);
                }
            } else {
                int ax = 0;
                size_t mid = 0;
                if (sah && depth < kSahDepth) sah_split(b, e, clo, chi, &ax, &mid);
                if (mid <= b || mid >= e) {  // median split (no SAH split found, or deep nodes)
                    ax = 0;
                    for (int k = 1; k < 3; ++k)
                        if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
                    mid = (b + e) / 2;
                    std::nth_element(it.begin() + b, it.begin() + mid, it.begin() + e,
                                     [ax](const Item& x, const Item& y) { return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.id < y.id); });
                }
                nd.axis = ax;
                build(b, mid, depth + 1);
                nd.a = (int32_t)p.bvh.size();  // global index of the right child
                build(mid, e, depth + 1);
            }
            p.bvh[node] = nd;
        }
    } rec{p, it, tri_base, bvh_sah_enabled()};
    if (n > 0) rec.build(0, n, 0);
}

// RT_OK, or RT_E_INVAL when the octree tables cannot encode the mesh (kid_leaf: leaf ids < 2^25). Parent
// ordinals beyond a KidSlot entry's range (>= kSlotMaxNode, counted over the scene's meshes) leave the scene
// without slot tables: its walks then read node_kids (walk_step<false>, the same result without the
// subtree culls).
int pack_scene(rt_scene* s) {
    using namespace rt::host;
    Packed& p = s->packed;
    const Scene& sc = s->host;
    bool slots_ok = true;
    // RT_TEST_SLOT_MAX_PID (tests only): a lower limit on the parent ordinals (pid, the slot rows a KidSlot
    // entry can name), down to 0 = no slot tables (the node_kids walk for every scene), standing in for a
    // mesh whose pids exceed the encoding (kSlotMaxNode); named as a test switch so no stray setting of a
    // production-sounding variable slows every scene down
    int32_t slot_max = rt::kSlotMaxNode;
    if (const char* v = std::getenv("RT_TEST_SLOT_MAX_PID")) slot_max = std::max(0, std::min(slot_max, std::atoi(v)));
    if (slot_max == 0) slots_ok = false;
    for (const Mesh& m : sc.meshes) {
        rt::DevMesh dm{};
        dm.node_base = (int32_t)p.up.size();
        dm.n_nodes = (int32_t)m.octree.size();
        dm.root_leaf = -1;
        dm.max_depth = (int32_t)m.octree.max_depth;
        dm.tri_base = (int32_t)p.tris.size();
        dm.n_tris = (int32_t)m.num_triangles();
        const Box& rb = m.octree.root;
        double rbox[6] = {rb.min.x, rb.min.y, rb.min.z, rb.max.x, rb.max.y, rb.max.z};
        std::memcpy(dm.root_box, rbox, sizeof rbox);
        // root octant centres, with the same arithmetic as BoundingBox::octant(i).center()
        D3 c{(rb.min.x + rb.max.x) / 2.0, (rb.min.y + rb.max.y) / 2.0, (rb.min.z + rb.max.z) / 2.0};
        for (int i = 0; i < 8; ++i) {
            D3 lo{(i & 4) ? c.x : rb.min.x, (i & 2) ? c.y : rb.min.y, (i & 1) ? c.z : rb.min.z};
            D3 hi{(i & 4) ? rb.max.x : c.x, (i & 2) ? rb.max.y : c.y, (i & 1) ? rb.max.z : c.z};
            dm.oct_center[i][0] = (lo.x + hi.x) / 2.0;
            dm.oct_center[i][1] = (lo.y + hi.y) / 2.0;
            dm.oct_center[i][2] = (lo.z + hi.z) / 2.0;
        }
        dm.surface_area = m.surface_area;
        std::memcpy(dm.cull_box, rbox, sizeof rbox);
        for (const D3& v : m.vertices) {
            const double xyz[3] = {v.x, v.y, v.z};
            for (int k = 0; k < 3; ++k) {
                dm.cull_box[k] = std::fmin(dm.cull_box[k], xyz[k]);
                dm.cull_box[3 + k] = std::fmax(dm.cull_box[3 + k], xyz[k]);
            }
        }
        {
            double mx = 1.0;
            for (double v : dm.cull_box) mx = std::fmax(mx, std::fabs(v));
            dm.cull_pad = 1e-7 * mx;
            // f32 copy rounded outward (path_f64.h near_mesh32)
            for (int k = 0; k < 3; ++k) {
                float lo = (float)dm.cull_box[k], hi = (float)dm.cull_box[3 + k];
                if ((double)lo > dm.cull_box[k]) lo = std::nextafter(lo, -INFINITY);
                if ((double)hi < dm.cull_box[3 + k]) hi = std::nextafter(hi, INFINITY);
                dm.cull32[k] = lo;
                dm.cull32[3 + k] = hi;
            }
            dm.cull32_s = (float)mx * (1.0f + 0x1p-20f);
        }
        double cum = 0.0;
        for (size_t t = 0; t < m.num_triangles(); ++t) {
            D3 a = m.vertices[m.indices[3 * t]], b = m.vertices[m.indices[3 * t + 1]], cc = m.vertices[m.indices[3 * t + 2]];
            rt::DevTri dt{};
            D3 ab{b.x - a.x, b.y - a.y, b.z - a.z}, ac{cc.x - a.x, cc.y - a.y, cc.z - a.z};
            // Triangle::normal: (c - a).cross(b - a).norm()
            D3 cr{ac.y * ab.z - ac.z * ab.y, ac.z * ab.x - ac.x * ab.z, ac.x * ab.y - ac.y * ab.x};
            double mg = std::sqrt(cr.x * cr.x + cr.y * cr.y + cr.z * cr.z);
            D3 n{cr.x / mg, cr.y / mg, cr.z / mg};
            cp3(dt.a, a);
            cp3(dt.ab, ab);
            cp3(dt.ac, ac);
            cp3(dt.n, n);
            p.tris.push_back(dt);
            cum += t < m.areas.size() ? m.areas[t] : 0.0;
            p.cum_area.push_back(cum);
        }
        dm.total_weight = cum;
        const Octree& oc = m.octree;
        // leaf ids in node order; leaf triangles copied in the leaf's own order
        std::vector<int32_t> leaf_of(oc.size(), -1);
        for (size_t i = 0; i < oc.size(); ++i) {
            if (!oc.kind[i]) continue;
            leaf_of[i] = (int32_t)p.leaves.size();
            p.leaves.push_back(int2{(int32_t)p.ltri_id.size(), oc.leaf_cnt[i]});
            for (int32_t r = 0; r < oc.leaf_cnt[i]; ++r) {
                const int32_t t = oc.refs[oc.leaf_off[i] + r];
#if !RT_LTRI_INDEX
                const rt::DevTri& lt = p.tris[dm.tri_base + t];
#if RT_LTRI72
                rt::LeafTri l72{};
                for (int k = 0; k < 3; ++k) { l72.a[k] = lt.a[k]; l72.ab[k] = lt.ab[k]; l72.ac[k] = lt.ac[k]; }
                p.ltris.push_back(l72);
#else
                p.ltris.push_back(lt);
#endif
#endif
                p.ltri_id.push_back(dm.tri_base + t);
            }
        }
        if (oc.size() > 0 && oc.kind[0]) dm.root_leaf = leaf_of[0];
        // flat octree tables (DevMesh::flat): which leaves hold each triangle, leaf lists ascending
        dm.flat = 0;
        if (oc.size() > 0 && m.num_triangles() <= (size_t)rt::kFlatMaxTris) {
            bool ok = true;
            uint8_t lm[rt::kFlatMaxTris] = {0};
            auto add_leaf = [&](int32_t node, int bit) {
                int32_t prev = -1;
                for (int32_t r = 0; r < oc.leaf_cnt[node]; ++r) {
                    const int32_t t = oc.refs[oc.leaf_off[node] + r];
                    ok &= t > prev && t < (int32_t)m.num_triangles();
                    prev = t;
                    if (ok) lm[t] |= (uint8_t)(1u << bit);
                }
            };
            if (oc.kind[0]) {
                dm.flat_root_leaf = 1;
                dm.flat_kids = 1;
                add_leaf(0, 0);
            } else {
                dm.flat_root_leaf = 0;
                dm.flat_kids = 0;
                for (int k = 0; k < 8 && ok; ++k) {
                    const int32_t c8 = oc.child[k];
                    if (c8 < 0) continue;
                    ok &= oc.kind[c8] != 0;  // every child a leaf
                    if (ok) {
                        dm.flat_kids |= 1 << k;
                        add_leaf(c8, k);
                    }
                }
            }
            if (ok) {
                dm.flat = 1;
                for (int j = 0; j < rt::kFlatMaxTris; ++j) dm.flat_leaf[j / 4] |= (uint32_t)lm[j] << (8 * (j % 4));
            }
        }
        dm.bvh_base = (int32_t)p.bvh.size();
        dm.btri_base = (int32_t)p.btris.size();
        build_bvh(p, m, dm.tri_base);
        dm.bvh_n = (int32_t)p.bvh.size() - dm.bvh_base;
        for (size_t i = 0; i < oc.size(); ++i) {
            p.up.push_back(int2{oc.parent[i] >= 0 ? oc.parent[i] + dm.node_base : -1, oc.slot[i]});
            for (int k = 0; k < 8; ++k) {
                const int32_t c8 = oc.child[8 * i + k];
                if (c8 >= 0 && oc.kind[c8] && leaf_of[c8] >= (1 << 25))  // kid_leaf's escape keeps leaf << 6 in an int32
                    return fail(RT_E_INVAL, "mesh octree too large: leaf ids must stay below 2^25 (scene_layout.h kid_leaf)");
                p.kids.push_back(c8 < 0 ? rt::kKidEmpty
                                 : oc.kind[c8] ? rt::kid_leaf(leaf_of[c8], p.leaves[leaf_of[c8]].x, p.leaves[leaf_of[c8]].y)
                                               : c8 + dm.node_base);
            }
        }
        {
            // subtree triangle bounds (nodes are in DFS pre-order: children after their parent), then each
            // parent's children quantised against the parent's box (scene_layout.h kTightTop)
            std::vector<double> sb(oc.size() * 6);
            auto tri_grow = [&](double* b, uint32_t t) {
                const D3 v[3] = {m.vertices[m.indices[3 * t]], m.vertices[m.indices[3 * t + 1]], m.vertices[m.indices[3 * t + 2]]};
                const rt::DevTri& dt = p.tris[dm.tri_base + t];
                for (int k = 0; k < 3; ++k) {
                    // the vertices, and a + ab / a + ac as tri_t's parametrisation sees them
                    const double c[5] = {k == 0 ? v[0].x : k == 1 ? v[0].y : v[0].z, k == 0 ? v[1].x : k == 1 ? v[1].y : v[1].z,
                                         k == 0 ? v[2].x : k == 1 ? v[2].y : v[2].z, dt.a[k] + dt.ab[k], dt.a[k] + dt.ac[k]};
                    for (double x : c) {
                        b[k] = std::fmin(b[k], x);
                        b[3 + k] = std::fmax(b[3 + k], x);
                    }
                }
            };
            for (size_t j = oc.size(); j-- > 0;) {
                double* b = &sb[6 * j];
                for (int k = 0; k < 3; ++k) { b[k] = INFINITY; b[3 + k] = -INFINITY; }
                if (oc.kind[j]) {
                    for (int32_t r = 0; r < oc.leaf_cnt[j]; ++r) tri_grow(b, (uint32_t)oc.refs[oc.leaf_off[j] + r]);
                } else {
                    for (int k = 0; k < 8; ++k) {
                        const int32_t c8 = oc.child[8 * j + k];
                        if (c8 < 0) continue;
                        for (int q = 0; q < 3; ++q) {
                            b[q] = std::fmin(b[q], sb[6 * (size_t)c8 + q]);
                            b[3 + q] = std::fmax(b[3 + q], sb[6 * (size_t)c8 + 3 + q]);
                        }
                    }
                }
            }
            // every node's box as the walk computes it: the root box, then per level the octant of the
            // parent's box with c = (mn + mx) / 2 (path_f64.h walk_node_slots; DFS pre-order: parents first)
            std::vector<double> nb(6 * oc.size());
            for (size_t j = 0; j < oc.size(); ++j) {
                if (oc.parent[j] < 0) {
                    std::memcpy(&nb[6 * j], rbox, sizeof rbox);
                    continue;
                }
                const double* pb = &nb[6 * (size_t)oc.parent[j]];
                const uint32_t oi = (uint32_t)oc.slot[j];
                for (int k = 0; k < 3; ++k) {
                    const double c = (pb[k] + pb[3 + k]) / 2.0;
                    const bool hi = ((oi >> (2 - k)) & 1u) != 0;
                    nb[6 * j + k] = hi ? c : pb[k];
                    nb[6 * j + 3 + k] = hi ? pb[3 + k] : c;
                }
            }
            // parent ordinals (pid, the slot walk's rows: scene_layout.h KidSlot), DFS order, over all meshes
            std::vector<int32_t> pid(oc.size(), -1);
            for (size_t j = 0; j < oc.size(); ++j)
                if (!oc.kind[j]) {
                    pid[j] = (int32_t)(p.node_box.size() / 6);
                    p.node_box.insert(p.node_box.end(), &nb[6 * j], &nb[6 * j] + 6);
                }
            dm.root_pid = oc.size() > 0 && !oc.kind[0] ? pid[0] : -1;
            for (size_t j = 0; j < oc.size(); ++j)  // each parent's own parent, as a pid (the slot walk's pops
                if (!oc.kind[j]) p.pid_up.push_back(oc.parent[j] >= 0 ? pid[oc.parent[j]] : -1);  // without anc)
            // the 16-bit code range: the cull box's min - E .. min + 2E per axis (E its largest extent)
            double E = 0.0;
            for (int k = 0; k < 3; ++k) E = std::fmax(E, dm.cull_box[3 + k] - dm.cull_box[k]);
            for (int k = 0; k < 3; ++k) dm.tight_base[k] = dm.cull_box[k] - E;
            dm.tight_step = 3.0 * E / (double)rt::kTightTop;
            dm.root_exist = 0;
            if (oc.size() > 0 && !oc.kind[0])
                for (int q = 0; q < 8; ++q) dm.root_exist |= (oc.child[q] >= 0 ? 1 : 0) << q;
            for (size_t j = 0; j < oc.size(); ++j) {
                if (oc.kind[j]) continue;  // rows for parents only (row pid[j])
                for (int k = 0; k < 8; ++k) {
                    const int32_t c8 = oc.child[8 * j + k];
                    double b[6] = {0, 0, 0, 0, 0, 0};
                    if (c8 >= 0)
                        for (int q = 0; q < 3; ++q) {
                            b[q] = sb[6 * (size_t)c8 + q] - dm.cull_pad;
                            b[3 + q] = sb[6 * (size_t)c8 + 3 + q] + dm.cull_pad;
                        }
                    int32_t e = p.kids[8 * (j + (size_t)dm.node_base) + k];
                    if (e >= 0) {  // a parent: its row (pid) and its own existence mask (KidSlot)
                        e = pid[c8];
                        if (e >= slot_max) slots_ok = false;  // checked after the loop: no slot tables
                        uint32_t ex = 0;
                        for (int q = 0; q < 8; ++q) ex |= (oc.child[8 * (size_t)c8 + q] >= 0 ? 1u : 0u) << q;
                        e = rt::slot_parent(e, ex);
                    }
                    bool exact = true;
                    p.slots.push_back(make_slot(e, dm, b, &exact));
                    if (!exact) slots_ok = false;  // a clamped bound code: no slot tables (make_slot)
                }
            }
        }
        p.meshes.push_back(dm);
    }
    if (!slots_ok) {  // the node_kids walk: no slot rows, and no parent boxes (only the slot walk's pops read them)
        p.slots.clear();
        p.pid_up.clear();
        p.node_box.clear();
    }
    for (const Object& o : sc.objects) {
        rt::DevObject d{};
        d.geom = o.geom;
        d.brdf = o.brdf;
        d.mesh = o.mesh;
        d.ph_power = o.ph_power;
        cp3(d.emitted, o.emitted);
        cp3(d.k, o.k);
        cp3(d.pos, o.pos);
        d.r = o.r;
        cp3(d.n, o.n);
        d.ph_kd = o.ph_kd;
        d.ph_ks = o.ph_ks;
        cp3(d.color_d, o.color_d);
        cp3(d.color_s, o.color_s);
        d.emissive = (o.emitted.x != 0.0 || o.emitted.y != 0.0 || o.emitted.z != 0.0) ? 1 : 0;
        d.axis = -1;
        if (o.geom == RT_GEOM_PLANE) {
            const double n3[3] = {o.n.x, o.n.y, o.n.z};
            int nz = 0, ax = -1;
            for (int k = 0; k < 3; ++k)
                if (n3[k] != 0.0) { ++nz; ax = k; }
            if (nz == 1 && std::fabs(n3[ax]) == 1.0) d.axis = ax;
        }
        p.objects.push_back(d);
    }
    // diffuse objects: kd / pi and the NEE term's Le_light * kd / pi, with the device's operations
    // (path_f64.h brdf_eval: ld3(k) * FRAC_1_PI; integrator_f64.h: mult(Le, f)), so the same bits
    const double FRAC_1_PI = 0.318309886183790671537767526745028724;  // path_f64.h FRAC_1_PI
    for (rt::DevObject& d : p.objects) {
        if (d.brdf != rt::BRDF_DIFFUSE) continue;
        for (int k = 0; k < 3; ++k) d.kpi[k] = d.k[k] * FRAC_1_PI;
        if (sc.light >= 0 && sc.light < (int)p.objects.size())
            for (int k = 0; k < 3; ++k) d.lef[k] = p.objects[sc.light].emitted[k] * d.kpi[k];
    }
    return RT_OK;
}

// Groups objects for the compact trace (axis planes per axis, spheres, everything else).
void fill_compact(const Packed& p, rt::CompactTab* ds, int32_t* compact) {
    int nax[3] = {0, 0, 0}, ns = 0, ng = 0;
    bool ok = p.objects.size() <= (size_t)rt::kMaxCompactObjects;
    for (size_t i = 0; i < p.objects.size(); ++i) {
        const rt::DevObject& o = p.objects[i];
        if (o.geom == rt::GEOM_PLANE && o.axis >= 0) {
            // A later axis plane at the same coordinate as an earlier one yields the same t for
            // every ray (the axis path divides (pos_k - o_k) by d_k only), so it can never be the
            // nearest hit (ties go to the lower index, scene.rs:278) nor change a shadow test:
            // leave it out (cornell_box.toml's "wall behind camera" repeats the right wall).
            bool dup = false;
            for (int j = 0; j < nax[o.axis]; ++j) dup |= ds->ax_pos[o.axis][j] == o.pos[o.axis];
            if (dup) continue;
            if (nax[o.axis] == rt::kMaxAxisPlanes) { ok = false; break; }
            ds->ax_idx[o.axis][nax[o.axis]] = (int32_t)i;
            ds->ax_pos[o.axis][nax[o.axis]] = o.pos[o.axis];
            ++nax[o.axis];
        } else if (o.geom == rt::GEOM_SPHERE) {
            if (ns == rt::kMaxSpheres) { ok = false; break; }
            ds->sph_idx[ns] = (int32_t)i;
            ds->sph[ns][0] = o.pos[0];
            ds->sph[ns][1] = o.pos[1];
            ds->sph[ns][2] = o.pos[2];
            ds->sph[ns][3] = o.r * o.r;
            ++ns;
        } else {
            if (ng == rt::kMaxGeneric) { ok = false; break; }
            ds->gen_idx[ng++] = (int32_t)i;
        }
    }
    *compact = ok ? 1 : 0;
    for (int k = 0; k < 3; ++k) ds->n_ax[k] = ok ? nax[k] : 0;
    ds->n_sph = ok ? ns : 0;
    ds->n_gen = ok ? ng : 0;
    ds->last_mesh_g = -1;
    for (int g = 0; g < ds->n_gen; ++g)
        if (p.objects[ds->gen_idx[g]].geom == rt::GEOM_MESH) ds->last_mesh_g = g;
    ds->gen_analytic = 0;
    for (int g = 0; g < rt::kMaxGeneric; ++g) {
        ds->gen_mesh[g] = -1;
        if (g >= ds->n_gen) continue;
        const rt::DevObject& o = p.objects[ds->gen_idx[g]];
        if (o.geom == rt::GEOM_SPHERE || o.geom == rt::GEOM_PLANE) ds->gen_analytic |= 1u << g;
        if (o.geom == rt::GEOM_MESH && o.mesh >= 0 && o.mesh < (int)p.meshes.size() && p.meshes[o.mesh].n_nodes > 0) {
            const rt::DevMesh& m = p.meshes[o.mesh];
            ds->gen_mesh[g] = o.mesh;
            for (int k = 0; k < 6; ++k) ds->gen_cull32[g][k] = m.cull32[k];
            ds->gen_cull32[g][6] = m.cull32_s;
        }
    }
}

// f32 perf-mode tables (scene_layout.h: Obj32 / Bvh32 / Tri32). BVH boxes are rounded outward and
// padded by a few f32 ulps of their largest coordinate, so the f32 slab test never culls a box the
// f64 one would enter; off32 (the hit-point offset) is 2^-16 of the scene's largest coordinate.
float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
}
float f32_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}
void pack_f32(const Packed& p, std::vector<rt::Obj32>* objs, std::vector<rt::Bvh32>* bvh,
              std::vector<rt::Tri32>* tris, float* off32) {
    double scale = 1.0;
    auto grow = [&](double v) { scale = std::max(scale, std::fabs(v)); };
    for (const auto& o : p.objects) {
        rt::Obj32 q{};
        q.geom = o.geom;
        q.brdf = o.brdf;
        q.mesh = o.mesh;
        q.emissive = o.emissive;
        for (int k = 0; k < 3; ++k) {
            q.emitted[k] = (float)o.emitted[k];
            q.k[k] = (float)o.k[k];
            q.pos[k] = (float)o.pos[k];
            q.n[k] = (float)o.n[k];
            if (o.geom == rt::GEOM_SPHERE) grow(std::fabs(o.pos[k]) + o.r);
            else if (o.geom == rt::GEOM_PLANE && o.n[k] != 0.0) grow(o.pos[k]);
        }
        q.axis = o.geom == rt::GEOM_PLANE ? o.axis : -1;
        q.r = (float)o.r;
        q.r2 = (float)(o.r * o.r);
        objs->push_back(q);
    }
    for (const auto& m : p.meshes)
        for (int k = 0; k < 6; ++k) grow(m.root_box[k]);
    for (const auto& n : p.bvh) {
        rt::Bvh32 q{};
        double pad = 0.0;
        for (int k = 0; k < 3; ++k) pad = std::max({pad, std::fabs(n.bmin[k]), std::fabs(n.bmax[k])});
        pad *= 0x1p-20;
        for (int k = 0; k < 3; ++k) {
            q.bmin[k] = f32_down(n.bmin[k] - pad);
            q.bmax[k] = f32_up(n.bmax[k] + pad);
        }
        q.a = n.a;
        q.cnt_axis = n.count * 4 + n.axis;
        bvh->push_back(q);
    }
    for (const auto& t : p.btris) {
        rt::Tri32 q{};
        for (int k = 0; k < 3; ++k) {
            q.a[k] = (float)t.a[k];
            q.ab[k] = (float)t.ab[k];
            q.ac[k] = (float)t.ac[k];
            q.n[k] = (float)t.n[k];
        }
        tris->push_back(q);
    }
    *off32 = (float)std::max(1e-5, scale * 0x1p-16);
}

template <class T>
void put(std::vector<char>& blob, size_t* off, const std::vector<T>& v) {
    *off = align_up(blob.size(), 256);
    blob.resize(*off + v.size() * sizeof(T) + 16);
    if (!v.empty()) std::memcpy(blob.data() + *off, v.data(), v.size() * sizeof(T));
}

int upload(rt_scene* s, int device, rt::DevScene* out) {
    std::lock_guard<std::mutex> lk(s->mu);
    if ((int)s->dev.size() <= device) s->dev.resize(device + 1);
    DeviceCopy& dc = s->dev[device];
    if (!dc.ready) {
        const Packed& p = s->packed;
        std::vector<char> blob;
        size_t o_obj, o_mesh, o_kids, o_up, o_leaf, o_ltri, o_lid, o_tris, o_cum, o_tab, o_bvh, o_btri, o_bid;
        size_t o_obj32, o_bvh32, o_tri32;
        std::vector<rt::Obj32> obj32;
        std::vector<rt::Bvh32> bvh32;
        std::vector<rt::Tri32> tri32;
        float off32 = 0.f;
        pack_f32(p, &obj32, &bvh32, &tri32, &off32);
        std::vector<rt::CompactTab> tab(1);
        std::memset(tab.data(), 0, sizeof(rt::CompactTab));
        int32_t compact = 0;
        fill_compact(p, tab.data(), &compact);
        put(blob, &o_tab, tab);
        std::vector<rt::Compact32> tab32(1);
        {
            rt::Compact32& c = tab32[0];
            std::memset(&c, 0, sizeof c);
            const rt::CompactTab& t = tab[0];
            c.ok = compact;
            for (int k = 0; k < 3; ++k) {
                c.n_ax[k] = t.n_ax[k];
                for (int j = 0; j < rt::kMaxAxisPlanes; ++j) {
                    c.ax_idx[k][j] = t.ax_idx[k][j];
                    c.ax_pos[k][j] = (float)t.ax_pos[k][j];
                }
            }
            c.n_sph = t.n_sph;
            c.n_gen = t.n_gen;
            for (int j = 0; j < rt::kMaxSpheres; ++j) {
                c.sph_idx[j] = t.sph_idx[j];
                for (int q = 0; q < 4; ++q) c.sph[j][q] = (float)t.sph[j][q];
            }
            for (int j = 0; j < rt::kMaxGeneric; ++j) c.gen_idx[j] = t.gen_idx[j];
        }
        size_t o_tab32;
        put(blob, &o_tab32, tab32);
        put(blob, &o_obj, p.objects);
        put(blob, &o_mesh, p.meshes);
        put(blob, &o_kids, p.kids);
        put(blob, &o_up, p.up);
        put(blob, &o_leaf, p.leaves);
        put(blob, &o_ltri, p.ltris);
        put(blob, &o_lid, p.ltri_id);
        put(blob, &o_tris, p.tris);
        put(blob, &o_cum, p.cum_area);
        put(blob, &o_bvh, p.bvh);
        put(blob, &o_btri, p.btris);
        put(blob, &o_bid, p.btri_id);
        put(blob, &o_obj32, obj32);
        put(blob, &o_bvh32, bvh32);
        put(blob, &o_tri32, tri32);
        size_t o_slot;
        put(blob, &o_slot, p.slots);
        size_t o_nbox, o_pup;
        put(blob, &o_nbox, p.node_box);
        put(blob, &o_pup, p.pid_up);
        void* d = nullptr;
        HIP_TRY(hipMalloc(&d, blob.size()));
        hipError_t e = hipMemcpy(d, blob.data(), blob.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return fail(RT_E_HIP, std::string("scene upload: ") + hipGetErrorString(e));
        }
        char* b = (char*)d;
        rt::DevScene ds{};
        ds.objects = (const rt::DevObject*)(b + o_obj);
        ds.meshes = (const rt::DevMesh*)(b + o_mesh);
        ds.node_kids = (const int32_t*)(b + o_kids);
        ds.node_up = (const int2*)(b + o_up);
        ds.leaf_span = (const int2*)(b + o_leaf);
        ds.ltris = (const rt::LeafTri*)(b + o_ltri);
        ds.ltri_id = (const int32_t*)(b + o_lid);
        ds.tris = (const rt::DevTri*)(b + o_tris);
        ds.tri_cum_area = (const double*)(b + o_cum);
        ds.n_objects = (int32_t)p.objects.size();
        ds.ctab = (const rt::CompactTab*)(b + o_tab);
        ds.bvh = (const rt::DevBvhNode*)(b + o_bvh);
        ds.btris = (const rt::DevTri*)(b + o_btri);
        ds.btri_id = (const int32_t*)(b + o_bid);
        ds.obj32 = (const rt::Obj32*)(b + o_obj32);
        ds.bvh32 = (const rt::Bvh32*)(b + o_bvh32);
        ds.btris32 = (const rt::Tri32*)(b + o_tri32);
        ds.off32 = off32;
        ds.ctab32 = (const rt::Compact32*)(b + o_tab32);
        ds.compact = compact;
        ds.node_slot = p.slots.empty() ? nullptr : (const rt::KidSlot*)(b + o_slot);
        ds.node_box = p.slots.empty() ? nullptr : (const double*)(b + o_nbox);
        ds.pid_up = p.slots.empty() ? nullptr : (const int32_t*)(b + o_pup);
        ds.n_pid = p.slots.empty() ? 0 : (int32_t)p.pid_up.size();
        // RT_TEST_ANC_OFF (tests only): report more pids than a 16-bit ancestor column holds, so the role
        // pool's walkers pop through pid_up (the path of octrees with > 65536 parents)
        if (std::getenv("RT_TEST_ANC_OFF") && ds.n_pid > 0) ds.n_pid = 0x7FFFFFFF;
        ds.light = s->host.light;
        ds.light_pdf = 0.0;
        if (ds.light >= 0 && ds.light < (int32_t)p.objects.size()) {
            const rt::DevObject& L = p.objects[ds.light];
            const double PI = 3.14159265358979323846264338327950288;  // path_f64.h PI
            if (L.geom == rt::GEOM_SPHERE) ds.light_pdf = 1.0 / (4.0 * PI * L.r * L.r);  // geometry.rs:583
            else if (L.geom == rt::GEOM_MESH) ds.light_pdf = 1. / p.meshes[L.mesh].surface_area;  // :591
        }
        ds.n_meshes = (int32_t)p.meshes.size();
        cp3(ds.cam_pos, s->host.cam_pos);
        cp3(ds.cam_dir, s->host.cam_dir);
        dc.blob = d;
        dc.ds = ds;
        dc.ready = true;
    }
    *out = dc.ds;
    return RT_OK;
}

int check_params(const rt_render_params* p) {
    if (!p) return fail(RT_E_INVAL, "null params");
    if (p->width <= 0 || p->height <= 0) return fail(RT_E_INVAL, "width/height must be positive");
    if (p->row_step < 0) return fail(RT_E_INVAL, "row_step must be >= 0");
    const int64_t step = p->row_step > 1 ? p->row_step : 1;
    if (p->tile_w < 0 || p->tile_h < 0 || p->x0 < 0 || p->y0 < 0 || p->x0 + p->tile_w > p->width ||
        (p->tile_h > 0 && p->y0 + (int64_t)(p->tile_h - 1) * step >= p->height))
        return fail(RT_E_INVAL, "tile outside the image");
    if ((int64_t)p->width * p->height > (int64_t)UINT32_MAX) return fail(RT_E_INVAL, "image too large for 32-bit pixel ids");
    return RT_OK;
}

// Per-render scratch (ticket counter, subpixel buffer, split-tail buffer, wavefront streams) comes
// from a per-scene pool. rt_render_device returns before its kernels finish, so a pooled workspace
// may still be in use: an idle one (its completion event has fired) is taken first; else one last
// used on the same stream, with a device-side wait on its completion event enqueued on `st` (so the
// reuse is ordered even if the caller destroyed that stream and HIP handed its handle to a new one);
// otherwise a new workspace is made (concurrent renders on one scene each get their own, rt_ffi.h).
// A reused in-flight workspace never reallocates under its previous kernels: Workspace::ensure_*
// wait for `busy` before freeing (wavefront_f64.hip).
std::unique_ptr<rt::Workspace> take_workspace(rt_scene* s, int device, hipStream_t st, hipError_t* err) {
    std::lock_guard<std::mutex> lk(s->mu);
    size_t idle = s->pool.size(), same = s->pool.size();
    for (size_t i = 0; i < s->pool.size(); ++i) {
        rt::Workspace& w = *s->pool[i];
        if (w.device != device) continue;
        if (!w.in_flight || hipEventQuery(w.busy) == hipSuccess) {
            idle = i;
            break;
        }
        if (w.last_stream == st && same == s->pool.size()) same = i;
    }
    (void)hipGetLastError();  // hipErrorNotReady from the queries is not an error
    *err = hipSuccess;
    const size_t pick = idle < s->pool.size() ? idle : same;
    if (pick < s->pool.size()) {
        std::unique_ptr<rt::Workspace> w = std::move(s->pool[pick]);
        s->pool.erase(s->pool.begin() + pick);
        if (pick == idle) {
            w->in_flight = false;
        } else {
            *err = hipStreamWaitEvent(st, w->busy, 0);
            if (*err != hipSuccess) {  // keep it pooled; the caller fails the render
                s->pool.push_back(std::move(w));
                return nullptr;
            }
        }
        return w;
    }
    auto w = std::make_unique<rt::Workspace>();
    w->device = device;
    return w;
}
void give_workspace(rt_scene* s, std::unique_ptr<rt::Workspace> w, hipStream_t st) {
    hipError_t e = hipSuccess;
    if (!w->busy) e = hipEventCreateWithFlags(&w->busy, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(w->busy, st);
    if (e != hipSuccess) {  // cannot track its completion: wait for it here
        (void)hipGetLastError();
        (void)hipStreamSynchronize(st);
        w->in_flight = false;
    } else {
        w->in_flight = true;
        w->last_stream = st;
    }
    std::lock_guard<std::mutex> lk(s->mu);
    s->pool.push_back(std::move(w));
}

// Device-visible mirror of a caller's cancel flag: a pinned, mapped word the megakernels poll
// (RenderArgs::cancel) between subpixels. The caller's flag itself is never registered with HIP (it
// may be shared by concurrent renders, or sit on memory HIP cannot pin): the host thread that waits
// for the render copies it into the mirror (wait_stream), so its lifetime stays the caller's.
// The words come from a process-wide free list and go back to it once the render has drained: a
// cancellable render (the WebSocket server renders chunk by chunk with a flag) costs no pinned
// allocation after the first. The words are never freed (one per concurrently cancellable render).
struct CancelWord {
    int32_t* host;
    int32_t* dev;
};
struct CancelWordPool {
    std::mutex mu;
    std::vector<CancelWord> free;
};
CancelWordPool& cancel_words() {
    static CancelWordPool* pool = new CancelWordPool;  // never destroyed: no HIP calls at process teardown
    return *pool;
}
struct CancelMirror {
    int32_t* host = nullptr;
    int32_t* dev = nullptr;
    CancelMirror() = default;
    CancelMirror(const CancelMirror&) = delete;
    CancelMirror& operator=(const CancelMirror&) = delete;
    ~CancelMirror() {
        if (!host) return;
        CancelWordPool& p = cancel_words();
        std::lock_guard<std::mutex> lk(p.mu);
        p.free.push_back(CancelWord{host, dev});
    }
    hipError_t init() {
        {
            CancelWordPool& p = cancel_words();
            std::lock_guard<std::mutex> lk(p.mu);
            if (!p.free.empty()) {
                host = p.free.back().host;
                dev = p.free.back().dev;
                p.free.pop_back();
            }
        }
        if (!host) {
            // coherent (fine-grained): hipHostMalloc's default is non-coherent memory the GPU may cache, so
            // a host write could stay invisible to the polling kernel until the line is evicted
            hipError_t e = hipHostMalloc((void**)&host, sizeof(int32_t),
                                         hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent);
            if (e != hipSuccess) {
                host = nullptr;
                return e;
            }
            e = hipHostGetDevicePointer((void**)&dev, host, 0);
            if (e != hipSuccess) {
                (void)hipHostFree(host);
                host = nullptr;
                return e;
            }
        }
        __atomic_store_n(host, 0, __ATOMIC_RELEASE);
        return hipSuccess;
    }
    void raise() {
        if (host) __atomic_store_n(host, 1, __ATOMIC_RELEASE);
    }
};

// Waits for everything enqueued on `st`, copying the caller's cancel flag into the mirror meanwhile.
// Polls with a growing pause (10 us doubling to 200 us), so a short render (one WebSocket chunk) is
// seen done within about its own duration.
hipError_t wait_stream(hipStream_t st, const volatile int32_t* cancel, CancelMirror* mirror) {
    if (!cancel || !mirror || !mirror->host) return hipStreamSynchronize(st);
    int us = 10;
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        if (*cancel) mirror->raise();
        std::this_thread::sleep_for(std::chrono::microseconds(us));
        us = std::min(200, 2 * us);
    }
}

// Statistics of an enqueued megakernel render, completed once its stream has drained (finish): the
// render's HIP events and a pinned copy of the workspace's vertex counter (copied on the stream
// before the workspace goes back to the pool). Nothing here synchronises, so callers can keep several
// renders in flight (rt_render_multi) and still collect their stats. The events and the pinned word
// are made by the first init and reused by later ones (rt_render_multi: one PendingStats per band
// slot of a worker), and freed only when the object goes (after its renders have drained).
struct PendingStats {
    rt_render_stats* out = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    unsigned long long* count = nullptr;  // pinned host word
    int64_t samples = 0;
    bool device_done = false;  // the wavefront path filled `out` itself
    PendingStats() = default;
    PendingStats(const PendingStats&) = delete;
    PendingStats& operator=(const PendingStats&) = delete;
    ~PendingStats() {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (count) (void)hipHostFree(count);
    }
    hipError_t init(rt_render_stats* o) {
        out = o;
        std::memset(out, 0, sizeof *out);
        device_done = false;
        hipError_t e = hipSuccess;
        if (!e0) e = hipEventCreate(&e0);
        if (e == hipSuccess && !e1) e = hipEventCreate(&e1);
        if (e == hipSuccess && !count) e = hipHostMalloc((void**)&count, sizeof(unsigned long long), hipHostMallocDefault);
        if (e == hipSuccess) *count = 0;
        return e;
    }
    // after the render's stream has completed
    int finish(std::string* err) {
        if (!out) return RT_OK;
        if (!device_done) {
            float ms = 0.f;
            const hipError_t e = hipEventElapsedTime(&ms, e0, e1);
            if (e != hipSuccess) {
                *err = std::string("stats: ") + hipGetErrorString(e);
                return RT_E_HIP;
            }
            out->device_ms = ms;
            out->kernel_ms[0] = ms;
            out->kernel_launches[0] = 1;
            out->vertices = (int64_t)*count;
        }
        out->samples = samples;
        return RT_OK;
    }
};

// Enqueue one render on `st` (device buffers); returns without waiting for the device (except in
// wavefront mode, whose host loop drives the bounces and polls host_cancel). dcancel: device view of
// a cancel word the megakernels poll (CancelMirror::dev) or null; ps: stats to complete after the
// stream drains (PendingStats::finish) or null.
int render_enqueue(rt_scene* s, const rt_render_params* p, uint8_t* d_rgb, double* d_sub, hipStream_t st,
                   const int32_t* dcancel, const volatile int32_t* host_cancel, PendingStats* ps) {
    int rc = check_params(p);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipSetDevice(p->device));
    rt::DevScene ds;
    rc = upload(s, p->device, &ds);
    if (rc != RT_OK) return rc;
    rt::RenderArgs a{};
    a.width = p->width;
    a.height = p->height;
    a.x0 = p->x0;
    a.y0 = p->y0;
    a.row_step = p->row_step > 1 ? p->row_step : 1;
    a.tw = p->tile_w;
    a.th = p->tile_h;
    a.n_samples = p->spp > 0 ? p->spp / 4 : 0;  // server.rs:332 (i32 division)
    a.mis = (p->flags & RT_FLAG_MIS) ? 1 : 0;
    {
        bool phong = false, spec = false;
        for (const auto& o : s->host.objects) {
            phong |= o.brdf == RT_BRDF_PHONG;
            spec |= o.brdf == RT_BRDF_SPECULAR;
        }
        a.features = (s->host.meshes.empty() ? 0 : 1) | (phong ? 2 : 0) | (a.mis ? 4 : 0) | (ds.compact ? 8 : 0) |
                     (spec ? 0 : 32);
        if ((p->flags & RT_FLAG_MESH_NEAREST) && !s->host.meshes.empty()) a.features |= 16;
        for (const auto& m : s->host.meshes) a.mesh_nodes = std::max(a.mesh_nodes, (int32_t)m.octree.size());
        a.all_flat = !s->packed.meshes.empty() && s->packed.meshes.size() <= (size_t)rt::kFlatMeshes;
        for (const auto& dm : s->packed.meshes) a.all_flat &= dm.flat != 0;
    }
    a.seed = p->seed;
    rt::host::camera_frame(s->host, p->width, p->height, a.cx, a.cy);
    a.inv_n = a.n_samples > 0 ? 1. / (double)a.n_samples : 0.0;
    a.sub_out = d_sub;
    a.rgb_out = d_rgb;
    const bool fp32 = (p->flags & RT_FLAG_FP32) != 0;
    if (fp32) {
        // the f32 kernel covers diffuse / mirror BRDFs and sphere lights (every reference scene)
        for (const auto& o : s->host.objects)
            if (o.brdf == RT_BRDF_PHONG) return fail(RT_E_INVAL, "RT_FLAG_FP32: Phong BRDFs need the f64 path");
        const auto& L = s->packed.objects;
        if (ds.light >= 0 && ds.light < (int32_t)L.size() && L[ds.light].geom != rt::GEOM_SPHERE)
            return fail(RT_E_INVAL, "RT_FLAG_FP32: only sphere lights (mesh lights need the f64 path)");
    }
    if (!fp32 && (p->flags & RT_FLAG_MESH_NEAREST) && !(p->flags & RT_FLAG_MEGAKERNEL))
        return fail(RT_E_INVAL, "RT_FLAG_MESH_NEAREST needs RT_FLAG_MEGAKERNEL");
    const bool mk = fp32 || (p->flags & RT_FLAG_MEGAKERNEL);
    if (ps) {
        const hipError_t e = ps->init(ps->out);
        if (e != hipSuccess) return fail(RT_E_HIP, std::string("stats: ") + hipGetErrorString(e));
        ps->samples = (int64_t)p->tile_w * p->tile_h * 4 * (int64_t)a.n_samples;
        HIP_TRY(hipEventRecord(ps->e0, st));
    }
    hipError_t te;
    std::unique_ptr<rt::Workspace> ws = take_workspace(s, p->device, st, &te);
    if (!ws) return fail(RT_E_HIP, std::string("workspace: ") + hipGetErrorString(te));
    int out = RT_OK;
    std::string err;
    if (mk) {
        const size_t npix = (size_t)p->tile_w * p->tile_h;
        a.cancel = dcancel;
        hipError_t e = ws->ensure_counters();
        double* sub = d_sub;
        if (e == hipSuccess && !sub) {
            e = ws->ensure_sub(npix);
            sub = ws->sub_buf;
        }
        if (e == hipSuccess && ps) e = hipMemsetAsync(ws->counters, 0, 8 * sizeof(unsigned long long), st);
        if (e == hipSuccess && a.n_samples <= 0) e = hipMemsetAsync(sub, 0, npix * 12 * sizeof(double), st);
        if (e == hipSuccess) {
            a.counters = ps ? ws->counters : nullptr;
            // split-tail scratch (megakernel_common.h plan_tail): the samples after chunk 0 of the subpixels a
            // launch splits — kernels.h tail_split_x2 / 2 per resident lane in the analytic and flat-mesh kernels
            // (no more than 1024 lanes per CU: 4 waves/SIMD, the 1024-thread query pool), so 1536 per CU (393,216 on
            // 256 CUs: 2.1 GB at 1024 spp), 2048 for frames of <= 4 subpixels per lane; six per path slot in the
            // mesh walk kernels (<= 1024 slots per CU) — at most 3 GB. A smaller buffer only splits fewer
            // subpixels (plan_tail; rt_debug_last_split reports the split wanted and made), with the same frame bits.
            const bool walk = (a.features & 1) && !a.all_flat;
            int dev = 0, ncu = 256;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
            const size_t per_sub = rt::tail_scratch_per_subpixel(a.n_samples);
            // (A/B builds: RT_MK_TAIL_SCRATCH_PER_CU / RT_MK_TAIL_SCRATCH_MB override both bounds, ab_knobs.h)
            const long ncu_lanes = (long)std::max(ncu, 1) * 1024;
            const size_t per_cu = (size_t)rt::ab_knob("RT_MK_TAIL_SCRATCH_PER_CU",
                                                      walk ? 6 * 1024 : 512 * rt::tail_split_x2((long)npix * 4, ncu_lanes));
            const size_t cap = (size_t)rt::ab_knob("RT_MK_TAIL_SCRATCH_MB", 3072) << 20;
            const size_t want = std::min<size_t>(cap, per_sub * std::min<size_t>(npix * 4, (size_t)std::max(ncu, 1) * per_cu));
            if (!fp32 && per_sub > 0 && want >= per_sub) {
                if (ws->ensure_tail(want) != hipSuccess) (void)hipGetLastError();  // no tail split then
            }
            if (fp32) {
                static const int brute = (int)rt::ab_knob("RT_F32_BRUTE", 16);
                a.f32_brute = brute;
                e = rt::launch_megakernel_f32(ds, a, sub, (uint32_t*)(ws->counters + 4), st);
            } else {
                e = rt::launch_megakernel_f64(ds, a, sub, (uint32_t*)(ws->counters + 4), ws->tail_buf, ws->tail_cap, st);
            }
        }
        if (e == hipSuccess) e = rt::launch_finalize_f64(a, sub, st);
        if (e == hipSuccess && ps) e = hipEventRecord(ps->e1, st);
        if (e == hipSuccess && ps) e = hipMemcpyAsync(ps->count, ws->counters, sizeof(unsigned long long), hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) { out = RT_E_HIP; err = std::string("megakernel: ") + hipGetErrorString(e); }
    } else {
        out = rt::wavefront_render_f64(ds, a, *ws, st, host_cancel, ps ? ps->out : nullptr, &err);
        if (ps && out >= 0) {
            hipError_t e = hipEventRecord(ps->e1, st);
            if (e == hipSuccess) e = hipEventSynchronize(ps->e1);
            float ms = 0.f;
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, ps->e0, ps->e1);
            if (e != hipSuccess && out == RT_OK) { out = RT_E_HIP; err = std::string("stats: ") + hipGetErrorString(e); }
            ps->out->device_ms = ms;
            ps->device_done = true;
        }
    }
    give_workspace(s, std::move(ws), st);
    if (out < 0) return fail(out, err);
    return out;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static int finish_scene(rt::host::Scene&& sc, rt_scene** out) {
    auto s = std::make_unique<rt_scene>();
    s->host = std::move(sc);
    const int rc = pack_scene(s.get());
    if (rc != RT_OK) return rc;
    *out = s.release();
    return RT_OK;
}

int rt_scene_load_toml(const char* toml_path, const char* assets_dir, rt_scene** out) {
    if (!toml_path || !out) return fail(RT_E_INVAL, "null argument");
    *out = nullptr;
    std::string path(toml_path), assets;
    if (assets_dir) assets = assets_dir;
    else {
        size_t sl = path.find_last_of('/');
        assets = (sl == std::string::npos ? std::string(".") : path.substr(0, sl)) + "/assets";
    }
    rt::host::Scene sc;
    std::string err;
    int rc = rt::host::load_scene_toml(path, assets, &sc, &err);
    if (rc != RT_OK) return fail(rc, err);
    return finish_scene(std::move(sc), out);
}

int rt_scene_create(const rt_scene_desc* desc, rt_scene** out) {
    if (!out) return fail(RT_E_INVAL, "null argument");
    *out = nullptr;
    rt::host::Scene sc;
    std::string err;
    int rc = rt::host::scene_from_desc(desc, &sc, &err);
    if (rc != RT_OK) return fail(rc, err);
    return finish_scene(std::move(sc), out);
}

void rt_scene_destroy(rt_scene* s) { delete s; }

int rt_scene_info(const rt_scene* s, int64_t info[16]) {
    if (!s || !info) return fail(RT_E_INVAL, "null argument");
    std::memset(info, 0, 16 * sizeof(int64_t));
    info[0] = (int64_t)s->host.objects.size();
    info[1] = s->host.light;
    info[2] = (int64_t)s->host.meshes.size();
    for (const auto& m : s->host.meshes) {
        info[3] += (int64_t)m.octree.size();
        info[4] += m.octree.parents;
        info[5] += m.octree.leaves;
        info[6] += (int64_t)m.octree.refs.size();
        info[7] += (int64_t)m.num_triangles();
        info[8] += (int64_t)m.vertices.size();
        if (m.octree.max_leaf > info[9]) info[9] = m.octree.max_leaf;
        if (m.octree.max_depth > info[10]) info[10] = m.octree.max_depth;
    }
    info[11] = s->packed.slots.empty() ? 0 : 1;
    return RT_OK;
}

int rt_scene_mesh(const rt_scene* s, int32_t object, int64_t counts[4], double bbox[6], double* surface_area,
                  double* vertices, uint32_t* indices, int32_t* kind, int32_t* child, int32_t* leaf_off,
                  int32_t* leaf_cnt, int32_t* refs) {
    if (!s || object < 0 || (size_t)object >= s->host.objects.size()) return fail(RT_E_INVAL, "bad object index");
    const auto& o = s->host.objects[object];
    if (o.geom != RT_GEOM_MESH) return fail(RT_E_INVAL, "object is not a mesh");
    const auto& m = s->host.meshes[o.mesh];
    const auto& oc = m.octree;
    if (counts) {
        counts[0] = (int64_t)oc.size();
        counts[1] = (int64_t)oc.refs.size();
        counts[2] = (int64_t)m.num_triangles();
        counts[3] = (int64_t)m.vertices.size();
    }
    if (bbox) {
        double b[6] = {m.bbox.min.x, m.bbox.min.y, m.bbox.min.z, m.bbox.max.x, m.bbox.max.y, m.bbox.max.z};
        std::memcpy(bbox, b, sizeof b);
    }
    if (surface_area) *surface_area = m.surface_area;
    if (vertices)
        for (size_t i = 0; i < m.vertices.size(); ++i) {
            vertices[3 * i] = m.vertices[i].x;
            vertices[3 * i + 1] = m.vertices[i].y;
            vertices[3 * i + 2] = m.vertices[i].z;
        }
    if (indices) std::memcpy(indices, m.indices.data(), m.indices.size() * sizeof(uint32_t));
    for (size_t i = 0; i < oc.size(); ++i) {
        if (kind) kind[i] = oc.kind[i];
        if (child) std::memcpy(child + 8 * i, &oc.child[8 * i], 8 * sizeof(int32_t));
        if (leaf_off) leaf_off[i] = oc.leaf_off[i];
        if (leaf_cnt) leaf_cnt[i] = oc.leaf_cnt[i];
    }
    if (refs) std::memcpy(refs, oc.refs.data(), oc.refs.size() * sizeof(int32_t));
    return RT_OK;
}

int rt_render_device(const rt_scene* scene, const rt_render_params* params, void* d_rgb, void* d_sub, void* stream,
                     rt_render_stats* stats) {
    if (!scene || !d_rgb) return fail(RT_E_INVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    PendingStats ps;
    ps.out = stats;
    int rc = render_enqueue(const_cast<rt_scene*>(scene), params, (uint8_t*)d_rgb, (double*)d_sub, st, nullptr, nullptr,
                            stats ? &ps : nullptr);
    if (rc < 0 || !stats) return rc;
    const hipError_t e = hipStreamSynchronize(st);  // stats: synchronous with respect to the stream (rt_ffi.h)
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("stats sync: ") + hipGetErrorString(e));
    std::string err;
    const int f = ps.finish(&err);
    return f < 0 ? fail(f, err) : rc;
}

int rt_render(const rt_scene* scene, const rt_render_params* p, uint8_t* rgb_out, double* sub_out,
              const volatile int32_t* cancel, rt_render_stats* stats) {
    if (!scene || !rgb_out) return fail(RT_E_INVAL, "null argument");
    int rc = check_params(p);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipSetDevice(p->device));
    size_t npix = (size_t)p->tile_w * p->tile_h;
    if (npix == 0) return RT_OK;
    uint8_t* d_rgb = nullptr;
    double* d_sub = nullptr;
    hipStream_t st = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipError_t e = hipMalloc(&d_rgb, npix * 3);
    if (e == hipSuccess && sub_out) e = hipMalloc(&d_sub, npix * 12 * sizeof(double));
    CancelMirror mirror;
    if (e == hipSuccess && cancel) e = mirror.init();
    if (e != hipSuccess) {
        if (d_rgb) (void)hipFree(d_rgb);
        if (d_sub) (void)hipFree(d_sub);
        (void)hipStreamDestroy(st);
        return fail(e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP, std::string("output buffers: ") + hipGetErrorString(e));
    }
    rt_render_stats local;
    PendingStats ps;
    ps.out = stats ? stats : &local;
    rc = render_enqueue(const_cast<rt_scene*>(scene), p, d_rgb, d_sub, st, mirror.dev, cancel, &ps);
    std::string err = g_err;
    if (rc == RT_OK) {
        // wait for the render first (relaying the cancel flag), then copy back: a copy into the
        // caller's pageable buffers would block inside hipMemcpyAsync until the kernel ends, with
        // nobody relaying the flag
        e = wait_stream(st, cancel, &mirror);
        if (e == hipSuccess) e = hipMemcpyAsync(rgb_out, d_rgb, npix * 3, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess && sub_out) e = hipMemcpyAsync(sub_out, d_sub, npix * 12 * sizeof(double), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) { rc = RT_E_HIP; err = std::string("readback: ") + hipGetErrorString(e); }
        if (rc == RT_OK) {
            const int f = ps.finish(&err);
            if (f < 0) rc = f;
        }
        if (rc == RT_OK && cancel && *cancel) rc = RT_CANCELLED;
    } else {
        (void)hipStreamSynchronize(st);
    }
    (void)hipFree(d_rgb);
    if (d_sub) (void)hipFree(d_sub);
    (void)hipStreamDestroy(st);
    if (rc < 0) return fail(rc, err);
    return rc;
}

int32_t rt_band_plan(int32_t tile_h, int32_t n_workers, int32_t band_rows, int32_t cap, int32_t* first_row,
                     int32_t* rows) {
    if (tile_h <= 0) return 0;
    if (n_workers < 1) n_workers = 1;
    int32_t b = band_rows;
    if (b <= 0) b = std::max<int32_t>(1, (int32_t)(((int64_t)tile_h + 8LL * n_workers - 1) / (8LL * n_workers)));
    const int32_t n = (int32_t)(((int64_t)tile_h + b - 1) / b);
    for (int32_t i = 0; i < n && i < cap; ++i) {
        if (first_row) first_row[i] = i * b;
        if (rows) rows[i] = std::min(b, tile_h - i * b);
    }
    return n;
}

int rt_render_multi(const rt_scene* scene, const rt_render_params* p, const int32_t* devices, int32_t n_devices,
                    int32_t band_rows, uint8_t* rgb_out, const volatile int32_t* cancel, rt_render_stats* stats) {
    if (!scene || !rgb_out || !devices || n_devices <= 0) return fail(RT_E_INVAL, "null argument");
    int rc = check_params(p);
    if (rc != RT_OK) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {  // no GPU or no runtime: not the caller's error
        (void)hipGetLastError();
        return fail(RT_E_NODEVICE, "rt_render_multi: no HIP device visible");
    }
    // an ordinal no visible device has is the caller's error (RT_E_INVAL), checked before anything runs
    for (int32_t i = 0; i < n_devices; ++i)
        if (devices[i] < 0 || devices[i] >= ndev)
            return fail(RT_E_INVAL, "device ordinal " + std::to_string(devices[i]) + " out of range (" +
                                        std::to_string(ndev) + " HIP devices visible)");
    const int32_t tw = p->tile_w, th = p->tile_h;
    if ((size_t)tw * th == 0) return RT_OK;
    const int32_t nb = rt_band_plan(th, n_devices, band_rows, 0, nullptr, nullptr);
    std::vector<int32_t> first(nb), rows(nb);
    rt_band_plan(th, n_devices, band_rows, nb, first.data(), rows.data());
    int32_t bmax = 0;
    for (int32_t r : rows) bmax = std::max(bmax, r);
    const int64_t step = p->row_step > 1 ? p->row_step : 1;
    std::atomic<int32_t> next{0};
    std::atomic<int> err_code{RT_OK};
    std::atomic<bool> stop{false};
    std::atomic<int64_t> samples{0}, vertices{0};
    std::atomic<int32_t> done{0};
    std::mutex err_mu;
    std::string err_msg;
    const auto t0 = std::chrono::steady_clock::now();
    rt_scene* s = const_cast<rt_scene*>(scene);

    // one device-visible cancel word for every band of the call (the megakernels poll it between
    // subpixels; each worker copies the caller's flag into it while it waits for a band)
    CancelMirror mirror;
    if (cancel) {
        const hipError_t e = mirror.init();
        if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_render_multi: cancel word: ") + hipGetErrorString(e));
    }

    auto worker = [&](int32_t dev) {
        auto record = [&](int code, const std::string& m) {
            std::lock_guard<std::mutex> lk(err_mu);
            if (err_code.load() == RT_OK) { err_code = code; err_msg = m; }
            stop = true;
        };
        if (hipSetDevice(dev) != hipSuccess) { record(RT_E_HIP, "hipSetDevice"); return; }
        constexpr int kSlots = 2;  // bands in flight per worker
        hipStream_t st[kSlots] = {nullptr, nullptr};
        uint8_t* d_rgb[kSlots] = {nullptr, nullptr};
        uint8_t* h_rgb[kSlots] = {nullptr, nullptr};
        int32_t pending[kSlots] = {-1, -1};
        rt_render_stats bs[kSlots];
        PendingStats ps[kSlots];
        const size_t band_bytes = (size_t)bmax * tw * 3;
        bool ok = true;
        for (int k = 0; k < kSlots && ok; ++k) {
            ok = hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) == hipSuccess &&
                 hipMalloc(&d_rgb[k], band_bytes) == hipSuccess &&
                 hipHostMalloc((void**)&h_rgb[k], band_bytes, hipHostMallocDefault) == hipSuccess;
        }
        if (!ok) record(RT_E_OOM, "rt_render_multi: band buffers");
        // finishes band slot k: wait for its copy (relaying the cancel flag), collect its stats, put its
        // rows into the caller's frame
        auto drain = [&](int k) {
            if (pending[k] < 0) return;
            const int32_t b = pending[k];
            pending[k] = -1;
            if (wait_stream(st[k], cancel, &mirror) != hipSuccess) { record(RT_E_HIP, "rt_render_multi: band sync"); return; }
            if (stats) {
                std::string e;
                if (ps[k].finish(&e) < 0) { record(RT_E_HIP, "rt_render_multi: " + e); return; }
                samples += bs[k].samples;
                vertices += bs[k].vertices;
            }
            std::memcpy(rgb_out + (size_t)first[b] * tw * 3, h_rgb[k], (size_t)rows[b] * tw * 3);
            ++done;
        };
        for (int slot = 0; ok && !stop.load(); slot ^= 1) {
            drain(slot);
            if (stop.load() || (cancel && *cancel)) break;
            const int32_t b = next.fetch_add(1);
            if (b >= nb) break;
            rt_render_params q = *p;
            q.device = dev;
            q.y0 = (int32_t)(p->y0 + (int64_t)first[b] * step);
            q.tile_h = rows[b];
            ps[slot].out = &bs[slot];
            const int r = render_enqueue(s, &q, d_rgb[slot], nullptr, st[slot], mirror.dev, cancel, stats ? &ps[slot] : nullptr);
            if (r < 0) { record(r, g_err); break; }
            if (hipMemcpyAsync(h_rgb[slot], d_rgb[slot], (size_t)rows[b] * tw * 3, hipMemcpyDeviceToHost, st[slot]) !=
                hipSuccess) { record(RT_E_HIP, "rt_render_multi: band copy"); break; }
            pending[slot] = b;
        }
        for (int k = 0; k < kSlots; ++k) drain(k);
        for (int k = 0; k < kSlots; ++k) {
            if (st[k]) (void)hipStreamSynchronize(st[k]);
            if (d_rgb[k]) (void)hipFree(d_rgb[k]);
            if (h_rgb[k]) (void)hipHostFree(h_rgb[k]);
            if (st[k]) (void)hipStreamDestroy(st[k]);
        }
    };
    std::vector<std::thread> pool;
    for (int32_t i = 0; i < n_devices; ++i) pool.emplace_back(worker, devices[i]);
    for (auto& t : pool) t.join();
    if (err_code.load() != RT_OK) return fail(err_code.load(), err_msg);
    if (stats) {
        std::memset(stats, 0, sizeof *stats);
        stats->samples = samples.load();
        stats->vertices = vertices.load();
        stats->device_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->kernel_launches[0] = nb;
    }
    // only a cancel leaves bands unrendered without an error; a band whose kernel saw the cancel word
    // stopped handing out subpixels early
    if (done.load() < nb || (cancel && *cancel)) return RT_CANCELLED;
    return RT_OK;
}

int rt_trace_rays(const rt_scene* scene, int32_t device, int64_t n, const double* origins, const double* dirs, double* t,
                  int32_t* object, double* pos, double* normal) {
    return rt_trace_rays_flags(scene, device, 0u, n, origins, dirs, t, object, pos, normal);
}

int rt_trace_rays_flags(const rt_scene* scene, int32_t device, uint32_t flags, int64_t n, const double* origins,
                        const double* dirs, double* t, int32_t* object, double* pos, double* normal) {
    if (!scene || n < 0 || (n && (!origins || !dirs || !t || !object))) return fail(RT_E_INVAL, "null argument");
    if (n == 0) return RT_OK;
    HIP_TRY(hipSetDevice(device));
    rt::DevScene ds;
    int rc = upload(const_cast<rt_scene*>(scene), device, &ds);
    if (rc != RT_OK) return rc;
    size_t v3 = (size_t)n * 3 * sizeof(double);
    char* buf = nullptr;
    size_t total = 4 * v3 + (size_t)n * sizeof(double) + (size_t)n * sizeof(int32_t);
    HIP_TRY(hipMalloc((void**)&buf, total));
    double* d_o = (double*)buf;
    double* d_d = (double*)(buf + v3);
    double* d_pos = (double*)(buf + 2 * v3);
    double* d_n = (double*)(buf + 3 * v3);
    double* d_t = (double*)(buf + 4 * v3);
    int32_t* d_id = (int32_t*)(buf + 4 * v3 + (size_t)n * sizeof(double));
    hipError_t e = hipMemcpy(d_o, origins, v3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, dirs, v3, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = rt::launch_trace_f64(ds, (long)n, d_o, d_d, d_t, d_id, d_pos, d_n, (flags & RT_FLAG_MESH_NEAREST) != 0, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(t, d_t, (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(object, d_id, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && pos) e = hipMemcpy(pos, d_pos, v3, hipMemcpyDeviceToHost);
    if (e == hipSuccess && normal) e = hipMemcpy(normal, d_n, v3, hipMemcpyDeviceToHost);
    (void)hipFree(buf);
    if (e != hipSuccess) return fail(RT_E_HIP, std::string("rt_trace_rays: ") + hipGetErrorString(e));
    return RT_OK;
}

}  // extern "C"
