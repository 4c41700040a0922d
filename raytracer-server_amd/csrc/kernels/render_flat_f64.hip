// Block-synchronous megakernel for scenes whose meshes are all flat octrees (DevMesh::flat: the
// cubes scene's two 12-triangle cubes, a root parent with 8 leaves).
//
// In the per-lane megakernels a mesh query (the octree walk of Mesh::intersect, geometry.rs:883-905,
// 1237-1295) is needed by ~6% of the lanes per trace, but almost every wave has one such lane, so
// every wave pays for the walk with 1-4 lanes active (lane utilisation 0.22 on the cubes). Here the
// 4 waves of a block advance their paths one vertex per iteration in three phases separated by two
// barriers:
//   A  camera / analytic closest hit (planes, spheres); a lane whose ray may reach a mesh queues a
//      closest-hit query per mesh in LDS;
//   P  every query the block queued is processed densely, one lane per query and one wave per chunk
//      of up to 64 queries of one mesh and kind: the closest-hit queries of this vertex and the
//      shadow queries of the previous one (so the 4 waves share up to 4 chunks); flat_query evaluates
//      the walk's result from every triangle of that mesh (scalar loads: a chunk's lanes query the
//      same mesh);
//   C  the previous vertex's shadow results: its NEE term is added unless a mesh blocks the shadow
//      ray (mutually_visible); this vertex: the mesh hits merged in Scene::trace_ray's order (ties to
//      the lower object index), shading, and a shadow ray the analytic objects let through queued per
//      mesh for the next P; sample / subpixel bookkeeping and tickets. A path that ends with a shadow
//      query pending waits one iteration (no new path in A) until C has its result.
// Every query returns the same bits as the per-lane walk (same tri_t, same box_hit per octant, same
// visiting order), so frames are identical to k_megakernel_f64's and the wavefront's (tested).
// Its own translation unit (code object): launched by launch_megakernel_f64 (render_f64.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "../device/integrator_f64.h"
#include "kernels.h"
#include "megakernel_common.h"

namespace rt {
using namespace f64;

namespace {

constexpr int kBlk = 256;
typedef __attribute__((address_space(3))) double LdsD;
typedef __attribute__((address_space(3))) uint64_t LdsU;

// The first of the candidate octants `cand` (non-zero) in the walk's visiting order: the root's
// octants sorted by (mag(centre - origin), index) (geometry.rs:1248-1260, a stable insertion sort;
// root_order). Only the minimum is needed, so no sort: the argmin of the radicands d2 (sqrt is
// monotone), unless a lower-index candidate's d2 lies within 2^-50 of the minimum, where the two
// square roots may round equal and the index decides (then the argmin of the roots themselves).
template <class MT>
RT_DEV int first_visited(const MT& m, const Ray& ray, uint32_t cand) {
    double d2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const V3 dv = ld3(m.oct_center[i]) - ray.o;
        d2[i] = dv.x * dv.x + dv.y * dv.y + dv.z * dv.z;  // mag()'s radicand, same order
    }
    int best = -1;
    double bk = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (((cand >> i) & 1u) && (best < 0 || d2[i] < bk)) {
            best = i;
            bk = d2[i];
        }
    }
    bool close = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) close |= ((cand >> i) & 1u) && i < best && !(d2[i] > bk * (1.0 + 0x1p-50));
    if (close) {  // rare: compare the roots (mag() itself), ties to the lower index
        best = -1;
        bk = 0.0;
        for (int i = 0; i < 8; ++i) {
            if ((cand >> i) & 1u) {
                const double k = sqrt(d2[i]);
                if (best < 0 || k < bk) {
                    best = i;
                    bk = k;
                }
            }
        }
    }
    return best;
}

// Mesh::intersect of a flat octree for the ray (geometry.rs:883-905, 1237-1295): the walk visits the
// root's children (leaves) in the ray's order (distances to the ROOT octant centres, root_order),
// takes the first one whose octant box the ray hits (box_hit) and that holds a triangle hit, and
// returns that leaf's nearest triangle (strict <: the first in leaf order, i.e. the lowest index).
// Evaluated here from every triangle's tri_t (the walk's own test, same bits) with the nearest hit
// kept per leaf; box tests and the order only for lanes with a hit. A root leaf is its nearest hit
// without any box test (geometry.rs:1237-1241). All lanes of the calling wave query mesh `m`.
// (The general form, for rays with 3 or more triangle hits: flat_query below.)
RT_DEV bool flat_query_leaves(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, double* t_out,
                              int* prim_out) {
    double bt[8];
    int bi[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        bt[l] = INFINITY;
        bi[l] = -1;
    }
    uint32_t hit_leaves = 0;
    const int n = m.n_tris;
    for (int j = 0; j < n; ++j) {
        double tt;
        if (tri_t(sc.tris[m.tri_base + j], ray, &tt)) {
            const uint32_t lm = (m.flat_leaf[j >> 2] >> (8 * (j & 3))) & 0xFFu;
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                if (((lm >> l) & 1u) && tt < bt[l]) {
                    bt[l] = tt;
                    bi[l] = j;
                }
            }
            hit_leaves |= lm;
        }
    }
    int win = -1;
    if (m.flat_root_leaf) {
        win = bi[0] >= 0 ? 0 : -1;
    } else if (__any(hit_leaves != 0)) {
        if (hit_leaves != 0) {
            uint32_t cand = hit_leaves & (uint32_t)m.flat_kids;
            cand &= octant_mask(m.root_box, m.root_box + 3, ray, inv);  // the children's box_hit, bit i = octant i
            if (cand) win = first_visited(m, ray, cand);
        }
    }
    if (win < 0) return false;
    double t = bt[0];
    int j = bi[0];
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        if (win == l) {
            t = bt[l];
            j = bi[l];
        }
    }
    *t_out = t;
    *prim_out = m.tri_base + j;
    return true;
}

// The mesh and triangle tables of a flat query through constant-address-space pointers: every lane
// of the wave queries the same mesh, so the triangle loop reads them with scalar loads into SGPRs
// (no vector-memory round trip per triangle, no VGPRs for the 96 B of each triangle).
typedef const __attribute__((address_space(4))) DevMesh CMesh;
typedef const __attribute__((address_space(4))) DevTri CTri;

// flat_query_leaves' result from the first two triangle hits of the ray (a ray crosses a convex
// mesh's surface twice; a third hit, e.g. on an edge two triangles share, takes flat_query_leaves):
// the winning leaf is found as there, from the union of the hit triangles' leaves, and its nearest
// hit is the first of the two hits that lies in it unless the second is strictly nearer (the leaf
// lists are in triangle order, so the earlier hit is the lower index: the walk's strict <). Same
// bits as flat_query_leaves, without its per-leaf best-hit updates (8 leaves x 4 VALU per triangle).
// The ray reciprocals are taken only for lanes whose ray hits a triangle (the leaf boxes' test).
#ifndef RT_FLAT_GRID_ORDER
#define RT_FLAT_GRID_ORDER 1  // the winning leaf by root_order_grid's order (1) or first_visited's argmin (0: A/B)
#endif
RT_DEV bool flat_query(const DevScene& sc, int mi, const Ray& ray, double* t_out, int* prim_out) {
    CMesh* M = (CMesh*)(uintptr_t)(sc.meshes + mi);
    const int n = M->n_tris, base = M->tri_base;
    CTri* T = (CTri*)(uintptr_t)(sc.tris + base);
    double ta = 0.0, tb = 0.0;
    int ja = -1, jb = -1, nh = 0;
    uint32_t la = 0, lb = 0, hit_leaves = 0;
    for (int j = 0; j < n; ++j) {
        double tt;
        if (tri_t(T[j], ray, &tt)) {
            const uint32_t lm = (M->flat_leaf[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            hit_leaves |= lm;
            if (nh == 0) {
                ta = tt;
                ja = j;
                la = lm;
            } else if (nh == 1) {
                tb = tt;
                jb = j;
                lb = lm;
            }
            ++nh;
        }
    }
    if (__any(nh > 2)) {
        if (nh > 2) return flat_query_leaves(sc, sc.meshes[mi], ray, make_inv(ray.d), t_out, prim_out);
    }
    int win = -1;
    if (M->flat_root_leaf) {
        win = nh > 0 ? 0 : -1;
    } else if (__any(hit_leaves != 0)) {
        if (hit_leaves != 0) {
            uint32_t cand = hit_leaves & (uint32_t)M->flat_kids;
            double rb[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) rb[k] = M->root_box[k];
            cand &= octant_mask(rb, rb + 3, ray, make_inv(ray.d));  // the children's box_hit, bit i = octant i
            if (cand) {
#if RT_FLAT_GRID_ORDER
                // the whole visiting order from the octant centres' grid (path_f64.h root_order_grid: root_order's
                // result whenever no two radicands are near a tie), its first candidate; else first_visited
                uint32_t order;
                if (wave_all(root_order_grid(*M, ray, &order))) {
#pragma unroll
                    for (int q = 7; q >= 0; --q) {
                        const uint32_t oi = (order >> (4 * q)) & 0xFu;
                        win = ((cand >> oi) & 1u) ? (int)oi : win;
                    }
                } else {
                    win = first_visited(*M, ray, cand);
                }
#else
                win = first_visited(*M, ray, cand);
#endif
            }
        }
    }
    if (win < 0) return false;
    const bool ina = ((la >> win) & 1u) != 0, inb = nh > 1 && ((lb >> win) & 1u) != 0;
    const bool use_b = inb && (!ina || tb < ta);
    *t_out = use_b ? tb : ta;
    *prim_out = base + (use_b ? jb : ja);
    return true;
}

// Appends this block's lane `tid` to queue q (wave-aggregated LDS atomic). All lanes of the wave call.
RT_DEV void enqueue(int32_t* cnt, int32_t* queue, bool want) {
    const unsigned long long mk = __ballot(want);
    if (mk == 0ull) return;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)mk) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(cnt, __popcll(mk));
    base = __shfl(base, leader, 64);
    if (want) {
        const unsigned long long below = lane ? (mk & ((~0ull) >> (64 - lane))) : 0ull;
        queue[base + __popcll(below)] = (int32_t)threadIdx.x;
    }
}

// Phase P: the block's queued queries in chunks of up to 64 entries of one mesh, handed to the waves
// in turn (starting at wave `first`). A mesh's entries are its closest-hit queries (ray in qc;
// results t / prim to rt / rp [mesh][lane]) followed by its shadow queries (ray + |y - x| in qs;
// result occluded to ro [mesh][lane], mutually_visible: the walk's hit t with t + 0.001 < |y - x|):
// flat_query is the same for both, so one chunk serves both kinds.
#ifndef RT_FLAT_MERGE_KINDS
#define RT_FLAT_MERGE_KINDS 1
#endif
RT_DEV void process_queries(const DevScene& sc, const int32_t* cnt_c, const int32_t* queue_c, const int32_t* cnt_s,
                            const int32_t* queue_s, const LdsD* qc, const LdsD* qs, double* rt, int32_t* rp,
                            int32_t* ro, int first) {
    const int wv = threadIdx.x >> 6, ln = __lane_id();
    int ci = first;
#if RT_FLAT_MERGE_KINDS
    for (int m = 0; m < sc.n_meshes; ++m) {
        const int nc = cnt_c[m], c = nc + cnt_s[m];
        for (int k = 0; k * 64 < c; ++k, ++ci) {
            if ((ci & 3) != wv) continue;
            const int e = k * 64 + ln;
            RT_DBG_WAVE(13, lane_id_is0());
            RT_DBG_WAVE(12, e < c);
            if (e < c) {
                const int kind = e >= nc;
                const int who = kind ? queue_s[m * kBlk + e - nc] : queue_c[m * kBlk + e];
                const LdsD* q = kind ? qs : qc;
                const Ray r{v3(q[who], q[kBlk + who], q[2 * kBlk + who]),
                            v3(q[3 * kBlk + who], q[4 * kBlk + who], q[5 * kBlk + who])};
                double t = 0.0;
                int prim = -1;
                const bool hit = flat_query(sc, m, r, &t, &prim);
                if (kind == 0) {
                    rt[m * kBlk + who] = t;
                    rp[m * kBlk + who] = hit ? prim : -1;
                } else {
                    ro[m * kBlk + who] = hit && !(t + 0.001 >= q[6 * kBlk + who]) ? 1 : 0;
                }
            }
        }
    }
#else
    for (int kind = 0; kind < 2; ++kind) {
        const int32_t* cnt = kind ? cnt_s : cnt_c;
        const int32_t* queue = kind ? queue_s : queue_c;
        const LdsD* q = kind ? qs : qc;
        for (int m = 0; m < sc.n_meshes; ++m) {
            const int c = cnt[m];
            for (int k = 0; k * 64 < c; ++k, ++ci) {
                if ((ci & 3) != wv) continue;
                const int e = k * 64 + ln;
                RT_DBG_WAVE(13, lane_id_is0());
                RT_DBG_WAVE(12, e < c);
                if (e < c) {
                    const int who = queue[m * kBlk + e];
                    const Ray r{v3(q[who], q[kBlk + who], q[2 * kBlk + who]),
                                v3(q[3 * kBlk + who], q[4 * kBlk + who], q[5 * kBlk + who])};
                    double t = 0.0;
                    int prim = -1;
                    const bool hit = flat_query(sc, m, r, &t, &prim);
                    if (kind == 0) {
                        rt[m * kBlk + who] = t;
                        rp[m * kBlk + who] = hit ? prim : -1;
                    } else {
                        ro[m * kBlk + who] = hit && !(t + 0.001 >= q[6 * kBlk + who]) ? 1 : 0;
                    }
                }
            }
        }
    }
#endif
}

}  // namespace

template <int F, int W>
__global__ __launch_bounds__(kBlk, W) void k_megakernel_flat_f64(DevScene sc_g, RenderArgs a_g, double* __restrict__ sub_buf,
                                                                uint32_t* next_sub, long nsub) {
    using C = Cfg<F | kCfgLdsObj>;  // the object table in LDS (path_f64.h rt_lds_objects)
    static_assert(C::mesh && C::compact && !C::bvh, "flat-mesh kernel: compact scenes, octree meshes");
#if RT_KARG_VIEW
    const DevScene& sc = karg_scene();  // the arguments read in place (megakernel_common.h)
    const RenderArgs& a = karg_render_args();
#else
    const DevScene& sc = sc_g;
    const RenderArgs& a = a_g;
#endif
    lds_objects_fill(sc);
    // per lane (one column per thread): subpixel accumulator; the closest-hit query ray (o, d), the
    // shadow query ray (o, d, |y - x|); results per (mesh, lane); queues per (kind, parity, mesh):
    // the closest queries of iteration i and the shadow queries of i - 1 are in flight together
    __shared__ double s_acc[3 * kBlk];
    __shared__ double s_qc[6 * kBlk], s_qs[7 * kBlk];
    __shared__ double s_rt[kFlatMeshes * kBlk];
    __shared__ int32_t s_rp[kFlatMeshes * kBlk], s_ro[kFlatMeshes * kBlk];
    __shared__ int32_t s_queue[2][2][kFlatMeshes * kBlk];  // [kind][parity]
    __shared__ int32_t s_cnt[2][2][kFlatMeshes];
    __shared__ int32_t s_active;
    LdsD* acc_l = (LdsD*)s_acc + threadIdx.x;
    const int tid = threadIdx.x;
    if (tid < 4 * kFlatMeshes) (&s_cnt[0][0][0])[tid] = 0;
    if (tid == 0) s_active = 0;
    RT_DBG_TINIT();
    __syncthreads();

    uint32_t nverts = 0;
    const long n_split = nsub - a.n_whole;
    const long nunits = a.n_wunits + n_split * a.tail_cps;
    int id, end, s;
    const long t0 = wave_ticket(next_sub, true);
    unit_of(a, t0, id, end, s);
    bool active = t0 < nunits;
    {
        const unsigned long long m = __ballot(active);
        if (__lane_id() == 0 && m) atomicAdd(&s_active, __popcll(m));
    }
    acc_l[0] = 0.0; acc_l[kBlk] = 0.0; acc_l[2 * kBlk] = 0.0;
    PathState ps;
    bool fresh = true;
    bool pend = false;     // a shadow query of the last vertex is in flight
    bool waiting = false;  // the last vertex ended the sample; it is finished once its shadow result is in
    V3 pc = v3(0, 0, 0);   // that query's NEE term, added unless a mesh blocks the shadow ray
    uint32_t smask = 0;    // meshes the shadow query was queued for
    __syncthreads();
    for (int it = 0;; ++it) {
        const int par = it & 1;
        RT_DBG_WAVE(8, lane_id_is0());
        RT_DBG_WAVE(9, active);
        RT_DBG_TSTART(t_a);
        // ---------------- A: camera, analytic closest hit, closest-hit queries
        const bool go = active && !waiting;
        if (go && fresh) {
            begin_sample(sc, a, subpixel_of(a, id), s, ps);
            fresh = false;
        }
        HitRec h{0.0, -1, -1};
        RayInv inv{};
        double tmax = INFINITY;
        if (go) {
            inv = make_inv(ps.ray.d);
            h = trace_analytic<C>(sc, ps.ray, inv);
            tmax = h.obj >= 0 ? h.t : INFINITY;
            s_qc[tid] = ps.ray.o.x; s_qc[kBlk + tid] = ps.ray.o.y; s_qc[2 * kBlk + tid] = ps.ray.o.z;
            s_qc[3 * kBlk + tid] = ps.ray.d.x; s_qc[4 * kBlk + tid] = ps.ray.d.y; s_qc[5 * kBlk + tid] = ps.ray.d.z;
        }
        uint32_t qmask = 0;
        for (int m = 0; m < sc.n_meshes; ++m) {
            const DevMesh& M = sc.meshes[m];
            const bool want = go && near_box(M.cull_box, ps.ray, inv, M.cull_pad, tmax);
            qmask |= want ? (1u << m) : 0u;
            enqueue(&s_cnt[0][par][m], s_queue[0][par] + m * kBlk, want);
        }
        RT_DBG_TEND(1, t_a);
        RT_DBG_TSTART(t_w1);
        __syncthreads();
        RT_DBG_TEND(6, t_w1);
        if (s_active == 0) break;  // every lane of the block is done (stable between C and the next A)
        // ---------------- P: this vertex's closest-hit queries, the previous vertex's shadow queries
        RT_DBG_TSTART(t_p);
        process_queries(sc, s_cnt[0][par], s_queue[0][par], s_cnt[1][par ^ 1], s_queue[1][par ^ 1], (const LdsD*)s_qc,
                        (const LdsD*)s_qs, s_rt, s_rp, s_ro, it & 3);
        RT_DBG_TEND(2, t_p);
        RT_DBG_TSTART(t_w2);
        __syncthreads();
        RT_DBG_TEND(6, t_w2);
        RT_DBG_TSTART(t_c);
        // ---------------- C: shadow results, merge + shade, shadow queries, bookkeeping
        if (tid < kFlatMeshes) s_cnt[0][par][tid] = 0;            // next appended in A of iteration it + 2
        else if (tid < 2 * kFlatMeshes) s_cnt[1][par ^ 1][tid - kFlatMeshes] = 0;  // in C of it + 1
        bool finish = false;  // the sample of this lane's path is complete
        if (pend) {
            bool occluded = false;
            for (int m = 0; m < sc.n_meshes; ++m)
                if ((smask >> m) & 1u) occluded |= s_ro[m * kBlk + tid] != 0;
            if (!occluded) ps.L = ps.L + pc;
            pend = false;
            if (waiting) {
                waiting = false;
                finish = true;
            }
        }
        smask = 0;
        bool want_s = false;
        Ray sr{v3(0, 0, 0), v3(0, 0, 1)};
        RayInv sinv{};
        double dist = 0.0;
        if (go) {
            CTab* T = tables(sc);
            for (int g = 0; g < T->n_gen; ++g) {  // Scene::trace_ray's loop over the meshes (ties: lower index)
                const int mm = T->gen_mesh[g];   // the slot's mesh (CompactTab; -1: not a mesh, or empty)
                if (mm >= 0 && ((qmask >> mm) & 1u)) {
                    const int p = s_rp[mm * kBlk + tid];
                    if (p >= 0) consider(h, s_rt[mm * kBlk + tid], T->gen_idx[g], p);
                }
            }
            nverts += h.obj >= 0;
            ShadowDefer df;
            df.pending = false;
            const bool cont = shade_vertex<C>(sc, a, ps, h, &df);
            if (df.pending) {  // the analytic objects let the shadow ray through; a mesh may block it
                pend = true;
                pc = df.c;
                dist = df.dist;
                sr = Ray{df.o, df.d};
                sinv = make_inv(sr.d);
                s_qs[tid] = sr.o.x; s_qs[kBlk + tid] = sr.o.y; s_qs[2 * kBlk + tid] = sr.o.z;
                s_qs[3 * kBlk + tid] = sr.d.x; s_qs[4 * kBlk + tid] = sr.d.y; s_qs[5 * kBlk + tid] = sr.d.z;
                s_qs[6 * kBlk + tid] = dist;
            }
            if (!cont) {
                if (pend) waiting = true;  // finished in the next C
                else finish = true;
            }
        }
        for (int m = 0; m < sc.n_meshes; ++m) {
            const DevMesh& M = sc.meshes[m];
            const bool want = pend && go && near_box(M.cull_box, sr, sinv, M.cull_pad, dist);
            smask |= want ? (1u << m) : 0u;
            enqueue(&s_cnt[1][par][m], s_queue[1][par] + m * kBlk, want);
            want_s |= want;
        }
        if (go && pend && !want_s) {  // no mesh near the shadow segment: unblocked now
            ps.L = ps.L + pc;
            pend = false;
            if (waiting) {
                waiting = false;
                finish = true;
            }
        }
        bool done = false;
        if (finish) {
            fresh = true;
            if (id < a.n_whole) {
                V3 acc = v3(acc_l[0], acc_l[kBlk], acc_l[2 * kBlk]);
                acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                acc_l[0] = acc.x; acc_l[kBlk] = acc.y; acc_l[2 * kBlk] = acc.z;
                if (++s == a.n_samples) {
                    double* o = sub_buf + (size_t)id * 3;
                    o[0] = acc.x;
                    o[1] = acc.y;
                    o[2] = acc.z;
                    if (++id < end) {  // the next subpixel of the run, no ticket
                        s = 0;
                        acc_l[0] = 0.0; acc_l[kBlk] = 0.0; acc_l[2 * kBlk] = 0.0;
                    } else {
                        done = true;
                    }
                }
            } else if (tail_in_place(a, s)) {  // split tail, chunk 0: summed in place, its partial sum to sub_buf
                V3 acc = v3(acc_l[0], acc_l[kBlk], acc_l[2 * kBlk]);
                acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                acc_l[0] = acc.x; acc_l[kBlk] = acc.y; acc_l[2 * kBlk] = acc.z;
                done = !unit_has_next(a, id, s);
                if (done) {
                    double* o = sub_buf + (size_t)id * 3;
                    o[0] = acc.x;
                    o[1] = acc.y;
                    o[2] = acc.z;
                }
                ++s;
            } else {  // split tail, later chunks: each sample's radiance, summed in order by k_tail_sum_f64
                tail_store(a, id, s, ps.L);
                done = !unit_has_next(a, id, s);
                ++s;
            }
        }
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        flush_count_if_full(a.counters, nverts, done);
        bool ended = false;
        if (done) {
            unit_of(a, nt, id, end, s);
            active = !stop && nt < nunits;
            ended = !active;
            acc_l[0] = 0.0; acc_l[kBlk] = 0.0; acc_l[2 * kBlk] = 0.0;
            fresh = true;
        }
        {
            const unsigned long long m = __ballot(ended);
            if (__lane_id() == 0 && m) atomicSub(&s_active, __popcll(m));
        }
        RT_DBG_TEND(3, t_c);
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

// Query-pool variant (RT_MK_FPOOL, default): the same per-vertex work as k_megakernel_flat_f64 but
// without barriers. Each wave loops on its own: (1) for each mesh, if at least `pool_min` queries of
// that mesh are queued in the block's LDS queue (or < 16 of the wave's paths are ready), it takes up to 64 of
// them (any wave's, closest-hit and shadow mixed) and evaluates them with flat_query, one lane per
// query; (2) each of its paths whose queries are all answered (s_pend = 0) adds the previous shadow
// result, merges the mesh hits, shades, queues the shadow queries, and traces its next ray, queueing
// that ray's closest-hit queries. A path thus waits only for its own queries, queries are evaluated
// in fuller chunks, and no wave waits at a barrier for another wave's chunk (the block-synchronous
// kernel spent 24% of its wave time in barrier waits, 2 waves of 4 working in phase P).
#ifndef RT_FPOOL_BLOCK
#define RT_FPOOL_BLOCK 1024  // threads per query-pool block of the no-mirror instance: one block per CU (16 waves,
                             // 4 per SIMD, share one query queue per mesh; 128 VGPRs, 36 spilled): cubes +9.8% over
                             // 768 (3 waves/SIMD, profiles/r05w_ab_fp.log), which the running sums in sub_buf and
                             // the 16-bit rings made fit the LDS; or 256 (three blocks per CU, A/B)
#endif
#ifndef RT_FPOOL_PRIO
#define RT_FPOOL_PRIO 1  // the query chunks (stage 1) at raised issue priority (s_setprio 1: cubes +1.3%, r04ao), or not (0)
#endif
#ifndef RT_FPOOL_READY
#define RT_FPOOL_READY 16  // a wave with at least this many ready paths waits for chunks of pool_min queries
#endif
#ifndef RT_FPOOL_SINK
#define RT_FPOOL_SINK 1  // A/B: shade_vertex writes the shadow query's ray into the LDS columns (LdsQuerySink)
#endif

template <int F, int W, int B = kBlk>
__global__ __launch_bounds__(B, W) void k_megakernel_fpool_f64(DevScene sc_g, RenderArgs a_g, double* __restrict__ sub_buf,
                                                                 uint32_t* next_sub, long nsub, int pool_min, int refill) {
    using C = Cfg<F | kCfgLdsObj>;  // the object table in LDS (path_f64.h rt_lds_objects)
    static_assert(C::mesh && C::compact && !C::bvh, "flat-mesh kernel: compact scenes, octree meshes");
    static_assert(B % 64 == 0 && B <= 1024, "whole waves (path_f64.h: the diagnostic builds' per-wave LDS)");
    static_assert(C::nospec || B == 256, "LdsCold's columns have a stride of 256");
    // per mesh: at most B closest-hit + B shadow queries queued at once (a power of two)
    constexpr int kRing = B <= 256 ? 512 : B <= 512 ? 1024 : 2048;
#if RT_KARG_VIEW
    const DevScene& sc = karg_scene();  // the arguments read in place (megakernel_common.h)
    const RenderArgs& a = karg_render_args();
#else
    const DevScene& sc = sc_g;
    const RenderArgs& a = a_g;
#endif
    lds_objects_fill(sc);
    // per lane (one column per thread): the closest-hit query ray (o, d), the
    // shadow query ray (o, d, |y - x|); results per (mesh, lane); queries outstanding per lane
    // The closest-hit and the shadow query of a lane are issued in the same iteration from the same
    // point (the shadow ray's x and the next ray's origin, integrator_f64.h shade_vertex; a camera ray
    // never coexists with a shadow query: the path waits for it, `endwait`), so they share one origin
    // column: s_qo origin, s_qdc closest direction, s_qds shadow direction + |y - x|. Closest results:
    // t, and the hit triangle as its index within the mesh (flat meshes hold <= kFlatMaxTris). The
    // mirror-bounce state (o, pre-bounce throughput) lives in LDS as in k_megakernel_f64 (LdsCold):
    // 12 VGPRs less at 3 waves/SIMD.
    // Scenes without a mirror object (Cfg::nospec) have no mirror-bounce state: its 12 KB hold a
    // camera-sample buffer instead (as k_megakernel_f64's: the next sample's camera ray and RNG state,
    // computed for many lanes at once in a refill pass rather than by a few lanes per iteration).
    // Every per-lane 8-byte column lives in one array (RT_FPOOL_COLS): a lane's column addresses are then
    // one base plus immediate offsets, instead of a base per array, which the register allocator of the
    // 4-waves/SIMD instance (128 VGPRs) spilled to scratch and reloaded at each use.
    constexpr int kColQo = 0, kColQdc = 3, kColQds = 6, kColRt = 10, kColX = kColRt + kFlatMeshes;
    constexpr int kCols = kColX + (C::nospec ? 5 : 6);  // + camera sample (d, RNG) / mirror state (o, beta)
    __shared__ double s_cols[kCols * B];
    double* const s_qo = s_cols + kColQo * B;
    double* const s_qdc = s_cols + kColQdc * B;
    double* const s_qds = s_cols + kColQds * B;
    double* const s_rt = s_cols + kColRt * B;
    __shared__ uint8_t s_rp[kFlatMeshes * B];
    __shared__ uint8_t s_ro[kFlatMeshes * B];
    double* const s_cold = s_cols + kColX * B;  // !nospec: LdsCold's 6 columns (stride 256: B == 256)
    using Cold = std::conditional_t<C::nospec, RegCold, LdsCold>;
    Cold cold{};
    if constexpr (!C::nospec) cold = LdsCold{(LdsD*)s_cold + threadIdx.x};
    double* const s_nbd = s_cols + kColX * B;
    uint64_t* const s_nbr = (uint64_t*)(s_cols + (kColX + 3) * B);
    LdsD* nbd = (LdsD*)s_nbd + (C::nospec ? threadIdx.x : 0);
    __attribute__((address_space(3))) uint64_t* nbr = (__attribute__((address_space(3))) uint64_t*)s_nbr + (C::nospec ? threadIdx.x : 0);
    bool nvalid = false;  // nbd / nbr hold sample s + 1 of subpixel id
    __shared__ int32_t s_pend[B];
    // per mesh: queued queries, entry = lane (closest hit) or 256 + lane (shadow)
    __shared__ int16_t s_ring[kFlatMeshes][kRing];  // entries < 2 B <= 2048
    __shared__ uint32_t s_head[kFlatMeshes], s_tail[kFlatMeshes];
    const int tid = threadIdx.x;
    for (int i = tid; i < kFlatMeshes * kRing; i += B) (&s_ring[0][0])[i] = -1;
    if (tid < kFlatMeshes) {
        s_head[tid] = 0;
        s_tail[tid] = 0;
    }
    s_pend[tid] = 0;
    RT_DBG_TINIT();
    __syncthreads();
    const int nm = sc.n_meshes;

    uint32_t nverts = 0;
    const long n_split = nsub - a.n_whole;
    const long nunits = a.n_wunits + n_split * a.tail_cps;
    int id, end, s;
    const long t0 = wave_ticket(next_sub, true);
    unit_of(a, t0, id, end, s);
    bool active = t0 < nunits;
    PathState ps;
    bool fresh = true;
    bool traced = false;   // ps.ray has been traced: h is its analytic hit, qmask its closest-hit queries
    bool spend = false;    // a shadow query set of the last vertex is in flight (its NEE term in pc)
    bool endwait = false;  // the path has ended; the sample is finished once the shadow result is in
    HitRec h{0.0, -1, -1};
    uint32_t qmask = 0, smask = 0;
    V3 pc = v3(0, 0, 0);
    while (__any(active)) {
        RT_DBG_WAVE(8, lane_id_is0());
        RT_DBG_TSTART(t_q);
        // ---------------- (1) queued mesh queries, a chunk per mesh
#if RT_FPOOL_PRIO
        __builtin_amdgcn_s_setprio(RT_FPOOL_PRIO);  // A/B: the query chunks at raised issue priority (this level)
#endif
        {
            const bool rdy = active && __hip_atomic_load(&s_pend[tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
            // full chunks while this wave has paths to go on with; anything queued once most of its
            // paths wait (also the frame's end: no query waits for a quorum that never comes)
            const int need = __popcll(__ballot(rdy)) >= RT_FPOOL_READY ? pool_min : 1;
            for (int m = 0; m < nm; ++m) {
                const LdsQueue16 Q{s_ring[m], &s_head[m], &s_tail[m], (uint32_t)kRing - 1u};
                const int32_t e = queue_take(Q, need);
                if (!__any(e >= 0)) continue;
                RT_DBG_WAVE(13, lane_id_is0());
                RT_DBG_WAVE(12, e >= 0);
                if (e >= 0) {
                    const int kind = e >= B, who = kind ? e - B : e;  // entry = lane, or B + lane (shadow)
                    const LdsD* qo = (const LdsD*)s_qo;
                    const LdsD* q = kind ? (const LdsD*)s_qds : (const LdsD*)s_qdc;
                    const Ray r{v3(qo[who], qo[B + who], qo[2 * B + who]),
                                v3(q[who], q[B + who], q[2 * B + who])};
                    double t = 0.0;
                    int prim = -1;
                    const bool hit = flat_query(sc, m, r, &t, &prim);
                    RT_DBG(0);           // diagnostic builds: queries evaluated ...
                    if (hit) RT_DBG(1);  // ... and those with a triangle hit
                    if (kind == 0) {
                        s_rt[m * B + who] = t;
                        s_rp[m * B + who] = hit ? (uint8_t)(prim - sc.meshes[m].tri_base) : (uint8_t)0xFF;
                    } else {
                        s_ro[m * B + who] = hit && !(t + 0.001 >= q[3 * B + who]) ? 1 : 0;
                    }
                    const int32_t left = __hip_atomic_fetch_sub(&s_pend[who], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (RT_QCHECK && left <= 0) RT_QFAIL(2);
                }
            }
        }
#if RT_FPOOL_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        RT_DBG_TEND(1, t_q);
        RT_DBG_TSTART(t_v);
        // ---------------- (2) paths whose queries are all answered
        const bool ready = active && __hip_atomic_load(&s_pend[tid], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
        RT_DBG_WAVE(9, ready);
        bool finish = false, shadow_q = false;
#if !RT_FPOOL_SINK
        Ray sr{v3(0, 0, 0), v3(0, 0, 1)};
        double dist = 0.0;
#endif
        uint32_t near_s = 0;
        if (ready) {
            if (spend) {  // the last vertex's NEE term, unless a mesh blocks its shadow ray (mutually_visible)
                bool occluded = false;
                for (int m = 0; m < nm; ++m)
                    if ((smask >> m) & 1u) occluded |= s_ro[m * B + tid] != 0;
                if (!occluded) ps.L = ps.L + pc;
                spend = false;
            }
            if (endwait) {
                endwait = false;
                finish = true;
            } else if (traced) {
                CTab* T = tables(sc);
                for (int g = 0; g < T->n_gen; ++g) {  // Scene::trace_ray's loop over the meshes (ties: lower index)
                    // the slot's mesh from the compact table (-1: not a mesh, or an empty one, which has no hit)
                    const int mm = T->gen_mesh[g];
                    if (mm >= 0 && ((qmask >> mm) & 1u)) {
                        const int p = s_rp[mm * B + tid];
                        if (p != 0xFF) consider(h, s_rt[mm * B + tid], T->gen_idx[g], sc.meshes[mm].tri_base + p);
                    }
                }
                nverts += h.obj >= 0;
                ShadowDefer df;
                df.pending = false;
                df.c = v3(0.0, 0.0, 0.0);
#if RT_FPOOL_SINK
                // the shadow query's ray goes straight into this lane's query columns (its s_pend read 0)
                const LdsQuerySink qsink{(LdsD*)s_qo + tid, (LdsD*)s_qds + tid, B};
                const bool cont = shade_vertex<C, Cold, LdsQuerySink>(sc, a, ps, h, &df, cold, qsink);
#else
                const bool cont = shade_vertex<C, Cold>(sc, a, ps, h, &df, cold);
#endif
                traced = false;
                // pc is read only after a shadow query set it (spend): taking df.c unconditionally makes the old
                // value dead through shade_vertex, the kernel's register peak (the 1024-thread instance: 29 -> 21
                // spilled VGPRs, 76 -> 48 B of scratch per lane; cubes 1920x1080x256 1042.1 -> 1067.1 Msamples/s,
                // profiles/r06b_ab_pcdead.log)
                pc = df.c;
                if (df.pending) {  // the analytic objects let the shadow ray through; a mesh may block it
                    shadow_q = true;
#if !RT_FPOOL_SINK
                    dist = df.dist;
                    sr = Ray{df.o, df.d};
#endif
                    near_s = df.meshes;
                }
                if (!cont) {
                    if (shadow_q) endwait = true;
                    else finish = true;
                }
            }
        }
        RT_DBG_TEND(2, t_v);
        RT_DBG_TSTART(t_b);
        // shadow queries of this vertex, per mesh near the segment
        uint32_t want_s = 0;
        if (shadow_q) {
            want_s = near_s;  // shade_vertex's mesh_near_mask of the segment (non-zero: df.pending)
            if (want_s) {
#if !RT_FPOOL_SINK
                s_qo[tid] = sr.o.x; s_qo[B + tid] = sr.o.y; s_qo[2 * B + tid] = sr.o.z;
                s_qds[tid] = sr.d.x; s_qds[B + tid] = sr.d.y; s_qds[2 * B + tid] = sr.d.z;
                s_qds[3 * B + tid] = dist;
#endif
                spend = true;
                smask = want_s;
            } else {  // no mesh near the shadow segment: unblocked now
                ps.L = ps.L + pc;
                if (endwait) {
                    endwait = false;
                    finish = true;
                }
            }
        }
        // sample / subpixel bookkeeping, tickets
        bool done = false;
        if (finish) {
            fresh = true;
            if (id < a.n_whole || tail_in_place(a, s)) {
                // a whole subpixel, or the split tail's chunk 0: the running sum acc + L * inv_n from 0
                // (server.rs:357-358) kept in the subpixel's sub_buf entry (read back: the same bits), which
                // frees the LDS column it took
                double* o = sub_buf + (size_t)id * 3;
                V3 acc = v3(0.0, 0.0, 0.0);
                if (s != 0) acc = v3(o[0], o[1], o[2]);
                acc = acc + ps.L * a.inv_n;
                o[0] = acc.x;
                o[1] = acc.y;
                o[2] = acc.z;
                if (id < a.n_whole) {
                    if (++s == a.n_samples) {
                        if (++id < end) {  // the next subpixel of the run, no ticket
                            s = 0;
                            nvalid = false;
                        } else {
                            done = true;
                        }
                    }
                } else {
                    done = !unit_has_next(a, id, s);
                    ++s;
                }
            } else {  // split tail, later chunks: each sample's radiance, summed in order by k_tail_sum_f64
                tail_store(a, id, s, ps.L);
                done = !unit_has_next(a, id, s);
                ++s;
            }
        }
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        flush_count_if_full(a.counters, nverts, done);
        if (done) {
            unit_of(a, nt, id, end, s);
            active = !stop && nt < nunits;
            fresh = true;
            nvalid = false;
        }
        // camera-sample refill pass (no-mirror scenes): lanes with a sample in progress and a next
        // sample in the same unit, once at least `refill` of the wave's lanes need one
        if constexpr (C::nospec) {
            const bool need = active && !fresh && !nvalid && unit_has_next(a, id, s);
            if (refill > 0 && __popcll(__ballot(need)) >= refill) {
                if (need) {
                    const CameraSample nb = camera_sample(sc, a, subpixel_of(a, id), s + 1);
                    nbd[0] = nb.d.x; nbd[B] = nb.d.y; nbd[2 * B] = nb.d.z;
                    nbr[0] = nb.r0; nbr[B] = nb.r1;
                    nvalid = true;
                }
            }
        }
        // ---------------- the next ray (the path goes on, or a new sample), its closest-hit queries
        const bool tr = ready && active && !endwait && !traced;
        uint32_t want_c = 0;
        if (tr) {
            if (fresh) {
                if (C::nospec && nvalid) begin_path(sc, CameraSample{v3(nbd[0], nbd[B], nbd[2 * B]), nbr[0], nbr[B]}, ps);
                else begin_sample(sc, a, subpixel_of(a, id), s, ps);
                nvalid = false;
                fresh = false;
            }
            const RayInv inv = make_inv(ps.ray.d);
            h = trace_analytic<C>(sc, ps.ray, inv);
            const double tmax = h.obj >= 0 ? h.t : INFINITY;
            for (int m = 0; m < nm; ++m) {
                const DevMesh& M = sc.meshes[m];
#if RT_NEAR32
                if (near_mesh32(M, ps.ray, tmax)) want_c |= 1u << m;
#else
                if (near_box(M.cull_box, ps.ray, inv, M.cull_pad, tmax)) want_c |= 1u << m;
#endif
            }
            if (want_c) {
                s_qo[tid] = ps.ray.o.x; s_qo[B + tid] = ps.ray.o.y; s_qo[2 * B + tid] = ps.ray.o.z;
                s_qdc[tid] = ps.ray.d.x; s_qdc[B + tid] = ps.ray.d.y; s_qdc[2 * B + tid] = ps.ray.d.z;
            }
            qmask = want_c;
            traced = true;
        }
        // queue this lane's new queries (its s_pend is 0 until they are queued: nobody else writes it)
        if (RT_QCHECK && (want_s | want_c) && __hip_atomic_load(&s_pend[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0)
            RT_QFAIL(3);
        if (want_s | want_c) s_pend[tid] = __popc(want_s) + __popc(want_c);
        for (int m = 0; m < nm; ++m) {
            const LdsQueue16 Q{s_ring[m], &s_head[m], &s_tail[m], (uint32_t)kRing - 1u};
            queue_put(Q, (want_s >> m) & 1u, B + tid);
            queue_put(Q, (want_c >> m) & 1u, tid);
        }
        RT_DBG_TEND(3, t_b);
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

template <int F, int W, int B = kBlk>
static void launch_fpool(const DevScene& sc, RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                         double* tail_buf, size_t tail_cap, int pool_min, int refill, hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_fpool_f64<F, W, B>, (nsub + B - 1) / B, B);
    plan_tail(a, nsub, blocks * B, tail_buf, tail_cap, tail_split_x2(nsub, blocks * B));
    hipLaunchKernelGGL((k_megakernel_fpool_f64<F, W, B>), dim3((unsigned)blocks), dim3(B), 0, st, sc, a, sub_buf,
                       next_sub, nsub, pool_min, refill);
}

template <int F, int W>
static void launch_flat(const DevScene& sc, RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                        double* tail_buf, size_t tail_cap, hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_flat_f64<F, W>, (nsub + kBlk - 1) / kBlk);
    plan_tail(a, nsub, blocks * kBlk, tail_buf, tail_cap);
    hipLaunchKernelGGL((k_megakernel_flat_f64<F, W>), dim3((unsigned)blocks), dim3(kBlk), 0, st, sc, a, sub_buf,
                       next_sub, nsub);
}

// The flat-mesh megakernel (scenes whose meshes are all DevMesh::flat; octree mode).
// RT_MK_FLAT_WAVES: waves/SIMD requested from the register allocator (2 or 3).
hipError_t launch_megakernel_flat_f64(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub,
                                      double* tail_buf, size_t tail_cap, int refill, hipStream_t st) {
    const long nsub = (long)a_in.tw * a_in.th * 4;
    RenderArgs a = a_in;
    static const int waves = env_int("RT_MK_FLAT_WAVES", 3);
    static const int fpool = env_int("RT_MK_FPOOL", 1);
    // query chunks of pool_min (see RT_FPOOL_READY): 56 on the cubes 1024 spp 1093.3 Msamples/s (48: 1085.6, 64: 1087.6,
    // 80: 1061.0, 96: 1037.1; MIS 1027.5 -> 1034.2 at 56; profiles/r06ar_ab_fpool_min.log, r06as_ab_fpool_min.log)
    static const int pool_min = env_int("RT_MK_FPOOL_MIN", 56);
    static const int nospec = env_int("RT_MK_NOSPEC", 1);  // A/B: 0 = the mirror-capable kernel for every scene
    // camera-sample refill threshold of the query-pool kernel (no-mirror scenes): 16-24 lanes measured
    // best on the cubes (8: 736.9, 16: 747.2, 24: 745.2, 32: 737.3, 40: 730.9 Msamples/s; the analytic
    // kernel's `refill` is 40)
    static const int fpool_refill = env_int("RT_MK_FPOOL_REFILL", 20);
    (void)refill;
    // Product builds: the query pool at 3 waves/SIMD. The block-synchronous flat kernel (RT_MK_FPOOL=0) and the
    // 2-wave shapes exist only in A/B builds (ab_knobs.h).
#if RT_AB_KNOBS
#define RT_FLAT_CASE(F)                                                                       \
    case F:                                                                                   \
        if (fpool) {                                                                          \
            if (waves == 2) launch_fpool<F, 2>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, pool_min, fpool_refill, st); \
            else launch_fpool<F, 3>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, pool_min, fpool_refill, st); \
        } else if (waves == 2) launch_flat<F, 2>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, st); \
        else launch_flat<F, 3>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, st); \
        break;
#else
#define RT_FLAT_CASE(F)                                                                       \
    case F:                                                                                   \
        (void)waves;                                                                          \
        launch_fpool<F, 3>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, pool_min, fpool_refill, st); \
        break;
#endif
    if (fpool && nospec && (a.features & 32) && !(a.features & 2)) {  // no mirror, no Phong object
        switch (a.features & 15) {
            case 9: launch_fpool<9 | 32, RT_FPOOL_BLOCK / 256, RT_FPOOL_BLOCK>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, pool_min, fpool_refill, st); break;
            case 13: launch_fpool<13 | 32, RT_FPOOL_BLOCK / 256, RT_FPOOL_BLOCK>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, pool_min, fpool_refill, st); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (a.features & 15) {
            RT_FLAT_CASE(9) RT_FLAT_CASE(11) RT_FLAT_CASE(13) RT_FLAT_CASE(15)
            default: return hipErrorInvalidValue;
        }
    }
#undef RT_FLAT_CASE
    launch_tail_sum_f64(a, sub_buf, nsub - a.n_whole, st);
    return hipGetLastError();
}

#define RT_DIAG_TU_FN diag_read_flat
#include "diag_tu.h"

}  // namespace rt
