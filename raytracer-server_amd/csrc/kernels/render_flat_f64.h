// Block-synchronous megakernel for scenes whose meshes are all flat octrees (DevMesh::flat: the
// cubes scene's two 12-triangle cubes, a root parent with 8 leaves).
//
// In the per-lane megakernels a mesh query (the octree walk of Mesh::intersect, geometry.rs:883-905,
// 1237-1295) is needed by ~6% of the lanes per trace, but almost every wave has one such lane, so
// every wave pays for the walk with 1-4 lanes active (lane utilisation 0.22 on the cubes). Here the
// 4 waves of a block run each path vertex in lockstep phases separated by barriers:
//   A  camera / analytic closest hit (planes, spheres); lanes whose ray may reach a mesh queue a
//      closest-hit query per mesh in LDS;
//   B  the block's queued queries are processed densely, one lane per query, one wave per mesh chunk
//      of 64: flat_query evaluates the walk's result from every triangle of that mesh (scalar loads:
//      all lanes of a chunk query the same mesh);
//   C  the lane merges the mesh hits in Scene::trace_ray's order (ties to the lower object index),
//      shades the vertex; a shadow ray the analytic objects let through is queued per mesh;
//   D  shadow queries as in B;
//   E  the NEE term is added unless a mesh blocks the shadow ray (mutually_visible); sample and
//      subpixel bookkeeping, tickets.
// Every query returns the same bits as the per-lane walk (same tri_t, same box_hit per octant, same
// visiting order), so frames are identical to k_megakernel_f64's and the wavefront's (tested).
// Included by render_f64.hip (one code object: the diagnostic counters of path_f64.h are per code
// object).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../device/integrator_f64.h"
#include "kernels.h"
#include "megakernel_common.h"

namespace rt {
using namespace f64;

namespace {

constexpr int kFlatMeshes = 4;  // meshes of a flat scene (LDS queues)
constexpr int kBlk = 256;
typedef __attribute__((address_space(3))) double LdsD;
typedef __attribute__((address_space(3))) uint64_t LdsU;

// Mesh::intersect of a flat octree for the ray (geometry.rs:883-905, 1237-1295): the walk visits the
// root's children (leaves) in the ray's order (distances to the ROOT octant centres, root_order),
// takes the first one whose octant box the ray hits (box_hit) and that holds a triangle hit, and
// returns that leaf's nearest triangle (strict <: the first in leaf order, i.e. the lowest index).
// Evaluated here from every triangle's tri_t (the walk's own test, same bits) with the nearest hit
// kept per leaf; box tests and the order only for lanes with a hit. A root leaf is its nearest hit
// without any box test (geometry.rs:1237-1241). All lanes of the calling wave query mesh `m`.
RT_DEV bool flat_query(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, double* t_out,
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
            if (cand) {
                double d2[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const V3 dv = ld3(m.oct_center[i]) - ray.o;
                    d2[i] = dv.x * dv.x + dv.y * dv.y + dv.z * dv.z;  // mag()'s radicand, same order
                }
                const uint32_t order = root_order(d2);
#pragma unroll
                for (int q = 7; q >= 0; --q) {  // the first candidate in visiting order
                    const int oi = (int)((order >> (4 * q)) & 0xFu);
                    if ((cand >> oi) & 1u) win = oi;
                }
            }
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

// Phase B / D: the block's queued queries of round r, chunks of 64 entries of one mesh handed to
// the waves in turn; results to s_rt / s_rp [mesh][lane].
RT_DEV void process_queries(const DevScene& sc, const int32_t* cnt, const int32_t* queue, const LdsD* q,
                            double* rt, int32_t* rp) {
    const int wv = threadIdx.x >> 6, ln = __lane_id();
    int ci = 0;
    for (int m = 0; m < sc.n_meshes; ++m) {
        const int c = cnt[m];
        for (int k = 0; k * 64 < c; ++k, ++ci) {
            if ((ci & 3) != wv) continue;
            const int e = k * 64 + ln;
            RT_DBG_WAVE(13, lane_id_is0());
            RT_DBG_WAVE(12, e < c);
            if (e < c) {
                const int who = queue[m * kBlk + e];
                const Ray r{v3(q[who], q[kBlk + who], q[2 * kBlk + who]), v3(q[3 * kBlk + who], q[4 * kBlk + who], q[5 * kBlk + who])};
                const RayInv inv = make_inv(r.d);
                double t = 0.0;
                int prim = -1;
                const bool hit = flat_query(sc, sc.meshes[m], r, inv, &t, &prim);
                rt[m * kBlk + who] = t;
                rp[m * kBlk + who] = hit ? prim : -1;
            }
        }
    }
}

}  // namespace

template <int F, int W>
__global__ __launch_bounds__(kBlk, W) void k_megakernel_flat_f64(DevScene sc_g, RenderArgs a, double* __restrict__ sub_buf,
                                                                uint32_t* next_sub, long nsub, int refill) {
    using C = Cfg<F>;
    static_assert(C::mesh && C::compact && !C::bvh, "flat-mesh kernel: compact scenes, octree meshes");
    DevScene sc = sc_g;
    __shared__ DevObject s_objs[kMaxCompactObjects];
    {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(sc_g.objects);
        uint64_t* dst = reinterpret_cast<uint64_t*>(s_objs);
        const int nw = sc_g.n_objects * (int)(sizeof(DevObject) / 8);
        for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
        sc.objects = s_objs;
    }
    // per lane (one column per thread): subpixel accumulator, one-deep camera-sample buffer
    __shared__ double s_acc[3 * kBlk], s_nbd[3 * kBlk];
    __shared__ uint64_t s_nbr[2 * kBlk];
    LdsD* acc_l = (LdsD*)s_acc + threadIdx.x;
    LdsD* nbd = (LdsD*)s_nbd + threadIdx.x;
    LdsU* nbr = (LdsU*)s_nbr + threadIdx.x;
    // the lane's query ray (origin, direction) for the processing lane, results per (mesh, lane), and
    // the per-mesh queues of the closest (0) and shadow (1) rounds
    __shared__ double s_q[6 * kBlk];
    __shared__ double s_rt[kFlatMeshes * kBlk];
    __shared__ int32_t s_rp[kFlatMeshes * kBlk];
    __shared__ int32_t s_queue[kFlatMeshes * kBlk];
    __shared__ int32_t s_cnt[2][kFlatMeshes];
    __shared__ int32_t s_active;
    const int tid = threadIdx.x;
    if (tid < 2 * kFlatMeshes) s_cnt[tid / kFlatMeshes][tid % kFlatMeshes] = 0;
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
    bool fresh = true, nvalid = false;
    __syncthreads();
    for (;;) {
        RT_DBG_WAVE(8, lane_id_is0());
        RT_DBG_WAVE(9, active);
        RT_DBG_TSTART(t_a);
        // ---------------- A: camera, analytic closest hit, closest-hit queries
        if (tid < kFlatMeshes) s_cnt[1][tid] = 0;  // shadow round's queues (read in D of the last iteration)
        if (active && fresh && nvalid) {
            begin_path(sc, CameraSample{v3(nbd[0], nbd[kBlk], nbd[2 * kBlk]), nbr[0], nbr[kBlk]}, ps);
            fresh = false;
            nvalid = false;
        }
        {
            // camera pass: lanes starting a path now, plus buffer refills once >= refill lanes need one
            const bool now = active && fresh;
            const bool need = active && !fresh && !nvalid && unit_has_next(a, id, s);
            if (__any(now) || (refill > 0 && __popcll(__ballot(need)) >= refill)) {
                if (now || (refill > 0 && need)) {
                    const CameraSample nb = camera_sample(sc, a, subpixel_of(a, id), now ? s : s + 1);
                    if (now) {
                        begin_path(sc, nb, ps);
                        fresh = false;
                    } else {
                        nbd[0] = nb.d.x; nbd[kBlk] = nb.d.y; nbd[2 * kBlk] = nb.d.z;
                        nbr[0] = nb.r0; nbr[kBlk] = nb.r1;
                        nvalid = true;
                    }
                }
            }
        }
        HitRec h{0.0, -1, -1};
        RayInv inv{};
        double tmax = INFINITY;
        if (active) {
            inv = make_inv(ps.ray.d);
            h = trace_analytic<C>(sc, ps.ray, inv);
            tmax = h.obj >= 0 ? h.t : INFINITY;
            s_q[tid] = ps.ray.o.x; s_q[kBlk + tid] = ps.ray.o.y; s_q[2 * kBlk + tid] = ps.ray.o.z;
            s_q[3 * kBlk + tid] = ps.ray.d.x; s_q[4 * kBlk + tid] = ps.ray.d.y; s_q[5 * kBlk + tid] = ps.ray.d.z;
        }
        uint32_t qmask = 0;
        for (int m = 0; m < sc.n_meshes; ++m) {
            const DevMesh& M = sc.meshes[m];
            const bool want = active && near_box(M.cull_box, ps.ray, inv, M.cull_pad, tmax);
            qmask |= want ? (1u << m) : 0u;
            enqueue(&s_cnt[0][m], s_queue + m * kBlk, want);
        }
        RT_DBG_TEND(1, t_a);
        RT_DBG_TSTART(t_w1);
        __syncthreads();
        RT_DBG_TEND(6, t_w1);
        if (s_active == 0) break;  // every lane of the block is done (stable between E and the next A)
        // ---------------- B: closest-hit queries
        RT_DBG_TSTART(t_b);
        process_queries(sc, s_cnt[0], s_queue, (const LdsD*)s_q, s_rt, s_rp);
        RT_DBG_TEND(2, t_b);
        RT_DBG_TSTART(t_w2);
        __syncthreads();
        RT_DBG_TEND(6, t_w2);
        RT_DBG_TSTART(t_c);
        // ---------------- C: merge the mesh hits, shade, shadow queries
        if (tid < kFlatMeshes) s_cnt[0][tid] = 0;
        bool cont = false, pend = false;
        V3 pc = v3(0, 0, 0);
        double dist = 0.0;
        uint32_t smask = 0;
        Ray sr{v3(0, 0, 0), v3(0, 0, 1)};
        RayInv sinv{};
        if (active) {
            CTab* T = tables(sc);
            for (int g = 0; g < T->n_gen; ++g) {  // Scene::trace_ray's loop over the meshes (ties: lower index)
                const int idx = T->gen_idx[g];
                const DevObject& o = sc.objects[idx];
                if (o.geom == GEOM_MESH && ((qmask >> o.mesh) & 1u)) {
                    const int p = s_rp[o.mesh * kBlk + tid];
                    if (p >= 0) consider(h, s_rt[o.mesh * kBlk + tid], idx, p);
                }
            }
            nverts += h.obj >= 0;
            ShadowDefer df;
            df.pending = false;
            cont = shade_vertex<C>(sc, a, ps, h, &df);
            if (df.pending) {  // the analytic objects let the shadow ray through; a mesh may block it
                pend = true;
                pc = df.c;
                dist = df.dist;
                sr = Ray{df.o, df.d};
                sinv = make_inv(sr.d);
                s_q[tid] = sr.o.x; s_q[kBlk + tid] = sr.o.y; s_q[2 * kBlk + tid] = sr.o.z;
                s_q[3 * kBlk + tid] = sr.d.x; s_q[4 * kBlk + tid] = sr.d.y; s_q[5 * kBlk + tid] = sr.d.z;
            }
        }
        for (int m = 0; m < sc.n_meshes; ++m) {
            const DevMesh& M = sc.meshes[m];
            const bool want = pend && near_box(M.cull_box, sr, sinv, M.cull_pad, dist);
            smask |= want ? (1u << m) : 0u;
            enqueue(&s_cnt[1][m], s_queue + m * kBlk, want);
        }
        RT_DBG_TEND(3, t_c);
        RT_DBG_TSTART(t_w3);
        __syncthreads();
        RT_DBG_TEND(6, t_w3);
        // ---------------- D: shadow queries
        RT_DBG_TSTART(t_d);
        process_queries(sc, s_cnt[1], s_queue, (const LdsD*)s_q, s_rt, s_rp);
        RT_DBG_TEND(4, t_d);
        RT_DBG_TSTART(t_w4);
        __syncthreads();
        RT_DBG_TEND(6, t_w4);
        RT_DBG_TSTART(t_e);
        // ---------------- E: visibility, sample / subpixel bookkeeping, tickets
        bool done = false;
        if (active) {
            if (pend) {
                bool occluded = false;  // mutually_visible (scene.rs:258-270): t + 0.001 < |y - x|
                for (int m = 0; m < sc.n_meshes; ++m) {
                    if ((smask >> m) & 1u) {
                        const int p = s_rp[m * kBlk + tid];
                        occluded |= p >= 0 && !(s_rt[m * kBlk + tid] + 0.001 >= dist);
                    }
                }
                if (!occluded) ps.L = ps.L + pc;
            }
            if (!cont) {
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
                            nvalid = false;
                        } else {
                            done = true;
                        }
                    }
                } else {  // split tail (k_tail_sum_f64)
                    double* o = a.tail_buf + ((size_t)(id - a.n_whole) * (size_t)a.n_samples + (size_t)s) * 3;
                    o[0] = ps.L.x;
                    o[1] = ps.L.y;
                    o[2] = ps.L.z;
                    done = !unit_has_next(a, id, s);
                    ++s;
                }
            }
        }
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        if (__any(done)) flush_count(a.counters, nverts);
        bool ended = false;
        if (done) {
            unit_of(a, nt, id, end, s);
            active = !stop && nt < nunits;
            ended = !active;
            acc_l[0] = 0.0; acc_l[kBlk] = 0.0; acc_l[2 * kBlk] = 0.0;
            fresh = true;
            nvalid = false;
        }
        {
            const unsigned long long m = __ballot(ended);
            if (__lane_id() == 0 && m) atomicSub(&s_active, __popcll(m));
        }
        RT_DBG_TEND(5, t_e);
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

template <int F, int W>
static void launch_flat(const DevScene& sc, RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                        double* tail_buf, size_t tail_cap, int refill, hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_flat_f64<F, W>, (nsub + kBlk - 1) / kBlk);
    plan_tail(a, nsub, blocks * kBlk, tail_buf, tail_cap);
    hipLaunchKernelGGL((k_megakernel_flat_f64<F, W>), dim3((unsigned)blocks), dim3(kBlk), 0, st, sc, a, sub_buf,
                       next_sub, nsub, refill);
}

// The flat-mesh megakernel (scenes whose meshes are all DevMesh::flat; octree mode).
// RT_MK_FLAT_WAVES: waves/SIMD requested from the register allocator (2 or 3).
hipError_t launch_megakernel_flat_f64(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub,
                                      double* tail_buf, size_t tail_cap, int refill, hipStream_t st) {
    const long nsub = (long)a_in.tw * a_in.th * 4;
    RenderArgs a = a_in;
    static const int waves = env_int("RT_MK_FLAT_WAVES", 3);
#define RT_FLAT_CASE(F)                                                                       \
    case F:                                                                                   \
        if (waves == 2) launch_flat<F, 2>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, refill, st); \
        else launch_flat<F, 3>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, refill, st); \
        break;
    switch (a.features & 15) {
        RT_FLAT_CASE(9) RT_FLAT_CASE(11) RT_FLAT_CASE(13) RT_FLAT_CASE(15)
        default: return hipErrorInvalidValue;
    }
#undef RT_FLAT_CASE
    launch_tail_sum_f64(a, sub_buf, nsub - a.n_whole, st);
    return hipGetLastError();
}

}  // namespace rt
