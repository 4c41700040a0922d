// f64 render kernels for gfx950 (CDNA4).
//
//   k_megakernel_f64  — fused, persistent path loop (below); k_finalize_f64 — subpixel means -> RGB8.
//   k_trace_f64       — Scene::trace_ray for a batch of rays (parity tests of the intersectors).
//   wavefront kernels — see wavefront_f64.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../device/integrator_f64.h"
#include "kernels.h"
#include "megakernel_common.h"
#include "render_flat_f64.h"

namespace rt {
using namespace f64;

// Persistent megakernel: a resident grid whose lanes pull subpixels from a global counter. A lane
// walks the spp/4 sample paths of its subpixel vertex by vertex; when a path ends, the next sample
// starts in the same iteration (regeneration); when the subpixel is done its mean goes to
// sub_buf (sequential sum in sample order, server.rs:338-358) and the lane takes the next
// subpixel. Waves idle only in the frame's final tail, not per wave.
// W = minimum waves per SIMD requested from the register allocator.
#ifndef RT_CAM_DEPTH
#define RT_CAM_DEPTH 1  // camera samples buffered ahead per lane (k_megakernel_f64; 2 measured 1% slower)
#endif
constexpr int kCamDepth = RT_CAM_DEPTH;
typedef __attribute__((address_space(3))) double LdsDouble;
typedef __attribute__((address_space(3))) int32_t LdsInt;
typedef __attribute__((address_space(3))) uint64_t LdsU64;

#ifndef RT_OPT_LDSOBJ
#define RT_OPT_LDSOBJ 1  // A/B: the object table in LDS (per-lane object reads as ds_read)
#endif
#ifndef RT_OPT_COLD
#define RT_OPT_COLD 1  // A/B: mirror-bounce state (o, pre-bounce throughput) in LDS (LdsCold) or registers
#endif

template <int F, int W>
__global__ __launch_bounds__(256, W) void k_megakernel_f64(DevScene sc_g, RenderArgs a, double* __restrict__ sub_buf,
                                                          uint32_t* next_sub, long nsub, int refill) {
    using C = Cfg<F>;
    // Compact scenes (<= kMaxCompactObjects objects): the object table is copied into LDS, so the
    // shading's per-lane object reads (hit object, light) are ds_reads instead of global loads.
    DevScene sc = sc_g;
#if RT_OPT_LDSOBJ
    __shared__ DevObject s_objs[C::compact ? kMaxCompactObjects : 1];
    if constexpr (C::compact) {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(sc_g.objects);
        uint64_t* dst = reinterpret_cast<uint64_t*>(s_objs);
        const int nw = sc_g.n_objects * (int)(sizeof(DevObject) / 8);
        for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
        sc.objects = s_objs;
    }
#endif
    // Rarely touched per-lane state lives in LDS (one column per thread; VGPRs are the limit at 4
    // waves/SIMD): the subpixel accumulator (once per sample) and the camera-sample buffer — a ring
    // of kCamDepth next samples (camera ray + RNG state) per lane, computed ahead in passes the whole
    // wave runs once >= refill lanes have a free slot (begin_sample for the ~7% of lanes whose path
    // ended each iteration otherwise runs every iteration at that lane utilisation).
    __shared__ double s_acc[3 * 256], s_nbd[kCamDepth * 3 * 256];
    __shared__ uint64_t s_nbr[kCamDepth * 2 * 256];
#if RT_OPT_COLD
    __shared__ double s_cold[6 * 256];  // integrator_f64.h LdsCold: o and the pre-bounce throughput of mirror paths
    const LdsCold cold{(LdsDouble*)s_cold + threadIdx.x};
#else
    const RegCold cold{};
#endif
    LdsDouble* acc_l = (LdsDouble*)s_acc + threadIdx.x;  // component k at [k * 256]
    LdsDouble* nbd = (LdsDouble*)s_nbd + threadIdx.x;     // slot q, component k at [(q * 3 + k) * 256]
    LdsU64* nbr = (LdsU64*)s_nbr + threadIdx.x;           // slot q, word k at [(q * 2 + k) * 256]
    RT_DBG_TINIT();
    uint32_t nverts = 0;
    // tickets: whole subpixels, then the split tail's chunks (unit_of)
    const long n_split = nsub - a.n_whole;
    const long nunits = a.n_wunits + n_split * a.tail_cps;
    int id, s;  // subpixel (tile-local, < 2^31: rt_api.cpp check_params) and sample of the unit in hand
    const long t0 = wave_ticket(next_sub, true);
    {
        int end_unused;  // the run's end is recomputed when needed (run_end)
        unit_of(a, t0, id, end_unused, s);
    }
    bool active = t0 < nunits;
    acc_l[0] = 0.0; acc_l[256] = 0.0; acc_l[512] = 0.0;
    PathState ps;
    bool fresh = true;
    int nbuf = 0, hb = 0;  // buffered camera samples (s + 1 .. s + nbuf) and the ring's head slot
    while (__any(active)) {
        RT_DBG_REGION(0);
        RT_DBG_TSTART(t_it);
        bool done = false;
        // camera: a lane starting a path takes its next buffered sample, or joins the camera pass
        RT_DBG_TSTART(t_fr);
        if (active && fresh && nbuf > 0) {
            RT_DBG_REGION(2);
            const int q = hb * 3 * 256, r = hb * 2 * 256;
            begin_path(sc, CameraSample{v3(nbd[q], nbd[q + 256], nbd[q + 512]), nbr[r], nbr[r + 256]}, ps);
            fresh = false;
            hb = hb + 1 == kCamDepth ? 0 : hb + 1;
            --nbuf;
        }
        RT_DBG_TEND(1, t_fr);
        RT_DBG_TSTART(t_rf);
        // camera pass: lanes that start a path now without a buffered sample (sample s), plus lanes
        // with a free ring slot whose next sample (s + nbuf + 1) is in the same unit; run when any
        // lane needs a sample now or >= refill lanes have a free slot
        {
            const bool now = active && fresh;
            const bool need = active && !fresh && nbuf < kCamDepth && unit_has(a, id, s, s + nbuf + 1);
            if (__any(now) || (refill > 0 && __popcll(__ballot(need)) >= refill)) {
                if (now || (refill > 0 && need)) {
                    RT_DBG_REGION(3);
                    const CameraSample nb = camera_sample(sc, a, subpixel_of(a, id), now ? s : s + nbuf + 1);
                    if (now) {
                        begin_path(sc, nb, ps);
                        fresh = false;
                    } else {
                        int slot = hb + nbuf;
                        slot = slot >= kCamDepth ? slot - kCamDepth : slot;
                        const int q = slot * 3 * 256, r = slot * 2 * 256;
                        nbd[q] = nb.d.x; nbd[q + 256] = nb.d.y; nbd[q + 512] = nb.d.z;
                        nbr[r] = nb.r0; nbr[r + 256] = nb.r1;
                        ++nbuf;
                    }
                }
            }
        }
        RT_DBG_TEND(4, t_rf);
        if (active) {
            RT_DBG_REGION(1);
            RT_DBG_TSTART(t_tr);
            HitRec hr = trace_closest<C>(sc, ps.ray);
            RT_DBG_TEND(2, t_tr);
            nverts += hr.obj >= 0;
            RT_DBG_TSTART(t_sh);
            fresh = !shade_vertex<C>(sc, a, ps, hr, nullptr, cold);
            RT_DBG_TEND(3, t_sh);
            RT_DBG_TSTART(t_se);
            if (fresh) {
                RT_DBG_REGION(4);
                if (id < a.n_whole) {
                    V3 acc = v3(acc_l[0], acc_l[256], acc_l[512]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[256] = acc.y; acc_l[512] = acc.z;
                    if (++s == a.n_samples) {
                        double* o = sub_buf + (size_t)id * 3;
                        o[0] = acc.x;
                        o[1] = acc.y;
                        o[2] = acc.z;
                        if (id + 1 < run_end(a, id)) {  // the next subpixel of the run, no ticket
                            ++id;
                            s = 0;
                            acc_l[0] = 0.0; acc_l[256] = 0.0; acc_l[512] = 0.0;
                            nbuf = 0;
                            hb = 0;
                        } else {
                            done = true;
                        }
                    }
                } else {  // split tail: the sample's radiance, summed in order by k_tail_sum_f64
                    double* o = a.tail_buf + ((size_t)(id - a.n_whole) * (size_t)a.n_samples + (size_t)s) * 3;
                    o[0] = ps.L.x;
                    o[1] = ps.L.y;
                    o[2] = ps.L.z;
                    done = !unit_has_next(a, id, s);
                    ++s;
                }
            }
            RT_DBG_TEND(6, t_se);
        }
        RT_DBG_TSTART(t_bk);
        // cancellation (RenderJob::stop, server.rs:201-203): checked when a lane would start a new
        // subpixel; a set flag stops handing out work, lanes finish the subpixel they hold
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        if (__any(done)) flush_count(a.counters, nverts);  // keeps the 32-bit lane counts far from overflow
        if (done) {
            int end_unused;
            unit_of(a, nt, id, end_unused, s);
            active = !stop && nt < nunits;
            acc_l[0] = 0.0; acc_l[256] = 0.0; acc_l[512] = 0.0;
            fresh = true;
            nbuf = 0;
            hb = 0;
        }
        RT_DBG_TEND(5, t_bk);
        RT_DBG_TEND(0, t_it);
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

// Begins the octree walk of the next candidate mesh after gen slot g (Scene::trace_ray's /
// mutually_visible's loop over the mesh objects); false when no mesh is left.
// `top`: the LDS copy of mesh sc.top_mesh's top levels (walk-pool kernel), or null.
template <class C>
RT_DEV bool next_mesh_walk(const DevScene& sc, const Ray& r, const RayInv& inv, double tmax, int& g, int& mi,
                           OctWalk& w, const LdsTopI32* top = nullptr) {
    for (++g; g < tables(sc)->n_gen; ++g) {
        const DevObject& o = sc.objects[tables(sc)->gen_idx[g]];
        if (o.geom == GEOM_MESH &&
            walk_begin(sc, sc.meshes[o.mesh], r, inv, tmax, w, o.mesh == sc.top_mesh ? top : nullptr)) {
            mi = o.mesh;
            return true;
        }
    }
    return false;
}

// Megakernel for scenes with triangle meshes: octree walks interleaved with path vertices.
// A walk is long-tailed (tens of steps for the few rays that reach the mesh's box; none for the
// rest), so tracing it to completion inside the vertex makes every lane of the wave wait for the
// wave's longest walk. Here a lane whose ray needs a mesh walk parks its path and walks
// `ksteps` steps per iteration (walk_step is resumable), while the other lanes of the wave keep
// shading vertices; a lane rejoins the vertex work the iteration its walk ends. The walk queries
// are the wavefront's deferred ones (closest: the analytic hit, then the meshes in gen order with
// the reference's tie rule; shadow: the analytic objects let the ray through, then any mesh may
// block it), so every path produces the same bits as k_megakernel_f64 (tested).
enum : int { PH_TRACE = 0, PH_WALK_CLOSEST = 1, PH_WALK_SHADOW = 2 };

// The walk state of each lane lives in LDS between walk phases ("parked"), one column per thread
// of the block, so the vertex phase runs with the register footprint of the analytic kernel and
// the walk phase holds only the path state plus the walk (no scratch spills at 2 waves/SIMD).
// Doubles: ray o, d; 1/d; box mn, mx; walk best t; query t (closest hit so far / shadow distance);
// pending NEE term. Ints: walk cursor fields, closest hit object/prim, gen slot, mesh, occluded.
constexpr int kParkD = 21, kParkI = 16, kParkThreads = 256;
struct Park {  // typed in the LDS address space: ds_read/ds_write with one 32-bit base + immediate offsets
    LdsDouble* d;  // this thread's column of [kParkD][kParkThreads]
    LdsInt* i;     // [kParkI][kParkThreads]
    RT_DEV LdsDouble& D(int f) const { return d[f * kParkThreads]; }
    RT_DEV LdsInt& I(int f) const { return i[f * kParkThreads]; }
};
struct WalkRegs {  // the walk phase's working copy
    Ray wr;
    RayInv wi;
    OctWalk w;
    double wt;  // closest: hit t so far (h.t); shadow: |y - x|
    int32_t hobj, hprim, g, mi, occluded;
};
RT_DEV void park_store(const Park& p, const WalkRegs& r) {
    p.D(0) = r.wr.o.x; p.D(1) = r.wr.o.y; p.D(2) = r.wr.o.z;
    p.D(3) = r.wr.d.x; p.D(4) = r.wr.d.y; p.D(5) = r.wr.d.z;
    p.D(6) = r.wi.rx; p.D(7) = r.wi.ry; p.D(8) = r.wi.rz;
    for (int k = 0; k < 3; ++k) { p.D(9 + k) = r.w.mn[k]; p.D(12 + k) = r.w.mx[k]; }
    p.D(15) = r.w.bt;
    p.D(16) = r.wt;
    p.I(0) = r.w.cur; p.I(1) = r.w.depth; p.I(2) = (int32_t)r.w.path; p.I(3) = (int32_t)r.w.pm;
    p.I(4) = (int32_t)(uint32_t)r.w.stk; p.I(5) = (int32_t)(uint32_t)(r.w.stk >> 32); p.I(6) = (int32_t)r.w.stk8;
    p.I(7) = (int32_t)r.w.order; p.I(8) = r.w.lpos; p.I(9) = r.w.lend; p.I(10) = r.w.best;
    p.I(11) = r.hobj; p.I(12) = r.hprim; p.I(13) = r.g; p.I(14) = r.mi; p.I(15) = r.occluded;
}
RT_DEV void park_load(const Park& p, WalkRegs& r) {
    r.wr.o = v3(p.D(0), p.D(1), p.D(2));
    r.wr.d = v3(p.D(3), p.D(4), p.D(5));
    r.wi.rx = p.D(6); r.wi.ry = p.D(7); r.wi.rz = p.D(8);
    for (int k = 0; k < 3; ++k) { r.w.mn[k] = p.D(9 + k); r.w.mx[k] = p.D(12 + k); }
    r.w.bt = p.D(15);
    r.wt = p.D(16);
    r.w.cur = p.I(0); r.w.depth = p.I(1); r.w.path = (uint32_t)p.I(2); r.w.pm = (uint32_t)p.I(3);
    r.w.stk = (uint64_t)(uint32_t)p.I(4) | ((uint64_t)(uint32_t)p.I(5) << 32); r.w.stk8 = (uint32_t)p.I(6);
    r.w.order = (uint32_t)p.I(7); r.w.lpos = p.I(8); r.w.lend = p.I(9); r.w.best = p.I(10);
    r.hobj = p.I(11); r.hprim = p.I(12); r.g = p.I(13); r.mi = p.I(14); r.occluded = p.I(15);
}

// Nearest-triangle mode (Cfg::bvh): the BVH walk parks cur / sp / best / bt in the octree walk's
// slots I(0), I(1), I(10), D(15), and its stack in the slots the octree walk would use for its
// cursor (I(2..9)) and box (D(9..14) as int pairs): kBvhMaxDepth = 20 entries.
struct ParkStack {
    const Park& p;
    RT_DEV LdsInt& at(int e) const {
        return e < 8 ? p.I(2 + e) : ((LdsInt*)&p.D(9 + ((e - 8) >> 1)))[(e - 8) & 1];
    }
};
static_assert(kBvhMaxDepth <= 8 + 12, "BVH stack does not fit the park slots");
struct WalkRegsBvh {
    Ray wr;
    RayInv wi;
    BvhWalk w;
    double wt;
    int32_t hobj, hprim, g, mi, occluded;
};
RT_DEV void park_store_bvh(const Park& p, const WalkRegsBvh& r) {
    p.D(0) = r.wr.o.x; p.D(1) = r.wr.o.y; p.D(2) = r.wr.o.z;
    p.D(3) = r.wr.d.x; p.D(4) = r.wr.d.y; p.D(5) = r.wr.d.z;
    p.D(6) = r.wi.rx; p.D(7) = r.wi.ry; p.D(8) = r.wi.rz;
    p.D(15) = r.w.bt;
    p.D(16) = r.wt;
    p.I(0) = r.w.cur; p.I(1) = r.w.sp; p.I(10) = r.w.best;
    p.I(11) = r.hobj; p.I(12) = r.hprim; p.I(13) = r.g; p.I(14) = r.mi; p.I(15) = r.occluded;
}
RT_DEV void park_load_bvh(const Park& p, WalkRegsBvh& r) {
    r.wr.o = v3(p.D(0), p.D(1), p.D(2));
    r.wr.d = v3(p.D(3), p.D(4), p.D(5));
    r.wi.rx = p.D(6); r.wi.ry = p.D(7); r.wi.rz = p.D(8);
    r.w.bt = p.D(15);
    r.wt = p.D(16);
    r.w.cur = p.I(0); r.w.sp = p.I(1); r.w.best = p.I(10);
    r.hobj = p.I(11); r.hprim = p.I(12); r.g = p.I(13); r.mi = p.I(14); r.occluded = p.I(15);
}
// Begins the BVH walk of the next candidate mesh after gen slot g; false when no mesh is left.
template <class C>
RT_DEV bool next_mesh_walk_bvh(const DevScene& sc, const Ray& r, const RayInv& inv, double tmax, int& g, int& mi,
                               BvhWalk& w) {
    for (++g; g < tables(sc)->n_gen; ++g) {
        const DevObject& o = sc.objects[tables(sc)->gen_idx[g]];
        if (o.geom != GEOM_MESH) continue;
        const DevMesh& m = sc.meshes[o.mesh];
        if (m.bvh_n > 0 && near_box(m.cull_box, r, inv, m.cull_pad, tmax)) {
            mi = o.mesh;
            bvh_begin(m, tmax, w);
            return true;
        }
    }
    return false;
}

// A new walk query: ray, 1/d, query t (closest analytic hit / shadow distance) and hit so far; the
// first walk step begins the walk of the first candidate mesh (w.cur = -1: no walk in progress).
RT_DEV void park_query(const Park& p, const Ray& r, const RayInv& wi, double wt, int32_t hobj, int32_t hprim) {
    p.D(0) = r.o.x; p.D(1) = r.o.y; p.D(2) = r.o.z;
    p.D(3) = r.d.x; p.D(4) = r.d.y; p.D(5) = r.d.z;
    p.D(6) = wi.rx; p.D(7) = wi.ry; p.D(8) = wi.rz;
    p.D(16) = wt;
    p.I(0) = -1;
    p.I(11) = hobj; p.I(12) = hprim; p.I(13) = -1; p.I(15) = 0;
}

// One round of walk steps for the queries held by the lanes with `wk` (the query in park `pk`;
// closest: the closest-hit query of Scene::trace_ray, else the shadow query of mutually_visible):
// up to ksteps steps, after the first only while >= wmin lanes still walk. Returns, per lane,
// whether its query finished; the results are then in pk (D16 t, I11 object, I12 prim, I15
// occluded), otherwise the walk state is stored back into pk.
template <class C>
RT_DEV bool walk_round(const DevScene& sc, const Park& pk, const bool wk, const bool closest, int ksteps, int wmin) {
    bool walking = wk, done = false;
    if constexpr (C::bvh) {
      if (__any(walking)) {
        WalkRegsBvh r;
        if (walking) park_load_bvh(pk, r);
        const ParkStack stk{pk};
        for (int k = 0; k < ksteps && (k == 0 ? __any(walking) : __popcll(__ballot(walking)) >= wmin); ++k) {
            RT_DBG_WAVE(10, lane_id_is0());
            RT_DBG_WAVE(11, walking);
            if (walking) {
                bool fin = false;
                if (r.w.cur < 0) {  // begin the walk of the next candidate mesh (none left: done)
                    const double tmax = closest ? (r.hobj >= 0 ? r.wt : INFINITY) : r.wt;
                    fin = !next_mesh_walk_bvh<C>(sc, r.wr, r.wi, tmax, r.g, r.mi, r.w);
                } else {
                    const bool shadow = !closest;
                    const int st = bvh_step(sc, sc.meshes[r.mi], r.wr, r.wi, r.w, stk, shadow ? r.wt : -1.0);
                    if (st != WALK_RUN) {
                        if (!shadow) {
                            if (st == WALK_HIT) {
                                HitRec h{r.wt, r.hobj, r.hprim};
                                consider(h, r.w.bt, tables(sc)->gen_idx[r.g], r.w.best);
                                r.wt = h.t;
                                r.hobj = h.obj;
                                r.hprim = h.prim;
                            }
                        } else {
                            r.occluded = st == WALK_HIT && !(r.w.bt + 0.001 >= r.wt);  // mutually_visible
                            fin = r.occluded;
                        }
                        r.w.cur = -1;  // next step: the next mesh, if any
                    }
                }
                if (fin) {  // results for the vertex phase
                    walking = false;
                    done = true;
                    pk.D(16) = r.wt;
                    pk.I(11) = r.hobj;
                    pk.I(12) = r.hprim;
                    pk.I(15) = r.occluded;
                }
            }
        }
        if (walking) park_store_bvh(pk, r);
      }
    } else if (__any(walking)) {
        WalkRegs r;
        if (walking) park_load(pk, r);
        // up to ksteps steps; after the first, only while at least wmin lanes still walk
        for (int k = 0; k < ksteps && (k == 0 ? __any(walking) : __popcll(__ballot(walking)) >= wmin); ++k) {
            RT_DBG_WAVE(10, lane_id_is0());
            RT_DBG_WAVE(11, walking);
            if (walking) {
                bool fin = false;
                if (r.w.cur < 0) {  // begin the walk of the next candidate mesh (none left: done)
                    const double tmax = closest ? (r.hobj >= 0 ? r.wt : INFINITY) : r.wt;
                    fin = !next_mesh_walk<C>(sc, r.wr, r.wi, tmax, r.g, r.mi, r.w);
                } else {
                    double t;
                    int prim;
                    const int st = walk_step(sc, sc.meshes[r.mi], r.wr, r.wi, r.w, &t, &prim);
                    if (st != WALK_RUN) {
                        if (closest) {
                            if (st == WALK_HIT) {
                                HitRec h{r.wt, r.hobj, r.hprim};
                                consider(h, t, tables(sc)->gen_idx[r.g], prim);
                                r.wt = h.t;
                                r.hobj = h.obj;
                                r.hprim = h.prim;
                            }
                        } else {
                            r.occluded = st == WALK_HIT && !(t + 0.001 >= r.wt);  // mutually_visible's ERR_MARGIN
                            fin = r.occluded;
                        }
                        r.w.cur = -1;  // next step: the next mesh, if any
                    }
                }
                if (fin) {  // results for the vertex phase
                    walking = false;
                    done = true;
                    pk.D(16) = r.wt;
                    pk.I(11) = r.hobj;
                    pk.I(12) = r.hprim;
                    pk.I(15) = r.occluded;
                }
            }
        }
        if (walking) park_store(pk, r);
    }
    return done;
}

// Walk pool (P = true): the walk queries of a block go through one LDS work queue (LdsQueue,
// megakernel_common.h) instead of being walked by the lane that owns the path. A wave takes up to 64
// runnable queries from the queue (any owner's), walks them for `ksteps` steps, hands finished
// results to their owners (status word) and puts unfinished queries back. Walk steps then run with
// the block's queries packed into full waves instead of the ~27 walking lanes of the wave that owns
// them (the deep octree's walks are 0-40 steps long and needed by ~20% of the vertices, DESIGN.md
// §5). The queue holds each query at most once and a block has at most 256 queries (one per path),
// so a 256-entry ring cannot overflow.
struct WalkPool {
    LdsQueue q;
    uint8_t* status;    // LDS [256] per owner column: 0 closest query, 1 shadow query, 2 done
};
enum : uint8_t { POOL_CLOSEST = 0, POOL_SHADOW = 1, POOL_DONE = 2 };
constexpr int kPoolRefill = 8;  // refill only when at least this many lanes of the round are idle

// Compact park of the walk pool (fits 3 blocks of 256 threads per CU, i.e. 3 waves/SIMD): no 1/d
// (recomputed by make_inv when a query is loaded: the same bits), no NEE term (the owner keeps it in
// registers), depth / pm / stk8 packed in one word. Doubles: ray o, d; box mn, mx; walk best t;
// query t (closest hit so far / shadow distance). Ints: cur, depth | pm << 8 | stk8 << 16, path,
// stk (2 words), order, lpos, lend, best, hit object, hit prim, gen slot, mesh, occluded.
constexpr int kPark2D = 14, kPark2I = 14;
enum : int { P2_T = 13, P2_HOBJ = 9, P2_HPRIM = 10, P2_OCC = 13 };
RT_DEV void park2_store(const Park& p, const WalkRegs& r) {
    p.D(0) = r.wr.o.x; p.D(1) = r.wr.o.y; p.D(2) = r.wr.o.z;
    p.D(3) = r.wr.d.x; p.D(4) = r.wr.d.y; p.D(5) = r.wr.d.z;
    for (int k = 0; k < 3; ++k) { p.D(6 + k) = r.w.mn[k]; p.D(9 + k) = r.w.mx[k]; }
    p.D(12) = r.w.bt;
    p.D(13) = r.wt;
    p.I(0) = r.w.cur;
    p.I(1) = (int32_t)((uint32_t)r.w.depth | (r.w.pm << 8) | (r.w.stk8 << 16));
    p.I(2) = (int32_t)r.w.path;
    p.I(3) = (int32_t)(uint32_t)r.w.stk; p.I(4) = (int32_t)(uint32_t)(r.w.stk >> 32);
    p.I(5) = (int32_t)r.w.order; p.I(6) = r.w.lpos; p.I(7) = r.w.lend; p.I(8) = r.w.best;
    p.I(9) = r.hobj; p.I(10) = r.hprim; p.I(11) = r.g; p.I(12) = r.mi; p.I(13) = r.occluded;
}
RT_DEV void park2_load(const Park& p, WalkRegs& r) {
    r.wr.o = v3(p.D(0), p.D(1), p.D(2));
    r.wr.d = v3(p.D(3), p.D(4), p.D(5));
    r.wi = make_inv(r.wr.d);
    for (int k = 0; k < 3; ++k) { r.w.mn[k] = p.D(6 + k); r.w.mx[k] = p.D(9 + k); }
    r.w.bt = p.D(12);
    r.wt = p.D(13);
    r.w.cur = p.I(0);
    const uint32_t dps = (uint32_t)p.I(1);
    r.w.depth = (int32_t)(dps & 0xFFu); r.w.pm = (dps >> 8) & 0xFFu; r.w.stk8 = dps >> 16;
    r.w.path = (uint32_t)p.I(2);
    r.w.stk = (uint64_t)(uint32_t)p.I(3) | ((uint64_t)(uint32_t)p.I(4) << 32);
    r.w.order = (uint32_t)p.I(5); r.w.lpos = p.I(6); r.w.lend = p.I(7); r.w.best = p.I(8);
    r.hobj = p.I(9); r.hprim = p.I(10); r.g = p.I(11); r.mi = p.I(12); r.occluded = p.I(13);
}
// A new pool query (see park_query).
RT_DEV void park2_query(const Park& p, const Ray& r, double wt, int32_t hobj, int32_t hprim) {
    p.D(0) = r.o.x; p.D(1) = r.o.y; p.D(2) = r.o.z;
    p.D(3) = r.d.x; p.D(4) = r.d.y; p.D(5) = r.d.z;
    p.D(13) = wt;
    p.I(0) = -1;
    p.I(9) = hobj; p.I(10) = hprim; p.I(11) = -1; p.I(13) = 0;
}

// One pool round: up to ksteps walk steps over queries taken from the pool; a lane whose query
// finishes hands the result to its owner and, while steps remain, takes the next queued query
// (refill: the round keeps its lanes full). Unfinished queries go back to the pool. All lanes call.
template <class C>
RT_DEV bool pool_round(const DevScene& sc, const WalkPool& wp, LdsDouble* park_d, LdsInt* park_i, int need,
                       int ksteps, const LdsTopI32* top) {
    int32_t q = queue_take(wp.q, need);
    if (!__any(q >= 0)) return false;
    WalkRegs r;
    bool closest = false;
    auto col = [&](int32_t c) { return Park{park_d + c, park_i + c}; };
    if (q >= 0) {
        park2_load(col(q), r);
        closest = __hip_atomic_load(&wp.status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == POOL_CLOSEST;
    }
    for (int k = 0; k < ksteps; ++k) {
        RT_DBG_WAVE(10, lane_id_is0());
        RT_DBG_WAVE(11, q >= 0);
        if (q >= 0) {
            bool fin = false;
            if (r.w.cur < 0) {  // begin the walk of the next candidate mesh (none left: done)
                const double tmax = closest ? (r.hobj >= 0 ? r.wt : INFINITY) : r.wt;
                fin = !next_mesh_walk<C>(sc, r.wr, r.wi, tmax, r.g, r.mi, r.w, top);
            } else {
                double t;
                int prim;
                const int st = walk_step(sc, sc.meshes[r.mi], r.wr, r.wi, r.w, &t, &prim, r.mi == sc.top_mesh ? top : nullptr);
                if (st != WALK_RUN) {
                    if (closest) {
                        if (st == WALK_HIT) {
                            HitRec h{r.wt, r.hobj, r.hprim};
                            consider(h, t, tables(sc)->gen_idx[r.g], prim);
                            r.wt = h.t;
                            r.hobj = h.obj;
                            r.hprim = h.prim;
                        }
                    } else {
                        r.occluded = st == WALK_HIT && !(t + 0.001 >= r.wt);  // mutually_visible's ERR_MARGIN
                        fin = r.occluded;
                    }
                    r.w.cur = -1;  // next step: the next mesh, if any
                }
            }
            if (fin) {  // results for the owner's vertex phase, then the status word
                const Park pq = col(q);
                pq.D(P2_T) = r.wt;
                pq.I(P2_HOBJ) = r.hobj;
                pq.I(P2_HPRIM) = r.hprim;
                pq.I(P2_OCC) = r.occluded;
                __hip_atomic_store(&wp.status[q], (uint8_t)POOL_DONE, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                q = -1;
            }
        }
        if (k + 1 < ksteps && __popcll(__ballot(q < 0)) >= kPoolRefill) {
            const int32_t q2 = queue_take_each(wp.q, q < 0);
            if (q2 >= 0) {
                q = q2;
                park2_load(col(q), r);
                closest = __hip_atomic_load(&wp.status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == POOL_CLOSEST;
            }
        }
    }
    if (q >= 0) park2_store(col(q), r);
    queue_put(wp.q, q >= 0, q);
    return true;
}

template <int F, int W, bool P>
__global__ __launch_bounds__(256, W) void k_megakernel_mesh_f64(DevScene sc_g, RenderArgs a, double* __restrict__ sub_buf,
                                                               uint32_t* next_sub, long nsub, int ksteps, int wmin,
                                                               int refill, int pool_min, int pool_vmin) {
    using C = Cfg<F>;
    static_assert(C::mesh && C::compact, "mesh megakernel needs the compact tables");
    // object table in LDS, as in k_megakernel_f64 (2 blocks per CU: 2 x 78 KB of LDS)
    DevScene sc = sc_g;
#if RT_OPT_LDSOBJ
    __shared__ DevObject s_objs[kMaxCompactObjects];
    {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(sc_g.objects);
        uint64_t* dst = reinterpret_cast<uint64_t*>(s_objs);
        const int nw = sc_g.n_objects * (int)(sizeof(DevObject) / 8);
        for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
        sc.objects = s_objs;
    }
#endif
    __shared__ double s_park_d[(P ? kPark2D : kParkD) * kParkThreads];
    __shared__ int32_t s_park_i[(P ? kPark2I : kParkI) * kParkThreads];
    const Park park{(LdsDouble*)s_park_d + threadIdx.x, (LdsInt*)s_park_i + threadIdx.x};
    __shared__ int32_t s_ring[P ? 256 : 1];
    __shared__ uint8_t s_status[P ? 256 : 1];
    __shared__ uint32_t s_qhead, s_qtail;
    const WalkPool wp{LdsQueue{s_ring, &s_qhead, &s_qtail, 255u}, s_status};
    // pool: the top kTopDepth + 1 levels of the deepest mesh's octree in LDS (18.3 KB; the walks of
    // every query of the block start there), scene_layout.h: top_slot
    __shared__ int4 s_top[P ? kTopNodes * 2 : 1];
    const LdsTopI32* top = nullptr;
    if constexpr (P) {
        s_ring[threadIdx.x] = -1;
        if (threadIdx.x == 0) { s_qhead = 0; s_qtail = 0; }
        if (sc.top_mesh >= 0) {
            const int4* src = reinterpret_cast<const int4*>(sc.top_kids + sc.meshes[sc.top_mesh].top_base);
            for (int i = threadIdx.x; i < kTopNodes * 2; i += blockDim.x) s_top[i] = src[i];
            top = (const LdsTopI32*)(LdsInt*)s_top;
        }
        __syncthreads();
    }
    // subpixel accumulator and camera-sample buffer in LDS, as in k_megakernel_f64
    // (no camera-sample buffer in pool mode: its 10 KB of LDS are what a third block per CU needs)
    __shared__ double s_acc[3 * 256], s_nbd[P ? 1 : 3 * 256];
    __shared__ uint64_t s_nbr[P ? 1 : 2 * 256];
    LdsDouble* acc_l = (LdsDouble*)s_acc + threadIdx.x;
    LdsDouble* nbd = (LdsDouble*)s_nbd + (P ? 0 : threadIdx.x);
    LdsU64* nbr = (LdsU64*)s_nbr + (P ? 0 : threadIdx.x);
    if constexpr (P) refill = 0;
    V3 pc = v3(0, 0, 0);  // pool: the pending shadow query's NEE term (the park has no room for it)
    uint32_t nverts = 0;
    // tickets: whole subpixels, then the split tail's chunks (unit_of), as in k_megakernel_f64
    const long n_split = nsub - a.n_whole;
    const long nunits = a.n_wunits + n_split * a.tail_cps;
    int id, end, s;
    const long t0 = wave_ticket(next_sub, true);
    unit_of(a, t0, id, end, s);
    bool active = t0 < nunits;
    acc_l[0] = 0.0; acc_l[256] = 0.0; acc_l[512] = 0.0;
    PathState ps;
    bool fresh = true;
    bool nvalid = false;
    int phase = PH_TRACE;
    bool walking = false, cont = false;
    RT_DBG_TINIT();
    while (__any(active)) {
        RT_DBG_WAVE(8, lane_id_is0());
        RT_DBG_TSTART(t_it);
        RT_DBG_TSTART(t_wk);
        bool took = false;
        if constexpr (P) {
            // take queued queries (at least pool_min of them while this wave has paths to shade)
            const int ready = __popcll(__ballot(active && !walking));
            took = pool_round<C>(sc, wp, (LdsDouble*)s_park_d, (LdsInt*)s_park_i, ready ? pool_min : 1, ksteps, top);
            if (!took && !ready) {
                __builtin_amdgcn_s_sleep(2);  // every path of this wave waits on walks other waves hold
            }
            if (walking && __hip_atomic_load(&s_status[threadIdx.x], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == POOL_DONE)
                walking = false;
        } else if (__any(walking)) {
            if (walk_round<C>(sc, park, walking, phase == PH_WALK_CLOSEST, ksteps, wmin)) walking = false;
        }
        RT_DBG_TEND(1, t_wk);
        RT_DBG_TSTART(t_vx);
        bool done = false;
        const bool was_walking = walking;
        // pool: after a walk round, shade only once pool_vmin paths are ready (denser vertex phases)
        const bool vphase = !P || !took || __popcll(__ballot(active && !walking)) >= pool_vmin;
        RT_DBG_WAVE(9, vphase && active && !walking);
        if (vphase && active && !walking) {
            bool shade_now = false, sample_end = false, trace_now = true;
            HitRec h;
            if (phase == PH_WALK_SHADOW) {  // the shadow result, then (path going on) the next trace
                if constexpr (P) {
                    if (!park.I(P2_OCC)) ps.L = ps.L + pc;
                } else {
                    if (!park.I(15)) ps.L = ps.L + v3(park.D(17), park.D(18), park.D(19));
                }
                phase = PH_TRACE;
                sample_end = !cont;
                trace_now = cont;
            } else if (phase == PH_WALK_CLOSEST) {
                h = P ? HitRec{park.D(P2_T), park.I(P2_HOBJ), park.I(P2_HPRIM)} : HitRec{park.D(16), park.I(11), park.I(12)};
                shade_now = true;
                trace_now = false;
            }
            if (trace_now) {
                if (fresh) {
                    if (!P && nvalid) begin_path(sc, CameraSample{v3(nbd[0], nbd[256], nbd[512]), nbr[0], nbr[256]}, ps);
                    else begin_sample(sc, a, subpixel_of(a, id), s, ps);
                    nvalid = false;
                    fresh = false;
                }
                const RayInv wi = make_inv(ps.ray.d);
                h = trace_analytic<C>(sc, ps.ray, wi);
                if (mesh_candidate<C>(sc, ps.ray, wi, h.obj >= 0 ? h.t : INFINITY)) {
                    if constexpr (P) park2_query(park, ps.ray, h.t, h.obj, h.prim);
                    else park_query(park, ps.ray, wi, h.t, h.obj, h.prim);
                    if constexpr (P) s_status[threadIdx.x] = POOL_CLOSEST;
                    phase = PH_WALK_CLOSEST;
                    walking = true;
                } else {
                    shade_now = true;
                }
            }
            if (shade_now) {
                nverts += h.obj >= 0;
                ShadowDefer df;
                df.pending = false;
                cont = shade_vertex<C>(sc, a, ps, h, &df);
                phase = PH_TRACE;
                if (df.pending) {  // shade_vertex found a mesh that could block the shadow ray
                    const Ray sr{df.o, df.d};
                    if constexpr (P) {
                        park2_query(park, sr, df.dist, -1, -1);
                        pc = df.c;
                    } else {
                        park_query(park, sr, make_inv(sr.d), df.dist, -1, -1);
                        park.D(17) = df.c.x;
                        park.D(18) = df.c.y;
                        park.D(19) = df.c.z;
                    }
                    if constexpr (P) s_status[threadIdx.x] = POOL_SHADOW;
                    phase = PH_WALK_SHADOW;
                    walking = true;
                }
                if (!walking) sample_end = !cont;
            }
            if (sample_end) {
                fresh = true;
                if (id < a.n_whole) {
                    V3 acc = v3(acc_l[0], acc_l[256], acc_l[512]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[256] = acc.y; acc_l[512] = acc.z;
                    if (++s == a.n_samples) {
                        double* o = sub_buf + (size_t)id * 3;
                        o[0] = acc.x;
                        o[1] = acc.y;
                        o[2] = acc.z;
                        if (++id < end) {  // the next subpixel of the run, no ticket
                            s = 0;
                            acc_l[0] = 0.0; acc_l[256] = 0.0; acc_l[512] = 0.0;
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
        if constexpr (P) queue_put(wp.q, walking && !was_walking, (int32_t)threadIdx.x);
        RT_DBG_TEND(2, t_vx);
        RT_DBG_TSTART(t_bk);
        // camera-sample refill pass: lanes with a path in progress (walking or not) and a next sample
        // in the same unit
        const bool need = active && !fresh && !nvalid && unit_has_next(a, id, s);
        if (refill > 0 && __popcll(__ballot(need)) >= refill) {
            if (need) {
                const CameraSample nb = camera_sample(sc, a, subpixel_of(a, id), s + 1);
                nbd[0] = nb.d.x; nbd[256] = nb.d.y; nbd[512] = nb.d.z;
                nbr[0] = nb.r0; nbr[256] = nb.r1;
                nvalid = true;
            }
        }
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        if (__any(done)) flush_count(a.counters, nverts);  // keeps the 32-bit lane counts far from overflow
        if (done) {
            unit_of(a, nt, id, end, s);
            active = !stop && nt < nunits;
            acc_l[0] = 0.0; acc_l[256] = 0.0; acc_l[512] = 0.0;
            fresh = true;
            nvalid = false;
        }
        RT_DBG_TEND(4, t_bk);
        RT_DBG_TEND(0, t_it);
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

// Split tail: subpixel n_whole + j's mean from its samples' radiance, summed in sample order
// exactly as the megakernel's in-register accumulator (acc = acc + L * inv_n, server.rs:357-358).
// tail_buf is subpixel-major ([j][sample][3]): a chunk's lane writes one contiguous run (the
// sample-major layout scattered every write over the whole buffer: TLB misses, 2x slower tail).
__global__ __launch_bounds__(256) void k_tail_sum_f64(RenderArgs a, double* __restrict__ sub_buf, long n_split) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long j = (long)blockIdx.x * blockDim.x + threadIdx.x; j < n_split; j += stride) {
        V3 acc = v3(0.0, 0.0, 0.0);
        for (int s = 0; s < a.n_samples; ++s) {
            const double* L = a.tail_buf + ((size_t)j * (size_t)a.n_samples + (size_t)s) * 3;
            acc = acc + v3(L[0], L[1], L[2]) * a.inv_n;
        }
        double* o = sub_buf + (size_t)(a.n_whole + j) * 3;
        o[0] = acc.x;
        o[1] = acc.y;
        o[2] = acc.z;
    }
}

// 4 subpixel means -> RGB8 (server.rs:360 clamp-then-average, :366-368 gamma, :187-189 `as u8`).
__global__ __launch_bounds__(256) void k_finalize_f64(RenderArgs a, const double* __restrict__ sub_buf) {
    const long npix = (long)a.tw * a.th;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += stride) {
        const double* s = sub_buf + (size_t)p * 12;
        V3 pixel = v3(0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) pixel = pixel + clampv(v3(s[3 * j], s[3 * j + 1], s[3 * j + 2]), 0., 1.) * 0.25;
        V3 c = clampv(pixel, 0., 1.);
        const double g = 1.0 / 2.2;
        V3 gc = v3(pow(c.x, g), pow(c.y, g), pow(c.z, g)) * 255.0 + v3(0.5, 0.5, 0.5);
        a.rgb_out[p * 3 + 0] = as_u8(gc.x);
        a.rgb_out[p * 3 + 1] = as_u8(gc.y);
        a.rgb_out[p * 3 + 2] = as_u8(gc.z);
    }
}

__global__ __launch_bounds__(256) void k_trace_f64(DevScene sc, long n, const double* __restrict__ o,
                                                   const double* __restrict__ d, double* t, int32_t* obj,
                                                   double* pos, double* nrm, int nearest) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r{v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2])};
    HitRec h = nearest ? (sc.compact ? trace_closest<Cfg<25>>(sc, r) : trace_closest<Cfg<17>>(sc, r))
                       : (sc.compact ? trace_closest<Cfg<9>>(sc, r) : trace_closest<Cfg<1>>(sc, r));
    obj[i] = h.obj;
    t[i] = h.obj >= 0 ? h.t : 0.0;
    if (h.obj >= 0) {
        V3 p, nn;
        surface<Cfg<1>>(sc, r, h, &p, &nn);
        pos[3 * i] = p.x; pos[3 * i + 1] = p.y; pos[3 * i + 2] = p.z;
        nrm[3 * i] = nn.x; nrm[3 * i + 1] = nn.y; nrm[3 * i + 2] = nn.z;
    }
}

template <int F, int W>
static void launch_mk(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub, long nsub,
                      int refill, double* tail_buf, size_t tail_cap, hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_f64<F, W>, (nsub + 255) / 256);
    RenderArgs a = a_in;
    plan_tail(a, nsub, blocks * 256, tail_buf, tail_cap);
    hipLaunchKernelGGL((k_megakernel_f64<F, W>), dim3((unsigned)blocks), dim3(256), 0, st, sc, a, sub_buf, next_sub, nsub,
                       refill);
    const long n_split = nsub - a.n_whole;
    if (n_split > 0) {
        const long tb = std::max(1L, std::min(4096L, (n_split + 255) / 256));
        hipLaunchKernelGGL(k_tail_sum_f64, dim3((unsigned)tb), dim3(256), 0, st, a, sub_buf, n_split);
    }
}
template <int F, int W, bool P>
static void launch_mm(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub, long nsub,
                      int ksteps, int wmin, int refill, int pool_min, int pool_vmin, double* tail_buf, size_t tail_cap,
                      hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_mesh_f64<F, W, P>, (nsub + 255) / 256);
    RenderArgs a = a_in;
    plan_tail(a, nsub, blocks * 256, tail_buf, tail_cap);
    hipLaunchKernelGGL((k_megakernel_mesh_f64<F, W, P>), dim3((unsigned)blocks), dim3(256), 0, st, sc, a, sub_buf,
                       next_sub, nsub, ksteps, wmin, refill, pool_min, pool_vmin);
    const long n_split = nsub - a.n_whole;
    if (n_split > 0) {
        const long tb = std::max(1L, std::min(4096L, (n_split + 255) / 256));
        hipLaunchKernelGGL(k_tail_sum_f64, dim3((unsigned)tb), dim3(256), 0, st, a, sub_buf, n_split);
    }
}

hipError_t launch_megakernel_f64(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub,
                                 double* tail_buf, size_t tail_cap, hipStream_t st) {
    RenderArgs a = a_in;
    a.n_whole = (int32_t)((long)a.tw * a.th * 4);  // no split tail unless planned (analytic megakernel)
    a.chunk_lg = 0;
    a.tail_cps = 1;
    const long nsub = (long)a.tw * a.th * 4;
    if (nsub <= 0 || a.n_samples <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(next_sub, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    // Occupancy (waves/SIMD requested from the register allocator): 4 (128 VGPRs, a few spills)
    // measured fastest for the analytic scenes, 3 (no spills) for the fused mesh kernel
    // (profiles/r01_waves_ab.log); RT_MK_WAVES=3|4 overrides for A/B runs.
    static const int waves_env = env_int("RT_MK_WAVES", 0);
    const int waves = waves_env ? waves_env : ((a.features & 1) ? 3 : 4);
    // Mesh scenes with compact tables and an octree of at least RT_MK_INTERLEAVE nodes: interleaved
    // walks, RT_MK_KSTEPS walk steps per vertex iteration, 2 waves/SIMD (the parked walk state takes
    // 59 KB of LDS per block; 0 selects the fused per-vertex traversal for A/B runs). Shallow octrees (cubes: 9 nodes) walk in a few
    // steps: the fused traversal is faster there (profiles/r01_interleave_ab.log).
    static const int interleave = env_int("RT_MK_INTERLEAVE", 64);
    static const int ksteps = std::max(1, env_int("RT_MK_KSTEPS", 4));
    // camera-sample buffer refill threshold (lanes per wave; 0 disables the buffer)
    // (24 until round 2; 32-48 measured +0.6-0.9% on cornell, profiles/r02_ab.log)
    static const int refill = env_int("RT_MK_CAM_REFILL", 40);
    static const int wmin = std::max(1, env_int("RT_MK_WALK_MIN", 1));
    static const int bvh_fused = env_int("RT_MK_BVH_FUSED", 0);  // A/B: nearest-triangle mode without interleaving
    // scenes whose meshes are all flat octrees (the cubes): block-synchronous batched mesh queries
    static const int flat = env_int("RT_MK_FLAT", 1);
    if (flat && a.all_flat && (a.features & 25) == 9)
        return launch_megakernel_flat_f64(sc, a, sub_buf, next_sub, tail_buf, tail_cap, refill, st);
    if (interleave && (a.features & 9) == 9 && a.mesh_nodes >= interleave && !((a.features & 16) && bvh_fused)) {
        // octree walks through the block's walk pool, 2 waves/SIMD (RT_MK_POOL=3: 3 waves/SIMD, 37
        // spilled VGPRs, measured 6% slower; 0: each lane walks its own query)
        static const int pool = env_int("RT_MK_POOL", 1);
        static const int pool_min = env_int("RT_MK_POOL_MIN", 32);
        static const int pool_ksteps = std::max(1, env_int("RT_MK_POOL_KSTEPS", 6));
        static const int pool_vmin = env_int("RT_MK_POOL_VMIN", 0);
#define RT_MM_CASE(F)                                                                          \
    case F:                                                                                    \
        if (pool == 3) launch_mm<F, 3, true>(sc, a, sub_buf, next_sub, nsub, pool_ksteps, wmin, refill, pool_min, pool_vmin, tail_buf, tail_cap, st); \
        else if (pool) launch_mm<F, 2, true>(sc, a, sub_buf, next_sub, nsub, pool_ksteps, wmin, refill, pool_min, pool_vmin, tail_buf, tail_cap, st); \
        else launch_mm<F, 2, false>(sc, a, sub_buf, next_sub, nsub, ksteps, wmin, refill, 0, 0, tail_buf, tail_cap, st); \
        break;
#define RT_MMB_CASE(F)                                                                         \
    case F:                                                                                    \
        launch_mm<F, 2, false>(sc, a, sub_buf, next_sub, nsub, ksteps, wmin, refill, 0, 0, tail_buf, tail_cap, st); \
        break;
        switch (a.features & 31) {
            RT_MM_CASE(9) RT_MM_CASE(11) RT_MM_CASE(13) RT_MM_CASE(15)
            RT_MMB_CASE(25) RT_MMB_CASE(27) RT_MMB_CASE(29) RT_MMB_CASE(31)  // nearest-triangle meshes: BVH walks
        }
#undef RT_MMB_CASE
#undef RT_MM_CASE
        return hipGetLastError();
    }
    if (a.features & 16) {
        // nearest-triangle meshes (RT_FLAG_MESH_NEAREST) in small or non-compact scenes: BVH
        // traversal inline, 3 waves/SIMD
#define RT_MB_CASE(F)                                                                             \
    case F:                                                                                       \
        launch_mk<F, 3>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);          \
        break;
        switch (a.features & 31) {
            RT_MB_CASE(17) RT_MB_CASE(19) RT_MB_CASE(21) RT_MB_CASE(23) RT_MB_CASE(25) RT_MB_CASE(27) RT_MB_CASE(29)
            RT_MB_CASE(31)
        }
#undef RT_MB_CASE
        return hipGetLastError();
    }
#define RT_MK_CASE(F)                                                           \
    case F:                                                                     \
        if (waves == 3) launch_mk<F, 3>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);  \
        else launch_mk<F, RT_MK_W4>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);      \
        break;
    switch (a.features & 15) {
        RT_MK_CASE(0) RT_MK_CASE(1) RT_MK_CASE(2) RT_MK_CASE(3) RT_MK_CASE(4) RT_MK_CASE(5) RT_MK_CASE(6)
        RT_MK_CASE(7) RT_MK_CASE(8) RT_MK_CASE(9) RT_MK_CASE(10) RT_MK_CASE(11) RT_MK_CASE(12) RT_MK_CASE(13)
        RT_MK_CASE(14) RT_MK_CASE(15)
    }
#undef RT_MK_CASE
    return hipGetLastError();
}

void launch_tail_sum_f64(const RenderArgs& a, double* sub_buf, long n_split, hipStream_t st) {
    if (n_split <= 0) return;
    const long tb = std::max(1L, std::min(4096L, (n_split + 255) / 256));
    hipLaunchKernelGGL(k_tail_sum_f64, dim3((unsigned)tb), dim3(256), 0, st, a, sub_buf, n_split);
}

hipError_t launch_finalize_f64(const RenderArgs& a, const double* sub_buf, hipStream_t st) {
    const long npix = (long)a.tw * a.th;
    if (npix <= 0) return hipSuccess;
    const long blocks = std::max(1L, std::min(2048L, (npix + 255) / 256));
    hipLaunchKernelGGL(k_finalize_f64, dim3((unsigned)blocks), dim3(256), 0, st, a, sub_buf);
    return hipGetLastError();
}

// Self-test of the exact-arithmetic shortcuts against the IEEE operations they replace: for n
// pseudo-random (a, b) with |b| spread over [2^-900, 2^900] (every exponent, random and extreme
// mantissas), counts rcp_rn(b) != 1.0 / b and qdiv(a, b, rcp_rn(b)) != a / b.
__global__ void k_selftest_arith(long n, uint64_t seed, unsigned long long* bad) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rng g(seed, (uint32_t)i, (uint32_t)(i >> 32), 7u);
    const uint64_t m = g.next(), m2 = g.next(), sel = g.next();
    uint64_t mant = m & 0xFFFFFFFFFFFFFull;
    if ((sel & 7) == 0) mant = 0;                              // powers of two
    if ((sel & 7) == 1) mant = 0xFFFFFFFFFFFFFull;             // just below
    if ((sel & 7) == 2) mant = (sel >> 8) & 0xFF;              // just above
    const int ex = -900 + (int)((sel >> 16) % 1801);
    const uint64_t bits = ((uint64_t)(ex + 1023) << 52) | mant | ((sel >> 40) & 1 ? 0x8000000000000000ull : 0);
    const double b = __longlong_as_double((long long)bits);
    const double a = __longlong_as_double((long long)((m2 & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 + (int)((sel >> 48) % 200) - 100) << 52)));
    const double y = rcp_rn(b);
    unsigned long long e = 0;
    if (__double_as_longlong(y) != __double_as_longlong(1.0 / b)) e |= 1;
    if (__double_as_longlong(qdiv(a, b, y)) != __double_as_longlong(a / b)) e |= 2;
    if (e & 1) atomicAdd(&bad[0], 1ull);
    if (e & 2) atomicAdd(&bad[1], 1ull);
}

extern "C" int rt_selftest_arith(long n, unsigned long long seed, unsigned long long out[2]) {
    unsigned long long* d = nullptr;
    if (n <= 0 || hipMalloc(&d, 2 * sizeof(unsigned long long)) != hipSuccess) return -1;
    int rc = 0;
    if (hipMemset(d, 0, 2 * sizeof(unsigned long long)) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(k_selftest_arith, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, seed, d);
        if (hipGetLastError() != hipSuccess || hipMemcpy(out, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    }
    (void)hipFree(d);
    return rc;
}

// Diagnostic builds: read and clear the traversal counters (all zeros otherwise).
extern "C" int rt_debug_regions(unsigned long long out[64]) {
    for (int i = 0; i < 64; ++i) out[i] = 0;
    unsigned long long z[32] = {0};
#if RT_DEBUG_COUNTERS
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_region), sizeof(g_dbg_region)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_region), z, sizeof(g_dbg_region)) != hipSuccess) return -1;
#endif
#if RT_DEBUG_TIMERS
    if (hipMemcpyFromSymbol(out + 32, HIP_SYMBOL(g_dbg_time), sizeof(g_dbg_time)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_time), z, sizeof(g_dbg_time)) != hipSuccess) return -1;
#endif
    (void)z;
    return 0;
}

extern "C" int rt_debug_counters(unsigned long long out[16]) {
#if RT_DEBUG_COUNTERS
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(g_dbg)) != hipSuccess) return -1;
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), z, sizeof(z)) != hipSuccess) return -1;
#else
    for (int i = 0; i < 16; ++i) out[i] = 0;
#endif
    return 0;
}

hipError_t launch_trace_f64(const DevScene& sc, long n, const double* o, const double* d, double* t, int32_t* obj,
                            double* pos, double* nrm, bool mesh_nearest, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_trace_f64, dim3((unsigned)blocks), dim3(256), 0, st, sc, n, o, d, t, obj, pos, nrm,
                       mesh_nearest ? 1 : 0);
    return hipGetLastError();
}

}  // namespace rt
