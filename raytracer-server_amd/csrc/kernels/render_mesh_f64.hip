// f64 megakernel for scenes with deep triangle-mesh octrees (flying_unicorn): octree walks
// (Mesh::intersect, geometry.rs:883-905, 1237-1295) interleaved with path vertices, by default through
// the block's walk pool. Its own translation unit (code object): launched by launch_megakernel_f64
// (render_f64.hip) through launch_megakernel_mesh_f64.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../device/integrator_f64.h"
#include "kernels.h"
#include "megakernel_common.h"

namespace rt {
using namespace f64;

typedef __attribute__((address_space(3))) double LdsDouble;
typedef __attribute__((address_space(3))) int32_t LdsInt;
typedef __attribute__((address_space(3))) uint64_t LdsU64;
#ifndef RT_OPT_LDSOBJ
#define RT_OPT_LDSOBJ 1  // A/B: the object table in LDS (per-lane object reads as ds_read)
#endif

// Begins the octree walk of the next candidate mesh after gen slot g (Scene::trace_ray's /
// mutually_visible's loop over the mesh objects); false when no mesh is left. S: the slot walk
// (walk_step<true>, DevScene::node_slot) or the node_kids walk.
template <class C, bool S>
RT_DEV bool next_mesh_walk(const DevScene& sc, const Ray& r, const RayInv& inv, double tmax, int& g, int& mi,
                           OctWalk& w) {
    CTab* T = tables(sc);
    for (++g; g < T->n_gen; ++g) {
        const int mm = T->gen_mesh[g];  // the slot's mesh (non-empty octree), or -1 (CompactTab)
        if (mm >= 0 && walk_begin<S>(sc, sc.meshes[mm], r, inv, tmax, w)) {
            mi = mm;
            return true;
        }
    }
    return false;
}
// The walk pool's form: `near` = the meshes the query's owner found near the ray (mesh_near_mask, same
// tmax), so only those are begun, without repeating their near_box test.
template <class C, bool S>
RT_DEV bool next_mesh_walk_near(const DevScene& sc, const Ray& r, const RayInv& inv, double tmax, int& g, int& mi,
                                OctWalk& w, uint32_t near) {
    CTab* T = tables(sc);
    for (++g; g < T->n_gen; ++g) {
        // the slot's mesh from the compact table (one load, not the object and then its mesh); `near`
        // only has bits of meshes with a non-empty octree, like gen_mesh
        const int mm = T->gen_mesh[g];
        if (mm >= 0 && ((near >> mm) & 1u) && walk_begin<S>(sc, sc.meshes[mm], r, inv, tmax, w, false)) {
            mi = mm;
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
constexpr int kParkD = 21, kParkI = 18, kParkThreads = 256;
// Threads of a walk-pool block: 512 = one block per CU (150 KB of LDS) whose 8 waves share one walk queue,
// so a wave's pool round finds full sets of queries sooner (unicorn 1920x1080x32: 222.6 vs 219.3 Msamples/s
// with two 256-thread blocks per CU, profiles/r04_ab.log)
#ifndef RT_POOL_BLOCK
#define RT_POOL_BLOCK 512
#endif
constexpr int kPoolThreads = RT_POOL_BLOCK;
template <int T = kParkThreads>
struct ParkT {  // typed in the LDS address space: ds_read/ds_write with one 32-bit base + immediate offsets
    LdsDouble* d;  // this thread's column of [kParkD][T]
    LdsInt* i;     // [kParkI][T]
    RT_DEV LdsDouble& D(int f) const { return d[f * T]; }
    RT_DEV LdsInt& I(int f) const { return i[f * T]; }
};
using Park = ParkT<kParkThreads>;    // the per-lane walks (P = 0)
using Park2 = ParkT<kPoolThreads>;  // the walk pool's compact park
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
    p.I(0) = r.w.cur; p.I(1) = r.w.depth | (int32_t)(r.w.ndone << 24) | (int32_t)(r.w.enter << 25); p.I(2) = (int32_t)r.w.path;
    p.I(3) = (int32_t)r.w.pm;
    p.I(4) = (int32_t)(uint32_t)r.w.stk; p.I(5) = (int32_t)(uint32_t)(r.w.stk >> 32); p.I(6) = (int32_t)r.w.stk8;
    p.I(7) = (int32_t)r.w.order; p.I(8) = r.w.lpos; p.I(9) = r.w.lend; p.I(10) = r.w.best;
    p.I(11) = r.hobj; p.I(12) = r.hprim; p.I(13) = r.g; p.I(14) = r.mi; p.I(15) = r.occluded;
    p.I(16) = r.w.nlf; p.I(17) = r.w.nle;
}
RT_DEV void park_load(const Park& p, WalkRegs& r) {
    r.wr.o = v3(p.D(0), p.D(1), p.D(2));
    r.wr.d = v3(p.D(3), p.D(4), p.D(5));
    r.wi.rx = p.D(6); r.wi.ry = p.D(7); r.wi.rz = p.D(8);
    for (int k = 0; k < 3; ++k) { r.w.mn[k] = p.D(9 + k); r.w.mx[k] = p.D(12 + k); }
    r.w.bt = p.D(15);
    r.wt = p.D(16);
    r.w.cur = p.I(0); r.w.depth = p.I(1) & 0xFF; r.w.ndone = ((uint32_t)p.I(1) >> 24) & 1u;
    r.w.enter = ((uint32_t)p.I(1) >> 25) & 3u; r.w.path = (uint32_t)p.I(2);
    r.w.pm = (uint32_t)p.I(3);
    r.w.stk = (uint64_t)(uint32_t)p.I(4) | ((uint64_t)(uint32_t)p.I(5) << 32); r.w.stk8 = (uint32_t)p.I(6);
    r.w.order = (uint32_t)p.I(7); r.w.lpos = p.I(8); r.w.lend = p.I(9); r.w.best = p.I(10);
    r.hobj = p.I(11); r.hprim = p.I(12); r.g = p.I(13); r.mi = p.I(14); r.occluded = p.I(15);
    r.w.nlf = p.I(16); r.w.nle = p.I(17);
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
        const DevObject& o = object_at<C>(sc, tables(sc)->gen_idx[g]);
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
template <class C, bool S>
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
                    fin = !next_mesh_walk<C, S>(sc, r.wr, r.wi, tmax, r.g, r.mi, r.w);
                } else {
                    double t;
                    int prim;
                    const int st = walk_step<S, 256, C::phong ? 0 : RT_WALK_HOIST>(sc, sc.meshes[r.mi], r.wr, r.wi, r.w, &t, &prim);
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
// §5). The queue holds each query at most once and a block has at most one query per path (thread),
// so a ring with an entry per thread cannot overflow.
struct WalkPool {
    LdsQueue q;
    uint8_t* status;    // LDS [block] per owner column: 0 closest query, 1 shadow query, 2 done
};
enum : uint8_t { POOL_CLOSEST = 0, POOL_SHADOW = 1, POOL_DONE = 2 };
#ifndef RT_POOL_PRIO
#define RT_POOL_PRIO 1  // the walk round at raised issue priority (s_setprio 1: its dependent loads issue ahead of the
                        // other wave's shading; unicorn +2.3%, r04an), 0 = none, 2 = the vertex phase raised (-2.1%)
#endif
#ifndef RT_POOL_REFILL
#define RT_POOL_REFILL 32
#endif
#ifndef RT_POOL_CAMBUF
#define RT_POOL_CAMBUF 1  // A/B: the walk pool keeps a camera-sample buffer (refill pass) as k_megakernel_f64
#endif
constexpr int kPoolRefill = RT_POOL_REFILL;  // refill only when at least this many lanes of the round are idle

// Compact park of the walk pool (fits 3 blocks of 256 threads per CU, i.e. 3 waves/SIMD): no 1/d
// (recomputed by make_inv when a query is loaded: the same bits), no NEE term (the owner keeps it in
// registers), depth / pm / stk8 packed in one word. Doubles: ray o, d; box mn, mx; walk best t;
// query t (closest hit so far / shadow distance). Ints: cur, depth | pm << 8 | stk8 << 16, path,
// stk (2 words), order, lpos, lend, best, hit object, hit prim, gen slot, mesh, occluded.
#ifndef RT_PARK_INV
#define RT_PARK_INV 0  // A/B: the park keeps 1/d (1) or park2_load recomputes it (0; its 6 KB of LDS hold the
                       // pool's camera-sample buffer instead, RT_POOL_CAMBUF)
#endif
constexpr int kPark2D = RT_PARK_INV ? 17 : 14, kPark2I = 17;
enum : int { P2_T = 13, P2_HOBJ = 9, P2_HPRIM = 10, P2_OCC = 13, P2_NEAR = 16 };
RT_DEV void park2_store(const Park2& p, const WalkRegs& r) {
    p.D(0) = r.wr.o.x; p.D(1) = r.wr.o.y; p.D(2) = r.wr.o.z;
    p.D(3) = r.wr.d.x; p.D(4) = r.wr.d.y; p.D(5) = r.wr.d.z;
    for (int k = 0; k < 3; ++k) { p.D(6 + k) = r.w.mn[k]; p.D(9 + k) = r.w.mx[k]; }
    p.D(12) = r.w.bt;
    p.D(13) = r.wt;
#if RT_PARK_INV
    p.D(14) = r.wi.rx; p.D(15) = r.wi.ry; p.D(16) = r.wi.rz;
#endif
    p.I(0) = r.w.cur;
    p.I(1) = (int32_t)((uint32_t)r.w.depth | (r.w.pm << 8) | (r.w.stk8 << 16) | (r.w.ndone << 24) | (r.w.enter << 25));
    p.I(2) = (int32_t)r.w.path;
    p.I(3) = (int32_t)(uint32_t)r.w.stk; p.I(4) = (int32_t)(uint32_t)(r.w.stk >> 32);
    p.I(5) = (int32_t)r.w.order; p.I(6) = r.w.lpos; p.I(7) = r.w.lend; p.I(8) = r.w.best;
    p.I(9) = r.hobj; p.I(10) = r.hprim; p.I(11) = r.g; p.I(12) = r.mi; p.I(13) = r.occluded;
    p.I(14) = r.w.nlf; p.I(15) = r.w.nle;
}
RT_DEV void park2_load(const Park2& p, WalkRegs& r) {
    r.wr.o = v3(p.D(0), p.D(1), p.D(2));
    r.wr.d = v3(p.D(3), p.D(4), p.D(5));
#if RT_PARK_INV
    r.wi.rx = p.D(14); r.wi.ry = p.D(15); r.wi.rz = p.D(16);
#else
    r.wi = make_inv(r.wr.d);
#endif
    for (int k = 0; k < 3; ++k) { r.w.mn[k] = p.D(6 + k); r.w.mx[k] = p.D(9 + k); }
    r.w.bt = p.D(12);
    r.wt = p.D(13);
    r.w.cur = p.I(0);
    const uint32_t dps = (uint32_t)p.I(1);
    r.w.depth = (int32_t)(dps & 0xFFu); r.w.pm = (dps >> 8) & 0xFFu; r.w.stk8 = (dps >> 16) & 0xFFu;
    r.w.ndone = (dps >> 24) & 1u; r.w.enter = (dps >> 25) & 3u;
    r.w.path = (uint32_t)p.I(2);
    r.w.stk = (uint64_t)(uint32_t)p.I(3) | ((uint64_t)(uint32_t)p.I(4) << 32);
    r.w.order = (uint32_t)p.I(5); r.w.lpos = p.I(6); r.w.lend = p.I(7); r.w.best = p.I(8);
    r.hobj = p.I(9); r.hprim = p.I(10); r.g = p.I(11); r.mi = p.I(12); r.occluded = p.I(13);
    r.w.nlf = p.I(14); r.w.nle = p.I(15);
}
// A new pool query (see park_query); near: the meshes near the ray (mesh_near_mask).
RT_DEV void park2_query(const Park2& p, const Ray& r, const RayInv& wi, double wt, int32_t hobj, int32_t hprim,
                        uint32_t near) {
    p.I(P2_NEAR) = (int32_t)near;
#if RT_PARK_INV
    p.D(14) = wi.rx; p.D(15) = wi.ry; p.D(16) = wi.rz;
#else
    (void)wi;
#endif
    p.D(0) = r.o.x; p.D(1) = r.o.y; p.D(2) = r.o.z;
    p.D(3) = r.d.x; p.D(4) = r.d.y; p.D(5) = r.d.z;
    p.D(13) = wt;
    p.I(0) = -1;
    p.I(9) = hobj; p.I(10) = hprim; p.I(11) = -1; p.I(13) = 0;
}

// One pool round: up to ksteps walk steps over queries taken from the pool; a lane whose query
// finishes hands the result to its owner and, while steps remain, takes the next queued query
// (refill: the round keeps its lanes full). Unfinished queries go back to the pool. All lanes call.
template <class C, bool S>
RT_DEV bool pool_round(const DevScene& sc, const WalkPool& wp, LdsDouble* park_d, LdsInt* park_i, int need,
                       int ksteps) {
    RT_DBG_TSTART(t_tk);
    int32_t q = queue_take(wp.q, need);
    if (!__any(q >= 0)) {
        RT_DBG_TEND(3, t_tk);
        return false;
    }
    WalkRegs r;
    bool closest = false;
    auto col = [&](int32_t c) { return Park2{park_d + c, park_i + c}; };
    if (q >= 0) {
        park2_load(col(q), r);
        const uint8_t stq = __hip_atomic_load(&wp.status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        closest = stq == POOL_CLOSEST;
        if (RT_QCHECK && stq != POOL_CLOSEST && stq != POOL_SHADOW) RT_QFAIL(3);
    }
    RT_DBG_TEND(3, t_tk);
    for (int k = 0; k < ksteps; ++k) {
        RT_DBG_WAVE(10, lane_id_is0());
        RT_DBG_WAVE(11, q >= 0);
        if (q >= 0) {
            bool fin = false;
            if (r.w.cur < 0) {  // begin the walk of the next candidate mesh (none left: done)
                RT_DBG_TSTART(t_bg);
                const double tmax = closest ? (r.hobj >= 0 ? r.wt : INFINITY) : r.wt;
                fin = !next_mesh_walk_near<C, S>(sc, r.wr, r.wi, tmax, r.g, r.mi, r.w, (uint32_t)col(q).I(P2_NEAR));
                RT_DBG_TEND(15, t_bg);
            }
            // (a walk begun above takes its first step right away: the slot walk enters the root there)
            if (!fin && r.w.cur >= 0) {
                double t;
                int prim;
                const int st = walk_step<S, kPoolThreads, C::phong ? 0 : RT_WALK_HOIST>(sc, sc.meshes[r.mi], r.wr, r.wi, r.w, &t, &prim,
                                            S ? (LdsAncI32*)park_i + kPark2I * kPoolThreads + q : nullptr);
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
                    fin |= r.g >= tables(sc)->last_mesh_g;  // none: the query's result is complete now
                }
            }
            if (fin) {  // results for the owner's vertex phase, then the status word
                const Park2 pq = col(q);
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
                const uint8_t stq = __hip_atomic_load(&wp.status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                closest = stq == POOL_CLOSEST;
                if (RT_QCHECK && stq != POOL_CLOSEST && stq != POOL_SHADOW) RT_QFAIL(3);
            }
        }
    }
    RT_DBG_TSTART(t_pt);
    if (q >= 0) park2_store(col(q), r);
    queue_put(wp.q, q >= 0, q);
    RT_DBG_TEND(5, t_pt);
    return true;
}

template <int F, int W, int P, bool S, int B = P ? kPoolThreads : 256>
__global__ __launch_bounds__(B, W) void k_megakernel_mesh_f64(DevScene sc_g, RenderArgs a_g, double* __restrict__ sub_buf,
                                                               uint32_t* next_sub, long nsub, int ksteps, int wmin,
                                                               int refill, int pool_min, int pool_vmin) {
    using C = Cfg<F | (RT_OPT_LDSOBJ ? kCfgLdsObj : 0)>;
    static_assert(C::mesh && C::compact, "mesh megakernel needs the compact tables");
    static_assert(B % 64 == 0 && B <= 1024, "whole waves, at most 16 (path_f64.h: the diagnostic builds' per-wave LDS)");
    static_assert(!P || (B & (B - 1)) == 0, "the walk queue's ring (one entry per thread) masks its index with B - 1");
    // object table in LDS, as in k_megakernel_f64; the arguments read in place (megakernel_common.h)
#if RT_KARG_VIEW
    const DevScene& sc = karg_scene();
    const RenderArgs& a = karg_render_args();
#else
    const DevScene& sc = sc_g;
    const RenderArgs& a = a_g;
#endif
    if constexpr (C::ldsobj) lds_objects_fill(sc);
    __shared__ double s_park_d[(P ? kPark2D : kParkD) * B];
    // pool: + the slot walk's ancestor ids (walk_node_slots)
    __shared__ int32_t s_park_i[(P ? kPark2I + (S ? kSlotAncLevels : 0) : kParkI) * B];
    const ParkT<B> park{(LdsDouble*)s_park_d + threadIdx.x, (LdsInt*)s_park_i + threadIdx.x};
    // P = 1: one walk queue
    __shared__ int32_t s_ring[1][P ? B : 1];
    __shared__ uint8_t s_status[P ? B : 1];
    __shared__ uint32_t s_qhead[2], s_qtail[2];
    WalkPool wp;
    wp.q = LdsQueue{s_ring[0], s_qhead, s_qtail, (uint32_t)B - 1u};
    wp.status = s_status;
    if constexpr (P) {
        s_ring[0][threadIdx.x] = -1;
        if (threadIdx.x < 2) { s_qhead[threadIdx.x] = 0; s_qtail[threadIdx.x] = 0; }
        __syncthreads();
    }
    // subpixel accumulator and camera-sample buffer in LDS, as in k_megakernel_f64 (pool mode: the
    // buffer's 10 KB fit beside the park at 2 blocks per CU without the parked 1/d, RT_PARK_INV = 0)
    constexpr bool kCamBuf = !P || RT_POOL_CAMBUF;
    __shared__ double s_acc[3 * B], s_nbd[kCamBuf ? 3 * B : 1];
    __shared__ uint64_t s_nbr[kCamBuf ? 2 * B : 1];
    LdsDouble* acc_l = (LdsDouble*)s_acc + threadIdx.x;
    LdsDouble* nbd = (LdsDouble*)s_nbd + (kCamBuf ? threadIdx.x : 0);
    LdsU64* nbr = (LdsU64*)s_nbr + (kCamBuf ? threadIdx.x : 0);
    if constexpr (!kCamBuf) refill = 0;
    V3 pc = v3(0, 0, 0);  // pool: the pending shadow query's NEE term (the park has no room for it)
    uint32_t nverts = 0;
    // tickets: whole subpixels, then the split tail's chunks (unit_of), as in k_megakernel_f64
    const long n_split = nsub - a.n_whole;
    const long nunits = a.n_wunits + n_split * a.tail_cps;
    int id, end, s;
    const long t0 = wave_ticket(next_sub, true);
    unit_of(a, t0, id, end, s);
    bool active = t0 < nunits;
    acc_l[0] = 0.0; acc_l[B] = 0.0; acc_l[2 * B] = 0.0;
    PathState ps;
    bool fresh = true;
    bool nvalid = false;
    int phase = PH_TRACE;
    bool walking = false, cont = false;
    HitRec hh{0.0, -1, -1};  // pool kernel: the hit this path shades next (walk result or analytic trace)
    bool has_hit = false;
    RT_DBG_TINIT();
    while (__any(active)) {
        RT_DBG_WAVE(8, lane_id_is0());
        RT_DBG_TSTART(t_it);
        RT_DBG_TSTART(t_wk);
        bool took = false;
        if constexpr (P) {
            // take queued queries (at least pool_min of them while this wave has paths to shade)
            const int ready = __popcll(__ballot(active && !walking));
#if RT_POOL_PRIO == 1
            __builtin_amdgcn_s_setprio(1);  // A/B: the walk round at raised issue priority
#endif
            took = pool_round<C, S>(sc, wp, (LdsDouble*)s_park_d, (LdsInt*)s_park_i, ready ? pool_min : 1, ksteps);
#if RT_POOL_PRIO == 1
            __builtin_amdgcn_s_setprio(0);
#endif
            if (!took && !ready) {
                __builtin_amdgcn_s_sleep(2);  // every path of this wave waits on walks other waves hold
            }
            if (walking && __hip_atomic_load(&s_status[threadIdx.x], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == POOL_DONE)
                walking = false;
        } else if (__any(walking)) {
            if (walk_round<C, S>(sc, park, walking, phase == PH_WALK_CLOSEST, ksteps, wmin)) walking = false;
        }
        RT_DBG_TEND(1, t_wk);
        RT_DBG_TSTART(t_vx);
        bool done = false;
        const bool was_walking = walking;
        // pool: after a walk round, shade only once pool_vmin paths are ready (denser vertex phases)
        const bool vphase = !P || !took || __popcll(__ballot(active && !walking)) >= pool_vmin;
#if RT_POOL_PRIO == 2
        __builtin_amdgcn_s_setprio(1);  // A/B: the vertex phase at raised issue priority (lowered at the iteration's end)
#endif
        RT_DBG_WAVE(9, vphase && active && !walking);
        if constexpr (P) {
          // Pool kernel: per iteration a ready path first shades the hit it holds (the closest walk's
          // result, or its last trace's analytic hit), then traces its next ray (the path going on, or
          // the unit's next sample): one shade block and one trace block per iteration, and a vertex
          // whose closest hit needed a walk traces its successor in the same iteration as its shading.
          if (vphase && active && !walking) {
            bool sample_end = false;
#if RT_DEBUG_COUNTERS
            bool after_s = false;  // diagnostic: a closest query right after this vertex's shadow query
#endif
            if (phase == PH_WALK_SHADOW) {  // the shadow result (mutually_visible's mesh part)
                if (!park.I(P2_OCC)) ps.L = ps.L + pc;
                phase = PH_TRACE;
                sample_end = !cont;
#if RT_DEBUG_COUNTERS
                after_s = cont;
#endif
            } else if (phase == PH_WALK_CLOSEST) {  // the closest hit: shaded now
                hh = HitRec{park.D(P2_T), park.I(P2_HOBJ), park.I(P2_HPRIM)};
                has_hit = true;
                phase = PH_TRACE;
            }
            if (has_hit) {
                has_hit = false;
                nverts += hh.obj >= 0;
                ShadowDefer df;
                df.pending = false;
                RT_DBG_TSTART(t_sv);
                cont = shade_vertex<C>(sc, a, ps, hh, &df);
                RT_DBG_TEND(8, t_sv);
                if (df.pending) {  // shade_vertex found a mesh that could block the shadow ray
                    RT_DBG(12);
                    park2_query(park, Ray{df.o, df.d}, df.inv, df.dist, -1, -1, df.meshes);
                    pc = df.c;
                    s_status[threadIdx.x] = POOL_SHADOW;
                    phase = PH_WALK_SHADOW;
                    walking = true;
                } else {
                    sample_end = !cont;
                }
            }
            if (sample_end) {
                fresh = true;
                if (id < a.n_whole) {
                    V3 acc = v3(acc_l[0], acc_l[B], acc_l[2 * B]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[B] = acc.y; acc_l[2 * B] = acc.z;
                    if (++s == a.n_samples) {
                        double* o = sub_buf + (size_t)id * 3;
                        o[0] = acc.x;
                        o[1] = acc.y;
                        o[2] = acc.z;
                        if (++id < end) {  // the next subpixel of the run, no ticket
                            s = 0;
                            acc_l[0] = 0.0; acc_l[B] = 0.0; acc_l[2 * B] = 0.0;
                            nvalid = false;
                        } else {
                            done = true;
                        }
                    }
                } else if (tail_in_place(a, s)) {  // split tail, chunk 0: summed in place, its partial sum to sub_buf
                    V3 acc = v3(acc_l[0], acc_l[B], acc_l[2 * B]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[B] = acc.y; acc_l[2 * B] = acc.z;
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
            // the next ray, unless a shadow query is pending or the unit is done (a new ticket first)
            if (!walking && !done) {
                if (fresh) {
                    if (kCamBuf && nvalid) begin_path(sc, CameraSample{v3(nbd[0], nbd[B], nbd[2 * B]), nbr[0], nbr[B]}, ps);
                    else begin_sample(sc, a, subpixel_of(a, id), s, ps);
                    nvalid = false;
                    fresh = false;
                }
                RT_DBG_TSTART(t_ta);
                const RayInv wi = make_inv(ps.ray.d);
                const HitRec h = trace_analytic<C>(sc, ps.ray, wi);
                const uint32_t near = mesh_near_mask<C>(sc, ps.ray, wi, h.obj >= 0 ? h.t : INFINITY);
                RT_DBG_TEND(6, t_ta);
                if (near) {
                    RT_DBG(13);
#if RT_DEBUG_COUNTERS
                    if (after_s) RT_DBG(14);
#endif
                    park2_query(park, ps.ray, wi, h.t, h.obj, h.prim, near);
                    s_status[threadIdx.x] = POOL_CLOSEST;
                    phase = PH_WALK_CLOSEST;
                    walking = true;
                } else {
                    hh = h;  // shaded in the next iteration
                    has_hit = true;
                }
            }
          }
        } else {
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
                    if (!P && nvalid) begin_path(sc, CameraSample{v3(nbd[0], nbd[B], nbd[2 * B]), nbr[0], nbr[B]}, ps);
                    else begin_sample(sc, a, subpixel_of(a, id), s, ps);
                    nvalid = false;
                    fresh = false;
                }
                RT_DBG_TSTART(t_ta);
                const RayInv wi = make_inv(ps.ray.d);
                h = trace_analytic<C>(sc, ps.ray, wi);
                const uint32_t near = mesh_near_mask<C>(sc, ps.ray, wi, h.obj >= 0 ? h.t : INFINITY);
                const bool cand = near != 0;
                RT_DBG_TEND(6, t_ta);
                if (cand) {
                    if constexpr (P) park2_query(park, ps.ray, wi, h.t, h.obj, h.prim, near);
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
                RT_DBG_TSTART(t_sv);
                cont = shade_vertex<C>(sc, a, ps, h, &df);
                RT_DBG_TEND(8, t_sv);
                phase = PH_TRACE;
                if (df.pending) {  // shade_vertex found a mesh that could block the shadow ray
                    const Ray sr{df.o, df.d};
                    if constexpr (P) {
                        park2_query(park, sr, df.inv, df.dist, -1, -1, df.meshes);
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
                    V3 acc = v3(acc_l[0], acc_l[B], acc_l[2 * B]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[B] = acc.y; acc_l[2 * B] = acc.z;
                    if (++s == a.n_samples) {
                        double* o = sub_buf + (size_t)id * 3;
                        o[0] = acc.x;
                        o[1] = acc.y;
                        o[2] = acc.z;
                        if (++id < end) {  // the next subpixel of the run, no ticket
                            s = 0;
                            acc_l[0] = 0.0; acc_l[B] = 0.0; acc_l[2 * B] = 0.0;
                            nvalid = false;
                        } else {
                            done = true;
                        }
                    }
                } else if (tail_in_place(a, s)) {  // split tail, chunk 0: summed in place, its partial sum to sub_buf
                    V3 acc = v3(acc_l[0], acc_l[B], acc_l[2 * B]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[B] = acc.y; acc_l[2 * B] = acc.z;
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
                nbd[0] = nb.d.x; nbd[B] = nb.d.y; nbd[2 * B] = nb.d.z;
                nbr[0] = nb.r0; nbr[B] = nb.r1;
                nvalid = true;
            }
        }
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        flush_count_if_full(a.counters, nverts, done);
        if (done) {
            unit_of(a, nt, id, end, s);
            active = !stop && nt < nunits;
            acc_l[0] = 0.0; acc_l[B] = 0.0; acc_l[2 * B] = 0.0;
            fresh = true;
            nvalid = false;
        }
        RT_DBG_TEND(4, t_bk);
        RT_DBG_TEND(0, t_it);
#if RT_POOL_PRIO == 2
        __builtin_amdgcn_s_setprio(0);
#endif
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

// ---------------------------------------------------------------------------------------------------
// Role-split walk pool (P = 2, RT_MK_POOL=2): the block's waves are walkers or shaders, and paths are
// not owned by threads. A block holds RoleLayout::paths path slots in an LDS path store (SoA, RolePaths);
// a path is either in a shader lane's registers, queued (ready queue: to be shaded; walk queue: its
// closest or shadow query to be walked), or in a walker lane's registers while its query is walked.
//   shader waves: every idle lane takes any ready path (queue_take_each) and loads it; a lane shades
//     the hit its path holds, then traces the path's next ray (the same shade-then-trace order as the
//     walk pool, P = 1); a query that needs an octree walk parks the path in the store, queues it for
//     the walkers and frees the lane for the next ready path: vertex work runs on full waves instead of
//     the ~32 of 64 lanes whose own path is not walking (profiles/r05a_dbg_mesh.log).
//   walker waves: persistent walks (walk_step, one step per loop), each lane refilled from the walk
//     queue as its walk ends; the walk state never leaves registers (no park: a query is parked only
//     as its 68-B record before its first step), and a finished query's result goes into the store
//     (closest: the hit; shadow: the NEE term added to L unless a mesh blocks it) before the path is
//     queued as ready.
// Every path computes the same values in the same order as k_megakernel_f64 / the walk pool (the
// store keeps the doubles' bits), so frames are identical (tested).
#ifndef RT_ROLES_WALKERS
#define RT_ROLES_WALKERS 6  // walker waves of the block's 12
#endif
#ifndef RT_ROLES_REFILL
#define RT_ROLES_REFILL 16  // a walker wave refills once at least this many of its lanes are idle
#endif
#ifndef RT_ROLES_PRIO
#define RT_ROLES_PRIO 1  // walker waves at raised issue priority, this s_setprio level (their dependent loads issue first)
#endif
#ifndef RT_ROLES_BLOCK
#define RT_ROLES_BLOCK 768  // threads of a block (one per CU: the path store takes the LDS): 3 waves/SIMD (168 VGPRs);
                            // 512 threads (2 waves/SIMD) with 512 paths measured 17% slower (profiles/r05l_ab_b768.log)
#endif
// Path slots per block: as many as the LDS holds besides the queues, the walkers' ancestor columns and the
// object table (192 B each without MIS, 200 with). Throughput rises with the paths in flight (each waits
// ~14 walk steps per walk): 576 -> 632 slots +8.3% at 768 threads (profiles/r05l_ab_b768.log)
#if RT_DEBUG_COUNTERS || RT_DEBUG_TIMERS
#define RT_ROLES_DBG_LDS 16  // the diagnostic builds' per-block counters and timers take ~2.4 KB of LDS
#else
#define RT_ROLES_DBG_LDS 0
#endif
#ifndef RT_ROLES_PATHS
#define RT_ROLES_PATHS (784 - RT_ROLES_DBG_LDS)
#endif
#ifndef RT_ROLES_PATHS_MIS
#define RT_ROLES_PATHS_MIS (752 - RT_ROLES_DBG_LDS)
#endif
#ifndef RT_ANC16
#define RT_ANC16 1  // the walkers' ancestor columns hold 16-bit pids (scenes with more parents pop through pid_up)
#endif
using AncT = std::conditional_t<RT_ANC16 != 0, uint16_t, int32_t>;
// Block shape per instance: the Phong instances (the Phong BRDF's shading code: 32 spilled VGPRs at the
// 168 of 3 waves/SIMD) keep 512-thread blocks, 2 waves/SIMD, half of them walkers.
template <class C>
struct RoleShape {
    static constexpr int block = C::phong ? 512 : RT_ROLES_BLOCK;
    static constexpr int walkers = C::phong ? 4 : RT_ROLES_WALKERS;
    static constexpr int walk_threads = 64 * walkers;
    static_assert(walkers >= 1 && walkers < block / 64, "walkers and shaders both needed");
};
// doubles: ray o, d; beta; L; query: shadow direction, query t (closest: analytic hit t / result; shadow:
// distance; LdsQuerySink's fourth column), pending NEE term; pdf_prev (MIS only). (A slot's running sum
// over its unit's samples is kept in the unit's sub_buf entry, not here: role_sample_end.)
// The mirror state (bemit, o: RD_E, RD_C) shares the shadow query's columns: it is stored only when a
// mirror vertex has been shaded (ps.kind == K_SPEC: no NEE there, so no shadow query) and read back into
// registers when the path is loaded, before the next vertex's shading can write a shadow query.
enum : int {
    RD_O = 0, RD_D = 3, RD_B = 6, RD_L = 9, RD_QD = 12, RD_QT = 15, RD_PC = 16, RD_PDF = 19,
    RD_E = RD_QD, RD_C = RD_PC
};
static_assert(RD_QT == RD_QD + 3, "LdsQuerySink writes the distance after the direction");
template <class C>
struct RoleLayout {
    static constexpr int nd = C::mis ? RD_PDF + 1 : RD_PDF;  // doubles per path
    static constexpr int paths = C::mis ? RT_ROLES_PATHS_MIS : RT_ROLES_PATHS;
    static constexpr int ring = paths <= 256 ? 256 : paths <= 512 ? 512 : 1024;  // queue capacity (a power of two)
    static_assert(paths <= ring && ring <= 1024, "every path fits each queue once");
};
// ints: flags, unit id, sample, closest query's hit prim, near-mesh mask
enum : int { RI_FLAGS = 0, RI_ID = 1, RI_S = 2, RI_HPRIM = 3, RI_NEAR = 4, RI_N = 5 };
// RI_FLAGS: kind (2 bits), resume state << 2 (3 bits), closest query << 5, path continues << 6, the closest
// query's hit object + 1 << 7 (5 bits: compact scenes hold <= 16 objects), depth << 12
constexpr int kRfObj = 7, kRfDepth = 12;
static_assert(kMaxCompactObjects < 31, "a hit object id + 1 fits 5 bits");
RT_DEV int32_t rf_obj(int32_t obj) { return (obj + 1) << kRfObj; }
RT_DEV int32_t rf_get_obj(int flags) { return ((flags >> kRfObj) & 31) - 1; }
enum : int { RS_TRACE = 0, RS_SHADE = 1, RS_END = 2, RS_FRESH = 3 };
template <int NP>
struct RolePaths {
    static constexpr int np = NP;
    LdsDouble* d;  // [RoleLayout::nd][NP]
    LdsU64* u;     // [2][NP]: RNG state
    LdsInt* i;     // [RI_N][NP]
    RT_DEV LdsDouble& D(int f, int p) const { return d[f * NP + p]; }
    RT_DEV LdsU64& U(int f, int p) const { return u[f * NP + p]; }
    RT_DEV LdsInt& I(int f, int p) const { return i[f * NP + p]; }
    RT_DEV V3 D3(int f, int p) const { return v3(D(f, p), D(f + 1, p), D(f + 2, p)); }
    RT_DEV void set3(int f, int p, const V3& v) const { D(f, p) = v.x; D(f + 1, p) = v.y; D(f + 2, p) = v.z; }
};
// A shader lane's path in registers <-> the store. closest: the path parks for its closest query (the ray
// origin is stored, and the mirror state if the path is at a mirror bounce); otherwise for a shadow query,
// whose sink already wrote the origin x (the continuation's origin: the same bits when the path goes on)
// and whose direction and NEE term hold the mirror state's columns. (A path parked for a shadow query
// never needs the mirror state again: it continues from a diffuse vertex, or it has ended, in which case
// ps.kind can still read K_SPEC, the kind it entered that vertex with.)
template <class C, class RP>
RT_DEV void role_store(const RP& P, int p, const PathState& ps, int id, int s, int flags, bool closest) {
    if (closest) P.set3(RD_O, p, ps.ray.o);
    P.set3(RD_D, p, ps.ray.d);
    P.set3(RD_B, p, ps.beta);
    P.set3(RD_L, p, ps.L);
    if (!C::nospec && closest && ps.kind == K_SPEC) {
        P.set3(RD_E, p, ps.bemit);
        P.set3(RD_C, p, ps.o);
    }
    if (C::mis) P.D(RD_PDF, p) = ps.pdf_prev;
    P.U(0, p) = ps.r0;
    P.U(1, p) = ps.r1;
    P.I(RI_FLAGS, p) = flags | ps.kind | (int32_t)(ps.depth << kRfDepth);
    P.I(RI_ID, p) = id;
    P.I(RI_S, p) = s;
}
template <class C, class RP>
RT_DEV int role_load(const RP& P, int p, PathState& ps, int& id, int& s) {
    const int flags = P.I(RI_FLAGS, p);
    ps.kind = flags & 3;
    ps.ray = Ray{P.D3(RD_O, p), P.D3(RD_D, p)};
    ps.beta = P.D3(RD_B, p);
    ps.L = P.D3(RD_L, p);
    if (!C::nospec && ps.kind == K_SPEC) {
        ps.bemit = P.D3(RD_E, p);
        ps.o = P.D3(RD_C, p);
    }
    ps.pdf_prev = C::mis ? P.D(RD_PDF, p) : 0.0;
    ps.r0 = P.U(0, p);
    ps.r1 = P.U(1, p);
    ps.depth = (uint32_t)flags >> kRfDepth;
    id = P.I(RI_ID, p);
    s = P.I(RI_S, p);
    return flags;
}
// The path slot p's closest query stays in the store while it waits for a walker (record: the analytic
// hit so far and the near-mesh mask; the ray is the path's own; the hit object goes into the flags that
// role_store writes, rf_obj).
template <class RP>
RT_DEV void role_query_closest(const RP& P, int p, const HitRec& h, uint32_t near) {
    P.D(RD_QT, p) = h.t;
    P.I(RI_HPRIM, p) = h.prim;
    P.I(RI_NEAR, p) = (int32_t)near;
}

template <int F, int W, bool S, int B = RoleShape<Cfg<F>>::block>
__global__ __launch_bounds__(B, W) void k_megakernel_roles_f64(DevScene sc_g, RenderArgs a_g, double* __restrict__ sub_buf,
                                                                uint32_t* next_sub, long nsub) {
    using C = Cfg<F | (RT_OPT_LDSOBJ ? kCfgLdsObj : 0)>;
    static_assert(C::mesh && C::compact && !C::bvh, "the role-split pool walks octrees");
    static_assert(B % 64 == 0 && B <= 1024, "whole waves, at most 16 (path_f64.h: the diagnostic builds' per-wave LDS)");
#if RT_KARG_VIEW
    const DevScene& sc = karg_scene();
    const RenderArgs& a = karg_render_args();
#else
    const DevScene& sc = sc_g;
    const RenderArgs& a = a_g;
#endif
    if constexpr (C::ldsobj) lds_objects_fill(sc);
    using RL = RoleLayout<C>;
    constexpr int NP = RL::paths, kRing = RL::ring;
    __shared__ double s_pd[RL::nd * NP];
    __shared__ uint64_t s_pu[2 * NP];
    __shared__ int32_t s_pi[RI_N * NP];
    __shared__ int16_t s_ring[2][kRing];  // [0] ready paths, [1] queued walks (path ids < 1024)
    __shared__ uint32_t s_qhead[2][2], s_qtail[2][2];
    using RS = RoleShape<C>;
    static_assert(RS::block == B, "the launch's block shape");
    // walker lanes' ancestor columns: 16-bit pids (RT_ANC16) when the scene's pids fit, else the pid_up chain
    __shared__ AncT s_anc[S ? kSlotAncLevels * RS::walk_threads : 1];
    __shared__ uint32_t s_live;  // path slots still holding work (the block ends at 0)
    const RolePaths<NP> P{(LdsDouble*)s_pd, (LdsU64*)s_pu, (LdsInt*)s_pi};
    const LdsQueue16 rq{s_ring[0], s_qhead[0], s_qtail[0], (uint32_t)kRing - 1u};
    const LdsQueue16 wq{s_ring[1], s_qhead[1], s_qtail[1], (uint32_t)kRing - 1u};
    const long n_split = nsub - a.n_whole;
    const long nunits = a.n_wunits + n_split * a.tail_cps;
    // every path slot starts without a unit: queued as ready with RS_FRESH and id = -1 (a ticket first)
    for (int p = threadIdx.x; p < kRing; p += B) {
        if (p < NP) {
            P.I(RI_FLAGS, p) = RS_FRESH << 2;
            P.I(RI_ID, p) = -1;
        }
        s_ring[0][p] = p < NP ? p : -1;
        s_ring[1][p] = -1;
    }
    {
        const int p = threadIdx.x;
        if (p < 2) {
            s_qhead[p][0] = 0; s_qhead[p][1] = 0;
            s_qtail[p][0] = 0; s_qtail[p][1] = 0;
        }
        if (p == 0) {
            s_qtail[0][0] = NP;
            s_live = NP;
        }
    }
    __syncthreads();
    (void)s_qhead[0][1]; (void)s_qtail[0][1];
    uint32_t nverts = 0;
    RT_DBG_TINIT();
    const bool walker = (int)(threadIdx.x >> 6) < RS::walkers;
    if (walker) {
        // ---- walker wave ----
        using LdsAnc = __attribute__((address_space(3))) AncT;
        LdsAnc* anc = S && (!RT_ANC16 || sc.n_pid <= 0x10000) ? (LdsAnc*)s_anc + threadIdx.x : nullptr;
        int32_t q = -1;
        bool closest = false;
        WalkRegs r;
#if RT_ROLES_PRIO
        __builtin_amdgcn_s_setprio(RT_ROLES_PRIO);
#endif
        for (;;) {
            RT_DBG_TSTART(t_wi);
            const int idle = __popcll(__ballot(q < 0));
            if (idle >= RT_ROLES_REFILL || idle == 64) {
                RT_DBG_TSTART(t_tk);
                const int32_t q2 = queue_take_each(wq, q < 0);
                if (q2 >= 0) {
                    q = q2;
                    const int flags = P.I(RI_FLAGS, q);
                    closest = (flags >> 5) & 1;
                    r.wr.o = P.D3(RD_O, q);
                    r.wr.d = closest ? P.D3(RD_D, q) : P.D3(RD_QD, q);
                    r.wi = make_inv(r.wr.d);
                    r.wt = P.D(RD_QT, q);
                    r.hobj = closest ? rf_get_obj(flags) : -1;
                    r.hprim = closest ? P.I(RI_HPRIM, q) : -1;
                    r.g = -1;
                    r.w.cur = -1;
                    r.occluded = 0;
                }
                RT_DBG_TEND(5, t_tk);
                if (!__any(q >= 0)) {
                    RT_DBG_TEND(4, t_wi);
                    if (__hip_atomic_load(&s_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) break;
                    __builtin_amdgcn_s_sleep(2);
                    continue;
                }
            }
            RT_DBG_TSTART(t_wk);
            RT_DBG_WAVE(10, lane_id_is0());
            RT_DBG_WAVE(11, q >= 0);
            bool fin = false;
            if (q >= 0) {
                if (r.w.cur < 0) {  // begin the walk of the next candidate mesh (none left: done)
                    const double tmax = closest ? (r.hobj >= 0 ? r.wt : INFINITY) : r.wt;
                    RT_DBG_TSTART(t_bg);
                    fin = !next_mesh_walk_near<C, S>(sc, r.wr, r.wi, tmax, r.g, r.mi, r.w, (uint32_t)P.I(RI_NEAR, q));
                    RT_DBG_TEND(15, t_bg);
                }
                if (!fin && r.w.cur >= 0) {
                    double t;
                    int prim;
                    const int st = walk_step<S, RS::walk_threads, C::phong ? 0 : RT_WALK_HOIST>(sc, sc.meshes[r.mi], r.wr, r.wi,
                                                                                             r.w, &t, &prim, anc);
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
                        r.w.cur = -1;
                        fin |= r.g >= tables(sc)->last_mesh_g;  // no mesh left: the query's result is complete
                    }
                }
                if (fin) {  // the result into the store, then the path to the ready queue
                    const int flags = P.I(RI_FLAGS, q);
                    int rs;
                    int fl = flags & ~(7 << 2);
                    if (closest) {
                        P.D(RD_QT, q) = r.wt;
                        P.I(RI_HPRIM, q) = r.hprim;
                        fl = (fl & ~(31 << kRfObj)) | rf_obj(r.hobj);
                        rs = RS_SHADE;
                    } else {
                        if (!r.occluded) P.set3(RD_L, q, P.D3(RD_L, q) + P.D3(RD_PC, q));  // mutually_visible: the NEE term
                        rs = ((flags >> 6) & 1) ? RS_TRACE : RS_END;
                    }
                    P.I(RI_FLAGS, q) = fl | (rs << 2);
                }
            }
            RT_DBG_TEND(1, t_wk);
            queue_put(rq, fin, q);
            if (fin) q = -1;
            RT_DBG_TEND(4, t_wi);
        }
#if RT_ROLES_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
    } else {
        // ---- shader wave ----
        int32_t p = -1;
        PathState ps;
        int id = 0, s = 0, rs = RS_FRESH;
        bool cont = false;
        HitRec hh{0.0, -1, -1};
        for (;;) {
            RT_DBG_TSTART(t_it);
            RT_DBG_TSTART(t_tk);
            if (__any(p < 0)) {
                const int32_t q = queue_take_each(rq, p < 0);
                if (q >= 0) {
                    p = q;
                    const int flags = role_load<C>(P, p, ps, id, s);
                    rs = (flags >> 2) & 7;
                    cont = (flags >> 6) & 1;
                    if (rs == RS_SHADE) hh = HitRec{P.D(RD_QT, p), rf_get_obj(flags), P.I(RI_HPRIM, p)};
                }
            }
            RT_DBG_TEND(3, t_tk);
            if (!__any(p >= 0)) {
                RT_DBG_TEND(0, t_it);
                if (__hip_atomic_load(&s_live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) break;
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            RT_DBG_TSTART(t_vx);
            RT_DBG_WAVE(8, lane_id_is0());
            RT_DBG_WAVE(9, p >= 0);
            bool park = false, done = false;
            if (p >= 0) {
                bool sample_end = rs == RS_END;
                if (rs == RS_SHADE) {
                    nverts += hh.obj >= 0;
                    ShadowDefer df;
                    df.pending = false;
                    RT_DBG_TSTART(t_sv);
                    // a pending shadow query's origin, direction and distance go straight into the store
                    const LdsQuerySink sink{&P.D(RD_O, p), &P.D(RD_QD, p), NP};
                    cont = shade_vertex<C>(sc, a, ps, hh, &df, RegCold(), sink);
                    RT_DBG_TEND(8, t_sv);
                    if (df.pending) {  // a mesh could block the shadow ray: the walkers decide
                        RT_DBG(12);
                        P.set3(RD_PC, p, df.c);
                        P.I(RI_NEAR, p) = (int32_t)df.meshes;
                        role_store<C>(P, p, ps, id, s, (cont ? 1 << 6 : 0), false);
                        park = true;
                    } else if (!cont) {
                        sample_end = true;
                    } else {
                        rs = RS_TRACE;
                    }
                }
                if (sample_end) {
                    rs = RS_FRESH;
                    if (id < a.n_whole || tail_in_place(a, s)) {
                        // a whole subpixel, or the split tail's chunk 0: the running sum acc + L * inv_n from 0
                        // (server.rs:357-358) in the subpixel's sub_buf entry (the partial sum of chunk 0 is what
                        // k_tail_sum_f64 continues from)
                        double* o = sub_buf + (size_t)id * 3;
                        V3 acc = v3(0.0, 0.0, 0.0);
                        if (s != 0) acc = v3(o[0], o[1], o[2]);
                        acc = acc + ps.L * a.inv_n;
                        o[0] = acc.x;
                        o[1] = acc.y;
                        o[2] = acc.z;
                        if (id < a.n_whole) {
                            if (++s == a.n_samples) {
                                if (id + 1 < run_end(a, id)) {  // the next subpixel of the run, no ticket
                                    ++id;
                                    s = 0;
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
                if (rs == RS_FRESH && id < 0) done = true;  // a slot's first unit
            }
            // tickets: a path slot whose unit is done takes the next one; none left (or cancelled): it retires
            bool stop = false;
            if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
            const long nt = wave_ticket(next_sub, done && !stop);
            flush_count_if_full(a.counters, nverts, done);
            bool retire = false;
            if (done) {
                int end_unused;
                unit_of(a, nt, id, end_unused, s);
                retire = stop || nt >= nunits;
            }
            {
                const unsigned long long m = __ballot(retire);
                if (m && __lane_id() == __ffsll((long long)m) - 1)
                    __hip_atomic_fetch_sub(&s_live, (uint32_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (retire) p = -1;
            // the next ray: the path going on, or its unit's next sample
            if (p >= 0 && !park && (rs == RS_TRACE || rs == RS_FRESH)) {
                if (rs == RS_FRESH) begin_sample(sc, a, subpixel_of(a, id), s, ps);
                RT_DBG_TSTART(t_ta);
                const RayInv wi = make_inv(ps.ray.d);
                const HitRec h = trace_analytic<C>(sc, ps.ray, wi);
                const uint32_t near = mesh_near_mask<C>(sc, ps.ray, wi, h.obj >= 0 ? h.t : INFINITY);
                RT_DBG_TEND(6, t_ta);
                if (near) {
                    RT_DBG(13);
                    role_query_closest(P, p, h, near);
                    role_store<C>(P, p, ps, id, s, 1 << 5 | rf_obj(h.obj), true);
                    park = true;
                } else {
                    hh = h;  // shaded in the next iteration
                    rs = RS_SHADE;
                }
            }
            queue_put(wq, park, p);
            if (park) p = -1;
            RT_DBG_TEND(2, t_vx);
            RT_DBG_TEND(0, t_it);
        }
    }
    flush_count(a.counters, nverts);
    RT_DBG_TFLUSH();
}

template <int F, bool S = (RT_WALK_TIGHT != 0)>
static void launch_roles(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub, long nsub,
                         double* tail_buf, size_t tail_cap, hipStream_t st) {
    constexpr int B = RoleShape<Cfg<F>>::block, W = B / 256;  // one block per CU: B / 256 waves per SIMD
    const long blocks = resident_blocks(k_megakernel_roles_f64<F, W, S>, (nsub + B - 1) / B, B);
    RenderArgs a = a_in;
    // the split tail and ticket runs planned for the lanes that hold paths (one path slot per thread)
    // six subpixels per path slot; runs of whole subpixels of ~64 samples (plan_units)
    plan_tail(a, nsub, blocks * RoleLayout<Cfg<F>>::paths, tail_buf, tail_cap, 12, 1, 64);
    hipLaunchKernelGGL((k_megakernel_roles_f64<F, W, S>), dim3((unsigned)blocks), dim3(B), 0, st, sc, a, sub_buf, next_sub,
                       nsub);
    launch_tail_sum_f64(a, sub_buf, nsub - a.n_whole, st);
}

template <int F, int W, int P, bool S = (RT_WALK_TIGHT != 0)>
static void launch_mm(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub, long nsub,
                      int ksteps, int wmin, int refill, int pool_min, int pool_vmin, double* tail_buf, size_t tail_cap,
                      hipStream_t st) {
    constexpr int B = P ? kPoolThreads : 256;
    const long blocks = resident_blocks(k_megakernel_mesh_f64<F, W, P, S>, (nsub + B - 1) / B, B);
    RenderArgs a = a_in;
    plan_tail(a, nsub, blocks * B, tail_buf, tail_cap, 12, 1, 64);
    hipLaunchKernelGGL((k_megakernel_mesh_f64<F, W, P, S>), dim3((unsigned)blocks), dim3(B), 0, st, sc, a, sub_buf,
                       next_sub, nsub, ksteps, wmin, refill, pool_min, pool_vmin);
    launch_tail_sum_f64(a, sub_buf, nsub - a.n_whole, st);
}

// Octree walks through the role-split pool (RT_MK_POOL=2, default) or the walk pool (1), 2 waves/SIMD (the walk
// pool at 3 waves/SIMD: 37 spilled VGPRs, measured 6% slower; RT_MK_POOL=0: each lane walks its own query,
// RT_MK_KSTEPS steps per iteration).
// Scenes without slot tables (DevScene::node_slot null: node ids >= kSlotMaxNode) walk node_kids.
hipError_t launch_megakernel_mesh_f64(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                      long nsub, int refill, int wmin, double* tail_buf, size_t tail_cap, hipStream_t st) {
    static const int ksteps = std::max(1, env_int("RT_MK_KSTEPS", 4));
    // 2: the role-split pool (k_megakernel_roles_f64: unicorn 1920x1080x512 269.9 -> 310.6 Msamples/s,
    // profiles/r05c_ab_c4.log); 1: the round-4 walk pool (every wave walks and shades its own paths); 0: per-lane walks
    [[maybe_unused]] static const int pool = env_int("RT_MK_POOL", 2);
    static const int pool_min = env_int("RT_MK_POOL_MIN", 48);  // 48 with the 512-thread pool (32 before)
    static const int pool_ksteps = std::max(1, env_int("RT_MK_POOL_KSTEPS", 6));
    static const int pool_vmin = env_int("RT_MK_POOL_VMIN", 0);
    static const int pool_refill = env_int("RT_MK_POOL_CAM_REFILL", 20);  // the walk pool's camera refill threshold
    // Product builds: the role-split pool, or the walk pool over node_kids for an octree without slot tables. The
    // superseded slot-walk instances (the round-4 walk pool, RT_MK_POOL=1; per-lane walks, RT_MK_POOL=0) exist
    // only in A/B builds (ab_knobs.h).
#if RT_AB_KNOBS
#define RT_MM_AB(F)                                                                            \
        else if (pool == 1) launch_mm<F, 2, 1>(sc, a, sub_buf, next_sub, nsub, pool_ksteps, wmin, pool_refill, pool_min, pool_vmin, tail_buf, tail_cap, st); \
        else if (pool == 0) launch_mm<F, 2, 0>(sc, a, sub_buf, next_sub, nsub, ksteps, wmin, refill, 0, 0, tail_buf, tail_cap, st);
#else
#define RT_MM_AB(F)
#endif
#define RT_MM_CASE(F)                                                                          \
    case F:                                                                                    \
        if (!sc.node_slot) launch_mm<F, 2, 1, false>(sc, a, sub_buf, next_sub, nsub, pool_ksteps, wmin, pool_refill, pool_min, pool_vmin, tail_buf, tail_cap, st); \
        RT_MM_AB(F)                                                                            \
        else launch_roles<F>(sc, a, sub_buf, next_sub, nsub, tail_buf, tail_cap, st);          \
        break;
#define RT_MMB_CASE(F)                                                                         \
    case F:                                                                                    \
        launch_mm<F, 2, 0>(sc, a, sub_buf, next_sub, nsub, ksteps, wmin, refill, 0, 0, tail_buf, tail_cap, st); \
        break;
    switch (a.features & 31) {
        RT_MM_CASE(9) RT_MM_CASE(11) RT_MM_CASE(13) RT_MM_CASE(15)
        RT_MMB_CASE(25) RT_MMB_CASE(27) RT_MMB_CASE(29) RT_MMB_CASE(31)  // nearest-triangle meshes: BVH walks
        default: return hipErrorInvalidValue;
    }
#undef RT_MMB_CASE
#undef RT_MM_CASE
#undef RT_MM_AB
    return hipGetLastError();
}

#define RT_DIAG_TU_FN diag_read_mesh
#include "diag_tu.h"

}  // namespace rt
