// Streaming wavefront path tracer (f64) for gfx950.
//
// One bounce = two kernels over a dense SoA path stream (ping-pong A -> B):
//   k_wf_extend : Scene::trace_ray of every live path's ray (scene.rs:272-289) -> hit (t, obj, prim)
//   k_wf_shade  : emission, next-event estimation (shadow ray traced inline), Russian roulette and
//                 BSDF sampling (scene.rs:161-244); finished samples are added to their subpixel
//                 mean in sample order and immediately replaced by the subpixel's next sample, or
//                 by a fresh subpixel from a global work counter (regeneration). Survivors and
//                 regenerated paths are compacted into stream B: wave ballot -> popcount prefix ->
//                 one atomicAdd per wave, every lane writing its state at base + prefix.
// Scenes with meshes: extend traces the analytic objects and queues (Q1) the rays a mesh could
// still change; k_wf_mesh_closest traverses exactly those, in full waves, and merges with the
// reference's tie rule. Shade tests shadow rays against the analytic objects and queues (Q2) the
// ones a mesh could still block; k_wf_shadow_mesh adds their NEE term to the path if unblocked.
// Paths that end with a pending shadow stay in the stream one more bounce as K_DONE, so every
// path's radiance is summed in exactly the megakernel's order (bit-identical images).
// Streams never hold two live paths of one subpixel, so each subpixel's mean is a sequential sum
// in sample order (identical to server.rs:338-358) with no atomics on the accumulator.
// k_wf_finalize turns the 4 subpixel means of each pixel into RGB8 (server.rs:360-368).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../device/integrator_f64.h"
#include "wavefront.h"
#include "../ab_knobs.h"

namespace rt {
using namespace f64;

namespace {

constexpr int kBlock = 256;
constexpr int K_DONE = 3;  // path finished; waiting for a deferred shadow result

RT_DEV void store_state(const PathStream& S, long i, const PathState& ps, int sub, int smp, bool mis) {
    S.ox[i] = ps.ray.o.x; S.oy[i] = ps.ray.o.y; S.oz[i] = ps.ray.o.z;
    S.dx[i] = ps.ray.d.x; S.dy[i] = ps.ray.d.y; S.dz[i] = ps.ray.d.z;
    S.bx[i] = ps.beta.x; S.by[i] = ps.beta.y; S.bz[i] = ps.beta.z;
    S.lx[i] = ps.L.x; S.ly[i] = ps.L.y; S.lz[i] = ps.L.z;
    if (ps.kind == K_SPEC) {  // only a mirror bounce carries `o` and the emission weight forward
        S.ex[i] = ps.bemit.x; S.ey[i] = ps.bemit.y; S.ez[i] = ps.bemit.z;
        S.wx[i] = ps.o.x; S.wy[i] = ps.o.y; S.wz[i] = ps.o.z;
    }
    if (mis) S.pdf[i] = ps.pdf_prev;
    S.r0[i] = ps.r0;
    S.r1[i] = ps.r1;
    S.sub[i] = sub;
    S.sample[i] = smp;
    S.dk[i] = (int32_t)((ps.depth << 2) | (uint32_t)ps.kind);
}

RT_DEV void load_state(const PathStream& S, long i, PathState& ps, int* sub, int* smp, bool mis) {
    ps.ray.o = v3(S.ox[i], S.oy[i], S.oz[i]);
    ps.ray.d = v3(S.dx[i], S.dy[i], S.dz[i]);
    ps.beta = v3(S.bx[i], S.by[i], S.bz[i]);
    ps.L = v3(S.lx[i], S.ly[i], S.lz[i]);
    int32_t dk = S.dk[i];
    ps.kind = dk & 3;
    ps.depth = (uint32_t)dk >> 2;
    if (ps.kind == K_SPEC) {
        ps.bemit = v3(S.ex[i], S.ey[i], S.ez[i]);
        ps.o = v3(S.wx[i], S.wy[i], S.wz[i]);
    } else {
        ps.bemit = v3(0, 0, 0);
        ps.o = v3(0, 0, 0);
    }
    ps.pdf_prev = mis ? S.pdf[i] : 0.0;
    ps.r0 = S.r0[i];
    ps.r1 = S.r1[i];
    *sub = S.sub[i];
    *smp = S.sample[i];
}

// Wave-aggregated append: returns this lane's slot (valid only where pred).
RT_DEV long wave_append(uint32_t* counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m == 0ull) return -1;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    const unsigned long long below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
    return pred ? (long)base + __popcll(below) : -1;
}

__global__ __launch_bounds__(kBlock) void k_wf_init(DevScene sc, RenderArgs a, PathStream A, uint32_t* ctrl,
                                                     long nsub, long slots, double* sub_buf) {
    const long n0 = nsub < slots ? nsub : slots;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n0; i += stride) {
        SubPixel sp = subpixel_of(a, i);
        PathState ps;
        begin_sample(sc, a, sp, 0, ps);
        store_state(A, i, ps, (int)i, 0, a.mis != 0);
    }
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nsub * 3; i += stride) sub_buf[i] = 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctrl[0] = (uint32_t)n0;
        ctrl[1] = 0;
        ctrl[2] = (uint32_t)n0;  // next subpixel to hand out
        ctrl[4] = 0;
        ctrl[5] = 0;
        ctrl[6] = 0;
        ctrl[7] = 0;
    }
}

template <int F>
__global__ __launch_bounds__(kBlock) void k_wf_extend(DevScene sc, PathStream A, const uint32_t* cnt_in,
                                                       uint32_t* cnt_out, double* __restrict__ ht,
                                                       int32_t* __restrict__ hobj, int32_t* __restrict__ hprim,
                                                       int32_t* __restrict__ q1, uint32_t* q1_cnt, uint32_t* q2_cnt,
                                                       uint32_t* heads) {
    using C = Cfg<F>;
    constexpr bool kDefer = C::mesh && C::compact;
    const long n = (long)*cnt_in;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *cnt_out = 0;  // stream B is refilled by k_wf_shade
        *q2_cnt = 0;   // Q2 is refilled by k_wf_shade (the previous k_wf_shadow_mesh has drained it)
        heads[0] = 0;  // Q1 / Q2 read heads of the persistent traversal kernels
        heads[1] = 0;
    }
    const long stride = (long)gridDim.x * blockDim.x;
    for (long base = (long)blockIdx.x * blockDim.x; base < n; base += stride) {
        const long i = base + threadIdx.x;
        bool cand = false;
        if (i < n) {
            Ray r{v3(A.ox[i], A.oy[i], A.oz[i]), v3(A.dx[i], A.dy[i], A.dz[i])};
            if ((A.dk[i] & 3) == K_DONE) {
                hobj[i] = -2;
            } else if constexpr (kDefer) {
                const RayInv inv = make_inv(r.d);
                HitRec h = trace_analytic<C>(sc, r, inv);
                ht[i] = h.t;
                hobj[i] = h.obj;
                hprim[i] = h.prim;
                cand = mesh_candidate<C>(sc, r, inv, h.obj >= 0 ? h.t : INFINITY);
            } else {
                HitRec h = trace_closest<C>(sc, r);
                ht[i] = h.t;
                hobj[i] = h.obj;
                hprim[i] = h.prim;
            }
        }
        if constexpr (kDefer) {
            long pos = wave_append(q1_cnt, cand);
            if (cand) q1[pos] = (int32_t)i;
        }
    }
}

// Persistent traversal of a query queue. Octree walks are long-tailed (a wave of independent rays
// is busy as long as its longest walk: measured 4-6% lane utilisation with one query per lane), so
// each lane runs a resumable walk (walk_step) and the wave refills lanes whose query finished from
// the queue as soon as `refill` lanes are idle. One atomic per refill, per wave.
// Query protocol (Q: query state type):
//   start(qi, Q&) -> bool   load query qi; false if it needs no traversal (already finished)
//   next_mesh(Q&) -> bool   begin the walk on the query's next candidate mesh; false when none left
//   hit(Q&, t, prim) -> bool  a walk hit; true when the query is finished
//   finish(Q&)              write the query's result
template <class Q>
RT_DEV void persistent_walks(const DevScene& sc, uint32_t n, uint32_t* head, int refill, Q& q) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t lt = (1ull << lane) - 1ull;
    bool busy = false, drained = false;
    while (true) {
        const uint64_t idle = __ballot(!busy);
        const int nidle = __popcll(idle);
        if (!drained && (nidle >= refill || nidle == 64)) {
            const int leader = __ffsll((unsigned long long)idle) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(head, (uint32_t)nidle);
            base = __shfl(base, leader, 64);
            if (base + (uint32_t)nidle >= n) drained = true;
            if (!busy) {
                const uint32_t qi = base + (uint32_t)__popcll(idle & lt);
                if (qi < n && q.start(qi)) {
                    busy = q.next_mesh();
                    if (!busy) q.finish();
                }
            }
        }
        if (__ballot(busy) == 0) {
            if (drained) break;
            continue;
        }
        if (busy) {
            double t;
            int prim;
            const int st = walk_step<false>(sc, sc.meshes[q.mesh()], q.ray, q.inv, q.w, &t, &prim);
            if (st != WALK_RUN) {
                bool done = st == WALK_HIT && q.hit(t, prim);
                if (!done) done = !q.next_mesh();
                if (done) {
                    q.finish();
                    busy = false;
                }
            }
        }
    }
}

// Mesh part of trace_ray for the queued rays (Scene::trace_ray's loop over the mesh objects).
struct ClosestQuery {
    const DevScene& sc;
    const PathStream& A;
    const int32_t* q1;
    double* ht;
    int32_t* hobj;
    int32_t* hprim;
    long i;
    Ray ray;
    RayInv inv;
    HitRec h;
    int g;  // position in the gen_idx table of the mesh being walked
    OctWalk w;
    RT_DEV bool start(uint32_t qi) {
        i = q1[qi];
        ray = Ray{v3(A.ox[i], A.oy[i], A.oz[i]), v3(A.dx[i], A.dy[i], A.dz[i])};
        inv = make_inv(ray.d);
        h = HitRec{ht[i], hobj[i], hprim[i]};
        g = -1;
        return true;
    }
    RT_DEV int mesh() const { return sc.objects[tables(sc)->gen_idx[g]].mesh; }
    RT_DEV bool next_mesh() {
        for (++g; g < tables(sc)->n_gen; ++g) {
            const DevObject& o = sc.objects[tables(sc)->gen_idx[g]];
            if (o.geom == GEOM_MESH && walk_begin<false>(sc, sc.meshes[o.mesh], ray, inv, h.obj >= 0 ? h.t : INFINITY, w))
                return true;
        }
        return false;
    }
    RT_DEV bool hit(double t, int prim) {
        consider(h, t, tables(sc)->gen_idx[g], prim);
        return false;
    }
    RT_DEV void finish() {
        ht[i] = h.t;
        hobj[i] = h.obj;
        hprim[i] = h.prim;
    }
};

template <int F>
__global__ __launch_bounds__(kBlock) void k_wf_mesh_closest(DevScene sc, PathStream A, const int32_t* __restrict__ q1,
                                                            const uint32_t* q1_cnt, uint32_t* q1_head,
                                                            double* __restrict__ ht, int32_t* __restrict__ hobj,
                                                            int32_t* __restrict__ hprim, int refill) {
    ClosestQuery q{sc, A, q1, ht, hobj, hprim};
    persistent_walks(sc, *q1_cnt, q1_head, refill, q);
}

// Mesh part of mutually_visible for the queued shadow rays; unblocked ones add their NEE term.
struct ShadowQuery {
    const DevScene& sc;
    const PathStream& B;
    const int32_t* q2_pos;
    const double* q2;
    long slots;
    uint32_t qi;
    Ray ray;
    RayInv inv;
    double dist;
    bool occluded;
    int g;
    OctWalk w;
    RT_DEV bool start(uint32_t q) {
        qi = q;
        ray = Ray{v3(q2[q], q2[slots + q], q2[2 * slots + q]), v3(q2[3 * slots + q], q2[4 * slots + q], q2[5 * slots + q])};
        dist = q2[6 * slots + q];
        inv = make_inv(ray.d);
        occluded = false;
        g = -1;
        return true;
    }
    RT_DEV int mesh() const { return sc.objects[tables(sc)->gen_idx[g]].mesh; }
    RT_DEV bool next_mesh() {
        for (++g; g < tables(sc)->n_gen; ++g) {
            const DevObject& o = sc.objects[tables(sc)->gen_idx[g]];
            if (o.geom == GEOM_MESH && walk_begin<false>(sc, sc.meshes[o.mesh], ray, inv, dist, w)) return true;
        }
        return false;
    }
    RT_DEV bool hit(double t, int) {
        occluded = !(t + 0.001 >= dist);  // mesh_occludes / mutually_visible's ERR_MARGIN
        return occluded;
    }
    RT_DEV void finish() {
        if (occluded) return;
        const long p = q2_pos[qi];
        B.lx[p] = B.lx[p] + q2[7 * slots + qi];
        B.ly[p] = B.ly[p] + q2[8 * slots + qi];
        B.lz[p] = B.lz[p] + q2[9 * slots + qi];
    }
};

template <int F>
__global__ __launch_bounds__(kBlock) void k_wf_shadow_mesh(DevScene sc, PathStream B, const int32_t* __restrict__ q2_pos,
                                                           const double* __restrict__ q2, const uint32_t* q2_cnt,
                                                           uint32_t* q2_head, long slots, uint32_t* q1_cnt, int refill) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *q1_cnt = 0;  // Q1 is refilled by the next k_wf_extend
    ShadowQuery q{sc, B, q2_pos, q2, slots};
    persistent_walks(sc, *q2_cnt, q2_head, refill, q);
}

template <int F>
__global__ __launch_bounds__(kBlock) void k_wf_shade(DevScene sc, RenderArgs a, PathStream A, PathStream B,
                                                      const uint32_t* cnt_in, uint32_t* cnt_out, uint32_t* next_sub,
                                                      long nsub, const double* __restrict__ ht,
                                                      const int32_t* __restrict__ hobj,
                                                      const int32_t* __restrict__ hprim, double* sub_buf,
                                                      unsigned long long* counters, int32_t* __restrict__ q2_pos,
                                                      double* __restrict__ q2, uint32_t* q2_cnt, long slots) {
    using C = Cfg<F>;
    constexpr bool kDefer = C::mesh && C::compact;
    const long n = (long)*cnt_in;
    const long stride = (long)gridDim.x * blockDim.x;
    const bool mis = a.mis != 0;
    unsigned long long nverts = 0;
    // uniform trip count per wave: every lane reaches wave_append
    for (long base = (long)blockIdx.x * blockDim.x; base < n; base += stride) {
        const long i = base + threadIdx.x;
        const bool active = i < n;
        PathState ps;
        ShadowDefer sd;
        sd.pending = false;
        int sub = 0, smp = 0;
        bool emit = false;
        if (active) {
            load_state(A, i, ps, &sub, &smp, mis);
            SubPixel sp = subpixel_of(a, sub);
            bool finished;
            if (ps.kind == K_DONE) {
                finished = true;  // its deferred shadow has been resolved: fold it in now
            } else {
                HitRec hr{ht[i], hobj[i], hprim[i]};
                nverts += hr.obj >= 0;
                emit = shade_vertex<C>(sc, a, ps, hr, kDefer ? &sd : nullptr);
                finished = !emit;
                if (finished && sd.pending) {
                    ps.kind = K_DONE;  // keep the path one more bounce for its shadow result
                    emit = true;
                    finished = false;
                }
            }
            if (finished) {
                // sample finished: sequential mean update (server.rs:357-358), then regenerate
                double* acc = sub_buf + (size_t)sub * 3;
                acc[0] = acc[0] + ps.L.x * a.inv_n;
                acc[1] = acc[1] + ps.L.y * a.inv_n;
                acc[2] = acc[2] + ps.L.z * a.inv_n;
                ++smp;
                if (smp >= a.n_samples) {
                    long nxt = (long)atomicAdd(next_sub, 1u);
                    sub = (int)nxt;
                    smp = 0;
                    if (nxt < nsub) {
                        sp = subpixel_of(a, nxt);
                        begin_sample(sc, a, sp, 0, ps);
                        emit = true;
                    }
                } else {
                    begin_sample(sc, a, sp, smp, ps);
                    emit = true;
                }
            }
        }
        long pos = wave_append(cnt_out, emit);
        if (emit) store_state(B, pos, ps, sub, smp, mis);
        if constexpr (kDefer) {
            long qp = wave_append(q2_cnt, sd.pending);
            if (sd.pending) {
                q2_pos[qp] = (int32_t)pos;
                q2[qp] = sd.o.x;
                q2[slots + qp] = sd.o.y;
                q2[2 * slots + qp] = sd.o.z;
                q2[3 * slots + qp] = sd.d.x;
                q2[4 * slots + qp] = sd.d.y;
                q2[5 * slots + qp] = sd.d.z;
                q2[6 * slots + qp] = sd.dist;
                q2[7 * slots + qp] = sd.c.x;
                q2[8 * slots + qp] = sd.c.y;
                q2[9 * slots + qp] = sd.c.z;
            }
        }
    }
    if (counters) {
        unsigned long long v = nverts;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(counters, v);
    }
}

// A/B overrides of the stream shape (ab_knobs.h: -DRT_AB_KNOBS=1 builds only)
size_t env_size(const char* name, size_t dflt) {
    const long x = ab_knob(name, (long)dflt);
    return x > 0 ? (size_t)x : dflt;
}

// Persistent traversal grid: as many blocks as are resident at once.
template <class K>
unsigned resident_grid(K kernel) {
    int dev = 0, ncu = 256, nb = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
    return (unsigned)(ncu * nb);
}

template <int F>
void launch_bounce_t(dim3 g, hipStream_t st, const DevScene& sc, const RenderArgs& a, Workspace& ws, int cur, int nxt,
                     long nsub, double* sub_buf, unsigned long long* counters) {
    constexpr bool kDefer = Cfg<F>::mesh && Cfg<F>::compact;
    static const unsigned g_closest = kDefer ? resident_grid(k_wf_mesh_closest<F>) : 1;
    static const unsigned g_shadow = kDefer ? resident_grid(k_wf_shadow_mesh<F>) : 1;
    static const int refill = (int)std::min<size_t>(64, std::max<size_t>(1, env_size("RT_WF_REFILL", 16)));
    hipLaunchKernelGGL(k_wf_extend<F>, g, dim3(kBlock), 0, st, sc, ws.s[cur], ws.ctrl + cur, ws.ctrl + nxt, ws.hit_t,
                       ws.hit_obj, ws.hit_prim, ws.q1, ws.ctrl + 4, ws.ctrl + 5, ws.ctrl + 6);
    if (kDefer)
        hipLaunchKernelGGL(k_wf_mesh_closest<F>, dim3(g_closest), dim3(kBlock), 0, st, sc, ws.s[cur],
                           (const int32_t*)ws.q1, (const uint32_t*)(ws.ctrl + 4), ws.ctrl + 6, ws.hit_t, ws.hit_obj,
                           ws.hit_prim, refill);
    hipLaunchKernelGGL(k_wf_shade<F>, g, dim3(kBlock), 0, st, sc, a, ws.s[cur], ws.s[nxt], ws.ctrl + cur,
                       ws.ctrl + nxt, ws.ctrl + 2, nsub, ws.hit_t, ws.hit_obj, ws.hit_prim, sub_buf, counters,
                       ws.q2_pos, ws.q2, ws.ctrl + 5, (long)ws.slots);
    if (kDefer)
        hipLaunchKernelGGL(k_wf_shadow_mesh<F>, dim3(g_shadow), dim3(kBlock), 0, st, sc, ws.s[nxt],
                           (const int32_t*)ws.q2_pos, (const double*)ws.q2, (const uint32_t*)(ws.ctrl + 5),
                           ws.ctrl + 7, (long)ws.slots, ws.ctrl + 4, refill);
}

void launch_bounce(int features, dim3 g, hipStream_t st, const DevScene& sc, const RenderArgs& a, Workspace& ws,
                   int cur, int nxt, long nsub, double* sub_buf, unsigned long long* counters) {
#define RT_WF_CASE(F) \
    case F: launch_bounce_t<F>(g, st, sc, a, ws, cur, nxt, nsub, sub_buf, counters); break;
    switch (features & 15) {
        RT_WF_CASE(0) RT_WF_CASE(1) RT_WF_CASE(2) RT_WF_CASE(3) RT_WF_CASE(4) RT_WF_CASE(5) RT_WF_CASE(6)
        RT_WF_CASE(7) RT_WF_CASE(8) RT_WF_CASE(9) RT_WF_CASE(10) RT_WF_CASE(11) RT_WF_CASE(12) RT_WF_CASE(13)
        RT_WF_CASE(14) RT_WF_CASE(15)
    }
#undef RT_WF_CASE
}

}  // namespace

hipError_t Workspace::ensure_counters() {
    if (counters) return hipSuccess;
    hipError_t e = hipMalloc(&counters, 64);
    if (e != hipSuccess) counters = nullptr;
    return e;
}

hipError_t Workspace::ensure_sub(size_t pixels) {
    if (sub_cap >= pixels) return hipSuccess;
    if (in_flight && busy) (void)hipEventSynchronize(busy);  // a reused workspace: its last render is done with it
    if (sub_buf) (void)hipFree(sub_buf);
    sub_buf = nullptr;
    sub_cap = 0;
    hipError_t e = hipMalloc(&sub_buf, pixels * 12 * sizeof(double));
    if (e == hipSuccess) sub_cap = pixels;
    return e;
}

hipError_t Workspace::ensure_tail(size_t bytes) {
    if (tail_cap >= bytes) return hipSuccess;
    if (in_flight && busy) (void)hipEventSynchronize(busy);  // a reused workspace: its last render is done with it
    if (tail_buf) (void)hipFree(tail_buf);
    tail_buf = nullptr;
    tail_cap = 0;
    hipError_t e = hipMalloc(&tail_buf, bytes);
    if (e == hipSuccess) tail_cap = bytes;
    return e;
}

hipError_t Workspace::ensure_slots(size_t n) {
    hipError_t e;
    if (!ctrl) {
        e = hipMalloc(&ctrl, 64);
        if (e != hipSuccess) return e;
        e = hipHostMalloc((void**)&host_ctrl, 64, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    if (slots >= n) return hipSuccess;
    if (in_flight && busy) (void)hipEventSynchronize(busy);
    if (blob) (void)hipFree(blob);
    blob = nullptr;
    slots = 0;
    // per stream: 19 f64 arrays + 2 u64 + 3 i32 arrays; hit: f64 + 2 i32
    const size_t per_stream = n * (21 * sizeof(double) + 3 * sizeof(int32_t));
    const size_t hits = n * (sizeof(double) + 2 * sizeof(int32_t));
    const size_t queues = n * (2 * sizeof(int32_t) + 10 * sizeof(double));
    const size_t pad = 64 * 1024;
    e = hipMalloc(&blob, 2 * per_stream + hits + queues + pad);
    if (e != hipSuccess) { blob = nullptr; return e; }
    char* p = (char*)blob;
    auto take = [&](size_t bytes) {
        char* r = p;
        p += (bytes + 255) / 256 * 256;
        return r;
    };
    for (int k = 0; k < 2; ++k) {
        PathStream& S = s[k];
        double** f[] = {&S.ox, &S.oy, &S.oz, &S.dx, &S.dy, &S.dz, &S.bx, &S.by, &S.bz, &S.lx,
                        &S.ly, &S.lz, &S.ex, &S.ey, &S.ez, &S.wx, &S.wy, &S.wz, &S.pdf};
        for (double** q : f) *q = (double*)take(n * sizeof(double));
        S.r0 = (uint64_t*)take(n * sizeof(uint64_t));
        S.r1 = (uint64_t*)take(n * sizeof(uint64_t));
        S.sub = (int32_t*)take(n * sizeof(int32_t));
        S.sample = (int32_t*)take(n * sizeof(int32_t));
        S.dk = (int32_t*)take(n * sizeof(int32_t));
    }
    hit_t = (double*)take(n * sizeof(double));
    hit_obj = (int32_t*)take(n * sizeof(int32_t));
    hit_prim = (int32_t*)take(n * sizeof(int32_t));
    q1 = (int32_t*)take(n * sizeof(int32_t));
    q2_pos = (int32_t*)take(n * sizeof(int32_t));
    q2 = (double*)take(10 * n * sizeof(double));
    slots = n;
    return hipSuccess;
}

Workspace::~Workspace() {
    if (counters) (void)hipFree(counters);
    if (blob) (void)hipFree(blob);
    if (ctrl) (void)hipFree(ctrl);
    if (sub_buf) (void)hipFree(sub_buf);
    if (tail_buf) (void)hipFree(tail_buf);
    if (host_ctrl) (void)hipHostFree(host_ctrl);
    if (ev) (void)hipEventDestroy(ev);
    if (busy) (void)hipEventDestroy(busy);
}

int wavefront_render_f64(const DevScene& sc, const RenderArgs& a_in, Workspace& ws, hipStream_t st,
                         const volatile int32_t* cancel, rt_render_stats* stats, std::string* err) {
    RenderArgs a = a_in;
    const long npix = (long)a.tw * a.th;
    if (npix == 0) return RT_OK;
    auto hip_fail = [&](hipError_t e, const char* what) {
        *err = std::string(what) + ": " + hipGetErrorString(e);
        return e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP;
    };
    hipError_t e;
    double* sub_buf = a.sub_out;
    if (!sub_buf) {
        if ((e = ws.ensure_sub((size_t)npix)) != hipSuccess) return hip_fail(e, "subpixel buffer");
        sub_buf = ws.sub_buf;
    }
    if ((e = ws.ensure_counters()) != hipSuccess) return hip_fail(e, "counters");
    if (stats && (e = hipMemsetAsync(ws.counters, 0, 64, st)) != hipSuccess) return hip_fail(e, "counters");
    const long nsub = npix * 4;
    const size_t slots = std::min<size_t>((size_t)nsub, env_size("RT_WF_SLOTS", (size_t)1 << 21));
    if ((e = ws.ensure_slots(slots)) != hipSuccess) return hip_fail(e, "path streams");

    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const long grid_cap = (long)ncu * (long)env_size("RT_WF_BLOCKS_PER_CU", 8);
    const long grid = std::max<long>(1, std::min<long>(grid_cap, ((long)slots + kBlock - 1) / kBlock));
    const int batch = (int)env_size("RT_WF_BATCH", 16);

    int64_t iters = 0;
    if (a.n_samples > 0) {
        hipLaunchKernelGGL(k_wf_init, dim3((unsigned)grid), dim3(kBlock), 0, st, sc, a, ws.s[0], ws.ctrl, nsub,
                           (long)slots, sub_buf);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "k_wf_init");
        int cur = 0;
        bool pending = false;
        while (true) {
            for (int k = 0; k < batch; ++k) {
                const int nxt = cur ^ 1;
                launch_bounce(a.features, dim3((unsigned)grid), st, sc, a, ws, cur, nxt, nsub, sub_buf,
                              stats ? ws.counters : nullptr);
                cur = nxt;
                ++iters;
            }
            if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "wavefront launch");
            // Termination check one batch behind: read the live count written by the previous
            // batch while this batch runs.
            if (pending) {
                if ((e = hipEventSynchronize(ws.ev)) != hipSuccess) return hip_fail(e, "wavefront sync");
                if (ws.host_ctrl[0] == 0 && ws.host_ctrl[1] == 0) break;
            }
            // safety net: RR (p = 0.9 past depth 5) makes 10^5 bounces per sample unreachable
            if (iters > (int64_t)a.n_samples * 4 * 100000 + 1000000) {
                *err = "wavefront did not drain (iteration cap reached)";
                return RT_E_HIP;
            }
            if (cancel && *cancel) {
                (void)hipStreamSynchronize(st);
                return RT_CANCELLED;
            }
            if ((e = hipMemcpyAsync(ws.host_ctrl, ws.ctrl, 16, hipMemcpyDeviceToHost, st)) != hipSuccess)
                return hip_fail(e, "ctrl readback");
            if ((e = hipEventRecord(ws.ev, st)) != hipSuccess) return hip_fail(e, "event");
            pending = true;
        }
    }
    if (a.n_samples <= 0) {
        if ((e = hipMemsetAsync(sub_buf, 0, (size_t)npix * 12 * sizeof(double), st)) != hipSuccess)
            return hip_fail(e, "memset");
    }
    if ((e = launch_finalize_f64(a, sub_buf, st)) != hipSuccess) return hip_fail(e, "finalize");
    if (stats) {
        unsigned long long c[1] = {0};
        if ((e = hipMemcpyAsync(c, ws.counters, sizeof c, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_fail(e, "stats");
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return hip_fail(e, "stats sync");
        stats->vertices = (int64_t)c[0];
        stats->iterations = iters;
        stats->kernel_launches[0] = iters;
        stats->kernel_launches[1] = iters;
    }
    return RT_OK;
}

}  // namespace rt
