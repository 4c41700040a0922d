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

namespace rt {
using namespace f64;

// Wave-aggregated ticket: every lane with `want` gets the next value of *counter (one atomic per
// wave). All 64 lanes must call it together.
__device__ __forceinline__ long wave_ticket(uint32_t* counter, bool want) {
    const unsigned long long m = __ballot(want);
    if (m == 0ull) return -1;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    const unsigned long long below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
    return want ? (long)base + __popcll(below) : -1;
}

// Adds the wave's vertex counts to *counter and zeroes them. All 64 lanes must call it together.
__device__ __forceinline__ void flush_count(unsigned long long* counter, uint32_t& n) {
    if (!counter) return;
    unsigned long long v = n;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (__lane_id() == 0 && v) atomicAdd(counter, v);
    n = 0;
}

// Persistent megakernel: a resident grid whose lanes pull subpixels from a global counter. A lane
// walks the spp/4 sample paths of its subpixel vertex by vertex; when a path ends, the next sample
// starts in the same iteration (regeneration); when the subpixel is done its mean goes to
// sub_buf (sequential sum in sample order, server.rs:338-358) and the lane takes the next
// subpixel. Waves idle only in the frame's final tail, not per wave.
// W = minimum waves per SIMD requested from the register allocator.
template <int F, int W>
__global__ __launch_bounds__(256, W) void k_megakernel_f64(DevScene sc, RenderArgs a, double* __restrict__ sub_buf,
                                                          uint32_t* next_sub, long nsub) {
    using C = Cfg<F>;
    uint32_t nverts = 0;
    long id = wave_ticket(next_sub, true);
    bool active = id < nsub;
    V3 acc = v3(0, 0, 0);
    int s = 0;
    PathState ps;
    bool fresh = true;
    while (__any(active)) {
        bool done = false;
        if (active) {
            if (fresh) begin_sample(sc, a, subpixel_of(a, id), s, ps);
            HitRec hr = trace_closest<C>(sc, ps.ray);
            nverts += hr.obj >= 0;
            fresh = !shade_vertex<C>(sc, a, ps, hr);
            if (fresh) {
                acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                if (++s == a.n_samples) {
                    double* o = sub_buf + (size_t)id * 3;
                    o[0] = acc.x;
                    o[1] = acc.y;
                    o[2] = acc.z;
                    done = true;
                }
            }
        }
        // cancellation (RenderJob::stop, server.rs:201-203): checked when a lane would start a new
        // subpixel; a set flag stops handing out work, lanes finish the subpixel they hold
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        long nid = wave_ticket(next_sub, done && !stop);
        if (__any(done)) flush_count(a.counters, nverts);  // keeps the 32-bit lane counts far from overflow
        if (done) {
            id = stop ? nsub : nid;
            active = id < nsub;
            acc = v3(0, 0, 0);
            s = 0;
            fresh = true;
        }
    }
    flush_count(a.counters, nverts);
}

__device__ __forceinline__ bool lane_id_is0() { return __lane_id() == 0; }

// Begins the octree walk of the next candidate mesh after gen slot g (Scene::trace_ray's /
// mutually_visible's loop over the mesh objects); false when no mesh is left.
template <class C>
RT_DEV bool next_mesh_walk(const DevScene& sc, const Ray& r, const RayInv& inv, double tmax, int& g, int& mi,
                           OctWalk& w) {
    for (++g; g < tables(sc)->n_gen; ++g) {
        const DevObject& o = sc.objects[tables(sc)->gen_idx[g]];
        if (o.geom == GEOM_MESH && walk_begin(sc, sc.meshes[o.mesh], r, inv, tmax, w)) {
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
template <int F, int W>
__global__ __launch_bounds__(256, W) void k_megakernel_mesh_f64(DevScene sc, RenderArgs a, double* __restrict__ sub_buf,
                                                               uint32_t* next_sub, long nsub, int ksteps) {
    using C = Cfg<F>;
    static_assert(C::mesh && C::compact, "mesh megakernel needs the compact tables");
    uint32_t nverts = 0;
    long id = wave_ticket(next_sub, true);
    bool active = id < nsub;
    V3 acc = v3(0, 0, 0);
    int s = 0;
    PathState ps;
    bool fresh = true;
    // walk state: the walked ray (ps.ray for a closest query, the shadow ray for a shadow query)
    int phase = PH_TRACE;
    bool walking = false, occluded = false, cont = false;
    Ray wr;
    RayInv wi;
    double wdist = 0.0;         // shadow: |y - x|
    HitRec h{0.0, -1, -1};      // closest: analytic hit merged with the finished mesh walks
    V3 wc = v3(0, 0, 0);        // shadow: the pending NEE term (already weighted by beta)
    int g = -1, mi = 0;         // gen slot and mesh being walked
    OctWalk w;
    while (__any(active)) {
        RT_DBG_WAVE(8, lane_id_is0());
        for (int k = 0; k < ksteps && __any(walking); ++k) {
            RT_DBG_WAVE(10, lane_id_is0());
            RT_DBG_WAVE(11, walking);
            if (walking) {
                double t;
                int prim;
                const int st = walk_step(sc, sc.meshes[mi], wr, wi, w, &t, &prim);
                if (st != WALK_RUN) {
                    bool fin;
                    if (phase == PH_WALK_CLOSEST) {
                        if (st == WALK_HIT) consider(h, t, tables(sc)->gen_idx[g], prim);
                        fin = !next_mesh_walk<C>(sc, wr, wi, h.obj >= 0 ? h.t : INFINITY, g, mi, w);
                    } else {
                        occluded = st == WALK_HIT && !(t + 0.001 >= wdist);  // mutually_visible's ERR_MARGIN
                        fin = occluded || !next_mesh_walk<C>(sc, wr, wi, wdist, g, mi, w);
                    }
                    walking = !fin;
                }
            }
        }
        bool done = false;
        RT_DBG_WAVE(9, active && !walking);
        if (active && !walking) {
            bool shade_now = false, sample_end = false;
            if (phase == PH_WALK_SHADOW) {
                if (!occluded) ps.L = ps.L + wc;
                phase = PH_TRACE;
                sample_end = !cont;
            } else if (phase == PH_WALK_CLOSEST) {
                shade_now = true;
            } else {
                if (fresh) {
                    begin_sample(sc, a, subpixel_of(a, id), s, ps);
                    fresh = false;
                }
                wr = ps.ray;
                wi = make_inv(wr.d);
                h = trace_analytic<C>(sc, wr, wi);
                g = -1;
                if (next_mesh_walk<C>(sc, wr, wi, h.obj >= 0 ? h.t : INFINITY, g, mi, w)) {
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
                if (df.pending) {
                    wr = Ray{df.o, df.d};
                    wi = make_inv(wr.d);
                    wdist = df.dist;
                    wc = df.c;
                    g = -1;
                    occluded = false;
                    if (next_mesh_walk<C>(sc, wr, wi, wdist, g, mi, w)) {
                        phase = PH_WALK_SHADOW;
                        walking = true;
                    } else {
                        ps.L = ps.L + wc;
                    }
                }
                if (!walking) sample_end = !cont;
            }
            if (sample_end) {
                acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                fresh = true;
                if (++s == a.n_samples) {
                    double* o = sub_buf + (size_t)id * 3;
                    o[0] = acc.x;
                    o[1] = acc.y;
                    o[2] = acc.z;
                    done = true;
                }
            }
        }
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        long nid = wave_ticket(next_sub, done && !stop);
        if (__any(done)) flush_count(a.counters, nverts);  // keeps the 32-bit lane counts far from overflow
        if (done) {
            id = stop ? nsub : nid;
            active = id < nsub;
            acc = v3(0, 0, 0);
            s = 0;
            fresh = true;
        }
    }
    flush_count(a.counters, nverts);
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
                                                   double* pos, double* nrm) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r{v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2])};
    HitRec h = sc.compact ? trace_closest<Cfg<9>>(sc, r) : trace_closest<Cfg<1>>(sc, r);
    obj[i] = h.obj;
    t[i] = h.obj >= 0 ? h.t : 0.0;
    if (h.obj >= 0) {
        V3 p, nn;
        surface<Cfg<1>>(sc, r, h, &p, &nn);
        pos[3 * i] = p.x; pos[3 * i + 1] = p.y; pos[3 * i + 2] = p.z;
        nrm[3 * i] = nn.x; nrm[3 * i + 1] = nn.y; nrm[3 * i + 2] = nn.z;
    }
}

// Resident grid of a persistent kernel: as many 256-thread blocks as fit on the device at once.
template <class K>
static long resident_blocks(K kernel, long want) {
    int dev = 0, ncu = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    return std::max(1L, std::min((long)ncu * per_cu, want));
}

static int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

template <int F, int W>
static void launch_mk(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                      hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_f64<F, W>, (nsub + 255) / 256);
    hipLaunchKernelGGL((k_megakernel_f64<F, W>), dim3((unsigned)blocks), dim3(256), 0, st, sc, a, sub_buf, next_sub, nsub);
}
template <int F, int W>
static void launch_mm(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                      int ksteps, hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_mesh_f64<F, W>, (nsub + 255) / 256);
    hipLaunchKernelGGL((k_megakernel_mesh_f64<F, W>), dim3((unsigned)blocks), dim3(256), 0, st, sc, a, sub_buf, next_sub,
                       nsub, ksteps);
}

hipError_t launch_megakernel_f64(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                 hipStream_t st) {
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
    // walks, RT_MK_KSTEPS walk steps per vertex iteration, RT_MK_MESH_WAVES waves/SIMD (0 selects the
    // fused per-vertex traversal for A/B runs). Shallow octrees (cubes: 9 nodes) walk in a few
    // steps: the fused traversal is faster there (profiles/r01_interleave_ab.log).
    static const int interleave = env_int("RT_MK_INTERLEAVE", 64);
    static const int ksteps = std::max(1, env_int("RT_MK_KSTEPS", 8));
    static const int mwaves = env_int("RT_MK_MESH_WAVES", 2);
    if (interleave && (a.features & 9) == 9 && a.mesh_nodes >= interleave) {
#define RT_MM_CASE(F)                                                                    \
    case F:                                                                              \
        if (mwaves == 4) launch_mm<F, 4>(sc, a, sub_buf, next_sub, nsub, ksteps, st);    \
        else launch_mm<F, 2>(sc, a, sub_buf, next_sub, nsub, ksteps, st);                \
        break;
        switch (a.features & 15) { RT_MM_CASE(9) RT_MM_CASE(11) RT_MM_CASE(13) RT_MM_CASE(15) }
#undef RT_MM_CASE
        return hipGetLastError();
    }
#define RT_MK_CASE(F)                                                           \
    case F:                                                                     \
        if (waves == 3) launch_mk<F, 3>(sc, a, sub_buf, next_sub, nsub, st);    \
        else launch_mk<F, 4>(sc, a, sub_buf, next_sub, nsub, st);               \
        break;
    switch (a.features & 15) {
        RT_MK_CASE(0) RT_MK_CASE(1) RT_MK_CASE(2) RT_MK_CASE(3) RT_MK_CASE(4) RT_MK_CASE(5) RT_MK_CASE(6)
        RT_MK_CASE(7) RT_MK_CASE(8) RT_MK_CASE(9) RT_MK_CASE(10) RT_MK_CASE(11) RT_MK_CASE(12) RT_MK_CASE(13)
        RT_MK_CASE(14) RT_MK_CASE(15)
    }
#undef RT_MK_CASE
    return hipGetLastError();
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
                            double* pos, double* nrm, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_trace_f64, dim3((unsigned)blocks), dim3(256), 0, st, sc, n, o, d, t, obj, pos, nrm);
    return hipGetLastError();
}

}  // namespace rt
