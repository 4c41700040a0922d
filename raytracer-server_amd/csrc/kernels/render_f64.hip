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
#ifndef RT_MK_BEGIN_AT_END
#define RT_MK_BEGIN_AT_END 1  // a lane whose sample ended starts its next buffered sample in the same divergent block
#endif                        // (0: at the top of the next iteration, a block of its own; cornell 1024 spp 2000.6 ->
                              // 2002.9, C2 MIS 1891.0 -> 1896.6, same frames: profiles/r06be_ab_begin_at_end.log)
#ifndef RT_MK_MIN_RUN
#define RT_MK_MIN_RUN 32  // samples per ticket at least, while the frame holds more than one run per lane (plan_units;
#endif                     // 1080p at 64 spp: 16 -> 1567.5, 24 / 32 -> 1804-1808, 64 -> 1744.9, 128 -> 1664.9 Msamples/s,
                           // profiles/r06br_ab_min_run_long.log, r06bs_ab_min_run_short.log)
#ifndef RT_OPT_COLD
#define RT_OPT_COLD 1  // A/B: mirror-bounce state (o, pre-bounce throughput) in LDS (LdsCold) or registers
#endif

// Diagnostic builds (RT_DEBUG_TIMERS): each wave of k_megakernel_f64 records, on the constant 100 MHz clock
// (s_memrealtime), when it started, when fewer than half of its lanes last held work (-1: never), and when it
// ended (rt_debug_wave_times, tools/end_probe.py --waves): the end phase of a launch, wave by wave.
#if RT_DEBUG_TIMERS
constexpr int kDbgWaves = 8192;
constexpr int kDbgWaveRec = 5;
__device__ unsigned long long g_dbg_wave[kDbgWaveRec * kDbgWaves];
#endif

template <int F, int W>
__global__ __launch_bounds__(256, W) void k_megakernel_f64(DevScene sc_g, RenderArgs a_g, double* __restrict__ sub_buf,
                                                          uint32_t* next_sub, long nsub, int refill) {
    // Compact scenes (<= kMaxCompactObjects objects): the object table is copied into LDS, so the
    // shading's per-lane object reads (hit object, light) are ds_reads instead of global loads.
    using C = Cfg<F | ((RT_OPT_LDSOBJ && (F & 8)) ? kCfgLdsObj : 0)>;
#if RT_KARG_VIEW
    const DevScene& sc = karg_scene();  // the arguments read in place (megakernel_common.h)
    const RenderArgs& a = karg_render_args();
#else
    const DevScene& sc = sc_g;
    const RenderArgs& a = a_g;
#endif
    if constexpr (C::ldsobj) lds_objects_fill(sc);
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
#if RT_DEBUG_TIMERS
    const unsigned long long w_t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long w_half = ~0ull;
    // per lane: when it took the unit it holds (l_take, l_unit) and when it ran out of work (l_end)
    unsigned long long l_take = w_t0, l_end = w_t0;
    long l_unit = t0;
#endif
    while (__any(active)) {
#if RT_DEBUG_TIMERS
        if (w_half == ~0ull && __popcll(__ballot(active)) < 32) w_half = __builtin_amdgcn_s_memrealtime();
#endif
        RT_DBG_REGION(0);
        RT_DBG_TSTART(t_it);
        bool done = false;
        // camera: a lane starting a path takes its next buffered sample, or joins the camera pass
        RT_DBG_TSTART(t_fr);
        if (!RT_MK_BEGIN_AT_END && active && fresh && nbuf > 0) {
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
                } else if (tail_in_place(a, s)) {  // split tail, chunk 0: summed in place, its partial sum to sub_buf
                    V3 acc = v3(acc_l[0], acc_l[256], acc_l[2 * 256]);
                    acc = acc + ps.L * a.inv_n;  // server.rs:357-358
                    acc_l[0] = acc.x; acc_l[256] = acc.y; acc_l[2 * 256] = acc.z;
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
#if RT_MK_BEGIN_AT_END
                // the next sample of the same unit from the camera buffer, here rather than in a block of its own
                // at the top of the next iteration (same lanes; the camera pass below sees the same ring state)
                if (!done && nbuf > 0) {
                    const int q = hb * 3 * 256, r = hb * 2 * 256;
                    begin_path(sc, CameraSample{v3(nbd[q], nbd[q + 256], nbd[q + 512]), nbr[r], nbr[r + 256]}, ps);
                    fresh = false;
                    hb = hb + 1 == kCamDepth ? 0 : hb + 1;
                    --nbuf;
                }
#endif
            }
            RT_DBG_TEND(6, t_se);
        }
        RT_DBG_TSTART(t_bk);
        // cancellation (RenderJob::stop, server.rs:201-203): checked when a lane would start a new
        // subpixel; a set flag stops handing out work, lanes finish the subpixel they hold
        bool stop = false;
        if (a.cancel && __any(done)) stop = __hip_atomic_load(a.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        const long nt = wave_ticket(next_sub, done && !stop);
        flush_count_if_full(a.counters, nverts, done);
#if RT_DEBUG_TIMERS
        if (done) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (nt < nunits) {
                l_take = now;
                l_unit = nt;
            } else {
                l_end = now;
            }
        }
#endif
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
#if RT_DEBUG_TIMERS
    {
        const unsigned long long w_t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        // the lane that ran out of work last: when it took its last unit, and which
        unsigned long long e = l_end, tk = l_take;
        long u = l_unit;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long e2 = __shfl_xor(e, off, 64), tk2 = __shfl_xor(tk, off, 64);
            const long u2 = __shfl_xor(u, off, 64);
            const bool take2 = e2 > e || (e2 == e && u2 > u);
            e = take2 ? e2 : e;
            tk = take2 ? tk2 : tk;
            u = take2 ? u2 : u;
        }
        if ((threadIdx.x & 63) == 0 && wid < (unsigned)kDbgWaves) {
            unsigned long long* r = g_dbg_wave + kDbgWaveRec * wid;
            r[0] = w_t0;
            r[1] = w_half;
            r[2] = w_t1;
            r[3] = tk;
            r[4] = (unsigned long long)u;
        }
    }
#endif
    RT_DBG_TFLUSH();
}

// Split tail: subpixel n_whole + j's mean, continuing the sequential sum chunk 0 left in sub_buf (its lane
// summed samples [0, c0) in place, megakernel_common.h tail_in_place) over the later chunks' stored sample
// radiance, in sample order, with the same acc + L * inv_n expression as the megakernel's accumulator
// (server.rs:357-358): the bits of one lane summing every sample. A thread per subpixel; tail_buf is
// subpixel-major (tail_store), so the block stages kTailStage samples of its 256 subpixels through LDS: the
// staging loads read each subpixel's 192-byte run with 16-byte lanes side by side (a thread reading its own run
// put every lane of a load on a line of its own: 2.8 GB in 1.0 ms at N = 8,
// profiles/r06af_ktrace_share8_kernel_stats.csv; staged: 0.68 ms, profiles/r06ap_ktrace_share8_kernel_stats.csv,
// the frame's kernel unchanged; a layout with contiguous reads, 0.46 ms, cost the megakernel's stores more, tail_store). LDS rows of kTailRow doubles (an odd count: the threads' 8-byte
// reads spread over the banks).
constexpr int kTailStage = 8, kTailRow = kTailStage * 3 + 1;
__global__ __launch_bounds__(256) void k_tail_sum_f64(RenderArgs a, double* __restrict__ sub_buf, long n_split) {
    __shared__ double stage[256 * kTailRow];
    const int c0 = 1 << a.chunk_lg;
    const int ns = a.n_samples - c0;
    const size_t run = (size_t)ns * 3;  // doubles per subpixel in tail_buf
    for (long base = (long)blockIdx.x * 256; base < n_split; base += (long)gridDim.x * 256) {
        const long j = base + threadIdx.x;
        const int nj = (int)min(256L, n_split - base);  // this block's subpixels
        double* o = sub_buf + (size_t)(a.n_whole + j) * 3;
        V3 acc = j < n_split ? v3(o[0], o[1], o[2]) : v3(0, 0, 0);
        const double* src = a.tail_buf + (size_t)base * run;
        for (int s0 = 0; s0 < ns; s0 += kTailStage) {
            const int nb = min(kTailStage, ns - s0);
            __syncthreads();  // the previous stage's reads are done
            if (nb == kTailStage && (run & 1) == 0) {
                // 12 16-byte pieces per subpixel (runs and stages start 16-byte aligned: run and s0 * 3 even),
                // 12 per thread: all loads issued before the LDS writes (one round trip per stage)
                double2 v[12];
#pragma unroll
                for (int i = 0; i < 12; ++i) {
                    const int e = threadIdx.x + 256 * i, q = e / 12, k = e - q * 12;
                    if (q < nj) v[i] = *(const double2*)(src + (size_t)q * run + (size_t)s0 * 3 + 2 * k);
                }
#pragma unroll
                for (int i = 0; i < 12; ++i) {
                    const int e = threadIdx.x + 256 * i, q = e / 12, k = e - q * 12;
                    if (q < nj) {
                        stage[q * kTailRow + 2 * k] = v[i].x;
                        stage[q * kTailRow + 2 * k + 1] = v[i].y;
                    }
                }
            } else {
                const int per = nb * 3;
                for (int e = threadIdx.x; e < nj * per; e += 256) {
                    const int q = e / per, k = e - q * per;
                    stage[q * kTailRow + k] = src[(size_t)q * run + (size_t)s0 * 3 + k];
                }
            }
            __syncthreads();
            if (j < n_split) {
                const double* r = stage + threadIdx.x * kTailRow;
                for (int k = 0; k < nb; ++k) acc = acc + v3(r[3 * k], r[3 * k + 1], r[3 * k + 2]) * a.inv_n;
            }
        }
        if (j < n_split) {
            o[0] = acc.x;
            o[1] = acc.y;
            o[2] = acc.z;
        }
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

thread_local TailPlan t_tail_plan;

template <int F, int W>
static void launch_mk(const DevScene& sc, const RenderArgs& a_in, double* sub_buf, uint32_t* next_sub, long nsub,
                      int refill, double* tail_buf, size_t tail_cap, hipStream_t st) {
    const long blocks = resident_blocks(k_megakernel_f64<F, W>, (nsub + 255) / 256);
    RenderArgs a = a_in;
    plan_tail(a, nsub, blocks * 256, tail_buf, tail_cap, tail_split_x2(nsub, blocks * 256), 2, 256, RT_MK_MIN_RUN);
    hipLaunchKernelGGL((k_megakernel_f64<F, W>), dim3((unsigned)blocks), dim3(256), 0, st, sc, a, sub_buf, next_sub, nsub,
                       refill);
    const long n_split = nsub - a.n_whole;
    if (n_split > 0) {
        const long tb = std::max(1L, std::min(4096L, (n_split + 255) / 256));
        hipLaunchKernelGGL(k_tail_sum_f64, dim3((unsigned)tb), dim3(256), 0, st, a, sub_buf, n_split);
    }
}

// The analytic / fused-mesh megakernel at its waves/SIMD: 4 for analytic scenes, 3 with meshes (the defaults);
// A/B builds (ab_knobs.h) compile both shapes of every instance for RT_MK_WAVES.
template <int F>
static void launch_mk_shape(int waves, const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                            long nsub, int refill, double* tail_buf, size_t tail_cap, hipStream_t st) {
    if constexpr (RT_AB_KNOBS != 0) {
        if (waves == 3) launch_mk<F, 3>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);
        else launch_mk<F, RT_MK_W4>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);
    } else if constexpr ((F & 1) != 0) {
        (void)waves;
        launch_mk<F, 3>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);
    } else {
        (void)waves;
        launch_mk<F, RT_MK_W4>(sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st);
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
    t_tail_plan = TailPlan{};
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
        return launch_megakernel_mesh_f64(sc, a, sub_buf, next_sub, nsub, refill, wmin, tail_buf, tail_cap, st);
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
        launch_mk_shape<F>(waves, sc, a, sub_buf, next_sub, nsub, refill, tail_buf, tail_cap, st); \
        break;
    switch (a.features & 15) {
        RT_MK_CASE(0) RT_MK_CASE(1) RT_MK_CASE(2) RT_MK_CASE(3) RT_MK_CASE(4) RT_MK_CASE(5) RT_MK_CASE(6)
        RT_MK_CASE(7) RT_MK_CASE(8) RT_MK_CASE(9) RT_MK_CASE(10) RT_MK_CASE(11) RT_MK_CASE(12) RT_MK_CASE(13)
        RT_MK_CASE(14) RT_MK_CASE(15)
    }
#undef RT_MK_CASE
    return hipGetLastError();
}

// Scratch bytes one split subpixel needs (plan_tail: the samples after chunk 0, at the default chunk size).
size_t tail_scratch_per_subpixel(int n_samples) {
    RenderArgs a{};
    a.n_samples = n_samples;
    plan_tail(a, 0, 0, nullptr, 0);
    return (size_t)std::max(0, n_samples - (1 << a.chunk_lg)) * 3 * sizeof(double);
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
// mantissas), counts rcp_rn(b) != 1.0 / b and qdiv(a, b, rcp_rn(b)) != a / b; and for x spread over
// sqrt_rn's fast range [2^-767, 2^1024) (every exponent, random and extreme mantissas), counts
// sqrt_rn(x) != sqrt(x) (the library sequence with its input scaling and 0/inf fixup). sqrt_rn takes
// its fast path only when the whole wave is in range (a wave vote), so bit equality with the library
// is what makes a lane's result independent of the other lanes of its wave.
__global__ void k_selftest_arith(long n, uint64_t seed, unsigned long long* bad) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Rng g(seed, (uint32_t)i, (uint32_t)(i >> 32), 7u);
    const uint64_t m = g.next(), m2 = g.next(), sel = g.next(), m3 = g.next(), sel2 = g.next();
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
    uint64_t sm = m3 & 0xFFFFFFFFFFFFFull;
    if ((sel2 & 7) == 0) sm = 0;
    if ((sel2 & 7) == 1) sm = 0xFFFFFFFFFFFFFull;
    if ((sel2 & 7) == 2) sm = (sel2 >> 8) & 0xFF;
    if ((sel2 & 7) == 3) sm = 0xFFFFFFFFFFFFFull - ((sel2 >> 8) & 0xFF);
    const int sx = -767 + (int)((sel2 >> 16) % 1791);  // [-767, 1023]
    const double x = __longlong_as_double((long long)(((uint64_t)(sx + 1023) << 52) | sm));
    if (__double_as_longlong(sqrt_rn(x)) != __double_as_longlong(sqrt(x))) e |= 4;
    if (e & 1) atomicAdd(&bad[0], 1ull);
    if (e & 2) atomicAdd(&bad[1], 1ull);
    if (e & 4) atomicAdd(&bad[2], 1ull);
}

// Diagnostic builds: the wave records of the last k_megakernel_f64 launches (start, half-idle, end per wave, on
// the 100 MHz s_memrealtime clock; zeros for waves that did not run), then cleared; 1 (zeros) without timers.
extern "C" int rt_debug_wave_times(unsigned long long* out, int n_waves) {
    if (!out || n_waves <= 0) return -1;
    for (long i = 0; i < 5L * n_waves; ++i) out[i] = 0;
#if RT_DEBUG_TIMERS
    const int n = std::min(n_waves, kDbgWaves);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_wave), kDbgWaveRec * sizeof(unsigned long long) * n) != hipSuccess) return -1;
    static unsigned long long zeros[kDbgWaveRec * kDbgWaves];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_wave), zeros, sizeof zeros) != hipSuccess) return -1;
    return 0;
#else
    return 1;
#endif
}

// The split tail of the calling thread's last megakernel launch (kernels.h TailPlan).
extern "C" int rt_debug_last_split(long long out[3]) {
    if (!out) return -1;
    out[0] = t_tail_plan.n_split;
    out[1] = t_tail_plan.want;
    out[2] = t_tail_plan.chunk;
    return 0;
}

// n_out: the caller's output count (at most 3 are written: reciprocal, quotient, square root)
extern "C" int rt_selftest_arith_n(long n, unsigned long long seed, unsigned long long* out, int n_out) {
    unsigned long long* d = nullptr;
    if (n <= 0 || !out || n_out <= 0 || hipMalloc(&d, 3 * sizeof(unsigned long long)) != hipSuccess) return -1;
    int rc = 0;
    unsigned long long h[3] = {0, 0, 0};
    if (hipMemset(d, 0, 3 * sizeof(unsigned long long)) != hipSuccess) rc = -1;
    if (!rc) {
        hipLaunchKernelGGL(k_selftest_arith, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, seed, d);
        if (hipGetLastError() != hipSuccess || hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    }
    (void)hipFree(d);
    for (int i = 0; i < n_out && i < 3; ++i) out[i] = h[i];
    return rc;
}
// The original two-output entry point (reciprocal, quotient), kept for callers built against it.
extern "C" int rt_selftest_arith(long n, unsigned long long seed, unsigned long long out[2]) {
    return rt_selftest_arith_n(n, seed, out, 2);
}

// Pointer round trips of the per-call views every trace call goes through (scene.rs:272-289 reads the
// scene's tables): the compact-table pointer rebuilt from two readfirstlane halves (tables()), the scene
// and render arguments read in place in the kernarg segment (karg_scene / karg_render_args at offsets 0
// and 248, the megakernels' own parameter order). out[0] tables() through the kernarg view, [1] tables()
// of the by-value argument, [2] the round-4 sign-extending form (tables_form<true>), [3] the kernarg
// view's raw ctab, [4] its node_slot, [5] karg_render_args().tail_buf. The pointers are never
// dereferenced, so fabricated addresses are safe.
__global__ __launch_bounds__(64) void k_selftest_tables(DevScene sc_g, RenderArgs a_g, unsigned long long* out) {
    const DevScene& sc = karg_scene();
    const RenderArgs& a = karg_render_args();
    const uint64_t v[6] = {(uint64_t)(uintptr_t)tables(sc), (uint64_t)(uintptr_t)tables(sc_g),
                           (uint64_t)(uintptr_t)tables_form<true>(sc), (uint64_t)(uintptr_t)sc.ctab,
                           (uint64_t)(uintptr_t)sc.node_slot, (uint64_t)(uintptr_t)a.tail_buf};
    (void)a_g;
    if (threadIdx.x < 6) out[threadIdx.x] = v[threadIdx.x];
}

extern "C" int rt_selftest_tables(const unsigned long long* ptrs, int n, unsigned long long* out) {
    if (!ptrs || !out || n <= 0) return -1;
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 6 * sizeof(unsigned long long)) != hipSuccess) return -1;
    int rc = 0;
    for (int i = 0; i < n && !rc; ++i) {
        DevScene sc{};
        RenderArgs a{};
        sc.ctab = (const CompactTab*)(uintptr_t)ptrs[i];
        sc.node_slot = (const KidSlot*)(uintptr_t)(ptrs[i] + 16);
        a.tail_buf = (double*)(uintptr_t)(ptrs[i] + 32);
        hipLaunchKernelGGL(k_selftest_tables, dim3(1), dim3(64), 0, 0, sc, a, d);
        if (hipGetLastError() != hipSuccess || hipMemcpy(out + 6 * (size_t)i, d, 6 * sizeof(unsigned long long),
                                                         hipMemcpyDeviceToHost) != hipSuccess)
            rc = -1;
    }
    (void)hipFree(d);
    return rc;
}

#define RT_DIAG_TU_FN diag_read_main
#include "diag_tu.h"

// Diagnostic builds: the counters of every kernel code object, summed, then cleared (zeros otherwise);
// a null output leaves that set alone.
static int diag_all(unsigned long long* cnt16, unsigned long long* reg32, unsigned long long* tim16, unsigned long long* q4) {
    for (int i = 0; i < 16; ++i) {
        if (cnt16) cnt16[i] = 0;
        if (tim16) tim16[i] = 0;
    }
    for (int i = 0; i < 32 && reg32; ++i) reg32[i] = 0;
    for (int i = 0; i < 4 && q4; ++i) q4[i] = 0;
    if (diag_read_main(cnt16, reg32, tim16, q4) || diag_read_mesh(cnt16, reg32, tim16, q4) ||
        diag_read_flat(cnt16, reg32, tim16, q4))
        return -1;
    return 0;
}

// RT_QCHECK builds: read and clear the LDS hand-off protocol counters (megakernel_common.h);
// returns 1 (and zeros) when the checks are not compiled in.
extern "C" int rt_debug_qcheck(unsigned long long out[4]) {
#if RT_QCHECK
    return diag_all(nullptr, nullptr, nullptr, out);
#else
    for (int i = 0; i < 4; ++i) out[i] = 0;
    return 1;
#endif
}

// Diagnostic builds: read and clear the region counters and timers (all zeros otherwise).
extern "C" int rt_debug_regions(unsigned long long out[64]) {
    for (int i = 48; i < 64; ++i) out[i] = 0;
    return diag_all(nullptr, out, out + 32, nullptr);
}

// Diagnostic builds: read and clear the traversal counters (all zeros otherwise).
extern "C" int rt_debug_counters(unsigned long long out[16]) {
    return diag_all(out, nullptr, nullptr, nullptr);
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
