// Scheduling shared by the persistent megakernels (render_f64.hip, render_flat_f64.hip): wave-
// aggregated tickets on one global counter, work units (runs of whole subpixels, split-tail chunks),
// and the host-side planning of both.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../ab_knobs.h"
#include "kernels.h"

namespace rt {

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

// The megakernels' own (DevScene, RenderArgs) arguments, read in place in the kernel-argument segment
// through an opaque constant-space pointer: every use is a scalar load (a K$ hit) issued where the
// value is needed. Held as values, their ~100 SGPRs live across the whole path loop and the register
// allocator spills them to VGPR lanes (v_writelane at entry, v_readlane at each use: VALU issue slots
// and SGPR hazard nops in a VALU-bound loop; 54 SGPR + 4 VGPR spills in k_megakernel_f64<8,4>). The
// megakernels take DevScene and RenderArgs as their first two arguments: by the AMDGPU kernarg layout
// at offset 0 and at sizeof(DevScene) rounded up to RenderArgs' alignment (248: the code objects'
// .args metadata). RT_KARG_VIEW=0 builds keep the by-value arguments (A/B).
#ifndef RT_KARG_VIEW
#define RT_KARG_VIEW 1
#endif
typedef const __attribute__((address_space(4))) char KargByte;
constexpr size_t kKargArgsOffset = (sizeof(DevScene) + alignof(RenderArgs) - 1) / alignof(RenderArgs) * alignof(RenderArgs);
static_assert(kKargArgsOffset == 248, "DevScene / RenderArgs kernarg layout changed: check the .args metadata");
__device__ __forceinline__ KargByte* karg_base() {
    KargByte* p = (KargByte*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));  // opaque: no value is hoisted to the kernel entry and held in SGPRs
    return p;
}
__device__ __forceinline__ const DevScene& karg_scene() {
    return *(const DevScene*)(const __attribute__((address_space(4))) DevScene*)karg_base();
}
__device__ __forceinline__ const RenderArgs& karg_render_args() {
    return *(const RenderArgs*)(const __attribute__((address_space(4))) RenderArgs*)(karg_base() + kKargArgsOffset);
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
// flush_count when a lane's 32-bit count nears overflow (at a unit switch, `done`): the per-lane counts of a
// launch stay far below 2^30 (a lane traces ~10^5 to 10^6 vertices), so in practice once, at the kernel's end.
// (Flushing at every unit switch put a second device-scope atomic on one address next to each ticket, in every
// render with stats: with 1.5 subpixels per lane split into 32-sample chunks, an N = 8 cornell share ran at 1688.7
// Msamples/s with it and 1903.4 without, profiles/r06s_ab_tail_share.log / r06u_ab_tail.log.)
constexpr uint32_t kFlushAt = 1u << 30;
__device__ __forceinline__ void flush_count_if_full(unsigned long long* counter, uint32_t& n, bool done) {
    if (__any(done && n >= kFlushAt)) flush_count(counter, n);
}

// Work unit of ticket t: the whole subpixels [id, end) (t < n_wunits: a run of unit_subs consecutive
// subpixels, samples [0, n) each), or chunk c = t - n_wunits of the split tail (subpixel
// n_whole + c / cps, samples [k 2^chunk_lg, (k + 1) 2^chunk_lg), k = c % cps; end = id + 1).
__device__ __forceinline__ void unit_of(const RenderArgs& a, long t, int& id, int& end, int& s) {
    if (t < a.n_wunits) {
        id = (int)t * a.unit_subs;
        end = min(id + a.unit_subs, a.n_whole);
        s = 0;
    } else {
        const uint32_t c = (uint32_t)(t - a.n_wunits);  // < n_split * cps < 2^32 (plan_tail)
        const uint32_t q = c / (uint32_t)a.tail_cps;
        id = a.n_whole + (int)q;
        end = id + 1;
        s = (int)(c - q * (uint32_t)a.tail_cps) << a.chunk_lg;
    }
}
// One past the last subpixel of the run of whole subpixels that holds subpixel id (< n_whole): runs
// are aligned to unit_subs, so no register holds the run's end (the analytic megakernel's VGPRs).
__device__ __forceinline__ int run_end(const RenderArgs& a, int id) {
    const int b = a.unit_subs;
    return min((id / b + 1) * b, a.n_whole);
}
// Is sample s2 (> s) part of the unit that holds sample s?
__device__ __forceinline__ bool unit_has(const RenderArgs& a, int id, int s, int s2) {
    return s2 < a.n_samples && (id < a.n_whole || (s2 >> a.chunk_lg) == (s >> a.chunk_lg));
}
// Is sample s + 1 still part of the unit that holds sample s? (No register for the unit's end: a
// split unit ends at the next multiple of 2^chunk_lg.)
__device__ __forceinline__ bool unit_has_next(const RenderArgs& a, int id, int s) {
    return s + 1 < a.n_samples && (id < a.n_whole || ((s + 1) >> a.chunk_lg) == (s >> a.chunk_lg));
}

__device__ __forceinline__ bool lane_id_is0() { return __lane_id() == 0; }

// Protocol checks of the LDS hand-offs below (build with -DRT_QCHECK=1; rt_debug_qcheck reads and
// clears them). A violation is counted, never trapped (a trap would fault the device):
//   [0] queue_put found its ring slot still holding an entry (not -1), or queue_read a value that is
//       not a queue entry;  [1] more entries queued than the ring holds (tail - head > capacity);
//   [2] an outstanding-query count (fpool s_pend) decremented below zero;
//   [3] an owner / taker state mismatch: a new count stored over a non-zero s_pend, or the walk pool
//       handing out a query whose status word is not CLOSEST / SHADOW.
#ifndef RT_QCHECK
#define RT_QCHECK 0
#endif
#if RT_QCHECK
__device__ unsigned long long g_qcheck[4];
#define RT_QFAIL(i) atomicAdd(&g_qcheck[i], 1ull)
#else
#define RT_QFAIL(i) ((void)0)
#endif

// Multi-producer multi-consumer work queue of int entries (>= 0) in LDS, shared by the waves of a
// block without barriers: a ring of mask + 1 entries (initialised to -1) with monotonically growing
// head / tail counters. The caller guarantees that no more than mask + 1 entries are ever queued
// at once (each query of a block is in the queue at most once). Entries are written after the tail
// is advanced, so a taker waits for its entry to turn non-negative; it then resets it to -1.
template <class E>
struct LdsQueueT {
    using T = E;
    E* ring;         // entries (>= 0), -1 = empty slot; int32_t, or int16_t for queues of < 2^15 entries
    uint32_t* head;  // next entry to take
    uint32_t* tail;  // next entry to fill
    uint32_t mask;   // capacity - 1 (a power of two)
};
using LdsQueue = LdsQueueT<int32_t>;
using LdsQueue16 = LdsQueueT<int16_t>;  // the role-split pool's path ids: half the ring's LDS
// Entries queued and not yet claimed (head read first: the tail read after it is >= it, so the
// difference never wraps).
template <class Q>
__device__ __forceinline__ uint32_t queue_len(const Q& q) {
    const uint32_t h = __hip_atomic_load(q.head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __hip_atomic_load(q.tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) - h;
}
// Appends v of every lane with `put` (wave-aggregated). All lanes of the wave call.
template <class Q>
__device__ __forceinline__ void queue_put(const Q& q, bool put, int32_t v) {
    using T = typename Q::T;
    const unsigned long long m = __ballot(put);
    if (m == 0ull) return;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = __hip_atomic_fetch_add(q.tail, (uint32_t)__popcll(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    base = __shfl(base, leader, 64);
    const unsigned long long below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
#if RT_QCHECK
    if (lane == leader) {
        const uint32_t h = __hip_atomic_load(q.head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // signed: takers may already have claimed past this append (head > base + n) while it is written
        if ((int32_t)(base + (uint32_t)__popcll(m) - h) > (int32_t)(q.mask + 1u)) RT_QFAIL(1);
    }
    if (put) {
        const T old = __hip_atomic_exchange(&q.ring[(base + (uint32_t)__popcll(below)) & q.mask], (T)v, __ATOMIC_RELEASE,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old != -1) RT_QFAIL(0);
    }
#else
    if (put) __hip_atomic_store(&q.ring[(base + (uint32_t)__popcll(below)) & q.mask], (T)v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}
// Claims up to `most` entries, but only if at least max(need, 1) are queued; the leader lane does the
// compare-and-swap. Returns the first claimed position and the count (wave-uniform).
template <class Q>
__device__ __forceinline__ void queue_claim(const Q& q, int leader, uint32_t most, int need, uint32_t& h, uint32_t& k) {
    h = 0;
    k = 0;
    if (__lane_id() == leader) {
        for (;;) {
            h = __hip_atomic_load(q.head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t t = __hip_atomic_load(q.tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t avail = t - h;
            if ((int)avail < max(need, 1)) { k = 0; break; }
            k = min(avail, most);
            uint32_t exp = h;
            if (__hip_atomic_compare_exchange_strong(q.head, &exp, h + k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP))
                break;
        }
    }
    h = __shfl(h, leader, 64);
    k = __shfl(k, leader, 64);
}
template <class Q>
__device__ __forceinline__ int32_t queue_read(const Q& q, uint32_t pos) {
    using T = typename Q::T;
    T* e = &q.ring[pos & q.mask];
    T v;
    while ((v = __hip_atomic_load(e, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < 0) __builtin_amdgcn_s_sleep(1);
    __hip_atomic_store(e, (T)-1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (RT_QCHECK && (uint32_t)v > q.mask) RT_QFAIL(0);  // entries (lane ids, + 256 for fpool shadow queries) < capacity
    return (int32_t)v;
}
// Takes up to 64 entries (lane i the i-th), but only if at least `need` are queued; -1 for lanes
// without one. All lanes of the wave call.
template <class Q>
__device__ __forceinline__ int32_t queue_take(const Q& q, int need) {
    uint32_t h, k;
    queue_claim(q, 0, 64u, need, h, k);
    return (uint32_t)__lane_id() < k ? queue_read(q, h + (uint32_t)__lane_id()) : -1;
}
// Every lane with `want` takes one entry while any are queued (-1 otherwise). All lanes call.
template <class Q>
__device__ __forceinline__ int32_t queue_take_each(const Q& q, bool want) {
    const unsigned long long m = __ballot(want);
    if (m == 0ull) return -1;
    const int lane = __lane_id();
    uint32_t h, k;
    queue_claim(q, __ffsll((long long)m) - 1, (uint32_t)__popcll(m), 1, h, k);
    const unsigned long long below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
    const uint32_t rank = (uint32_t)__popcll(below);
    return want && rank < k ? queue_read(q, h + rank) : -1;
}

// Resident grid of a persistent kernel: as many blocks (of `threads`) as fit on the device at once.
template <class K>
static inline long resident_blocks(K kernel, long want, int threads = 256) {
    int dev = 0, ncu = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    return std::max(1L, std::min((long)ncu * per_cu, want));
}

// A/B overrides (ab_knobs.h): RT_* environment variables in -DRT_AB_KNOBS=1 builds only
static inline int env_int(const char* name, int dflt) { return (int)ab_knob(name, dflt); }

#ifndef RT_MK_W4
#define RT_MK_W4 4  // waves/SIMD of the analytic-scene kernel (A/B builds: -DRT_MK_W4=5)
#endif
// Split tail (RenderArgs::n_whole): the last subpixels are handed out in chunks of samples, so the
// frame does not end with lanes idling while others finish a whole subpixel (the 1/N-sized frames
// of an N-GPU run hold only a few subpixels per lane). plan_tail's split_x2 / 2 subpixels per resident
// lane are split, at most nsub / cap_div, limited by the scratch buffer (tail_cap bytes); RT_MK_TAIL=0
// disables it.
// Runs of whole subpixels per ticket: about RT_MK_UNIT_SAMPLES (256) samples per ticket, but at least
// RT_MK_UNITS_PER_LANE (16) runs per resident lane, so the frame's end stays balanced (2 runs per lane
// left the unicorn's lanes idling behind a few long runs: -30%). At 1024 spp that is one subpixel per
// ticket; at 64 spp (16 samples per subpixel) a ticket per subpixel put every wave behind the one
// counter's atomic every few iterations (1920x1080x64: 2.3x the 1024-spp time per sample). The mesh walk
// kernels pass 64: their samples cost ~17x the analytic kernel's, so a run of 16 subpixels at 64 spp (C5) was
// 1/21 of a path slot's frame and left slots idle behind the last runs: C5 363.0 -> 367.5 Msamples/s
// (32: 368.0, 16: 368.5; profiles/r06av_ab_units_c5.log, r06aw_ab_units_c5.log), C4 unchanged.
static inline void plan_units(RenderArgs& a, long lanes, int unit_samples = 256, int min_run = 1) {
    static const int env_target = env_int("RT_MK_UNIT_SAMPLES", 0);
    const int target = std::max(1, env_target > 0 ? env_target : unit_samples);
    static const int per_lane = std::max(1, env_int("RT_MK_UNITS_PER_LANE", 16));
    // ... but, in the analytic kernel (min_run 32), never fewer than min_run samples per ticket while the frame has
    // more than one run per lane: one counter word takes ~88 returning atomics per microsecond
    // (MI355X_MICROARCH.md, "dequeue"), and a frame of a few samples per lane handed out a subpixel at a time is
    // bound by it. C1' (600x450, 4 spp: one sample per subpixel) 291.5 -> 393.6 Msamples/s, cornell 1920x1080 at
    // 64 spp 1570.6 -> 1808.7 (profiles/r06bo_ab_min_run.log; the kernel 3.70 -> 2.70 ms on C1',
    // r06bn_ktrace_c1p_kernel_stats.csv); the cubes' query pool at 64 spp measured 1.9% slower with it (min_run 1).
    const long n = std::max(1, a.n_samples), lanes1 = std::max(1L, lanes);
    const long b_rate = std::min((std::max(1, min_run) + n - 1) / n, std::max(1L, (long)a.n_whole / lanes1));
    long b = std::max(1L, target / n);
    b = std::max(1L, std::min(b, std::max(b_rate, (long)a.n_whole / (lanes1 * per_lane))));
    a.unit_subs = (int32_t)b;
    a.n_wunits = (int32_t)(((long)a.n_whole + b - 1) / b);
}

// split_x2 / 2 subpixels per resident lane, cap_div 2 (at most half the frame): the analytic and flat-mesh
// kernels pass kernels.h tail_split_x2 (1.5 per lane, 2 in frames of <= 4 per lane; the default 1 is half a
// subpixel per lane, the round-5 rule, which left the full frame's last waves behind whole subpixels). The mesh walk
// kernels pass 12 and 1 (six subpixels per path slot, up to the whole frame): a unicorn subpixel's cost
// depends on where it lies (walls or the mesh), and the last whole subpixels' spread left an N = 8 share
// at 0.81 of the full frame's rate with half a subpixel per slot, 0.96 with six (profiles/r05bc_tail.log).
static inline void plan_tail(RenderArgs& a, long nsub, long lanes, double* tail_buf, size_t tail_cap, int split_x2 = 1,
                             int cap_div = 2, int unit_samples = 256, int min_run = 1) {
    static const int tail_env = env_int("RT_MK_TAIL", 1);
    // A/B overrides: RT_MK_TAIL_MUL / RT_MK_TAIL_DIV subpixels per lane (defaults 1 / 2 once either is set),
    // RT_MK_TAIL_CAP_DIV, RT_MK_TAIL_MIN_LG (the shortest chunk, 2^min_lg samples)
    static const int env_mul = env_int("RT_MK_TAIL_MUL", 0), env_div = env_int("RT_MK_TAIL_DIV", 0);
    static const int env_cap = env_int("RT_MK_TAIL_CAP_DIV", 0);
    static const int min_lg = std::max(2, env_int("RT_MK_TAIL_MIN_LG", 5));
    const long split_want = (env_mul > 0 || env_div > 0)
                                ? lanes * std::max(1, env_mul) / (env_div > 0 ? env_div : 2)
                                : lanes * std::max(1, split_x2) / 2;
    if (env_cap > 0) cap_div = env_cap;
    // chunks of 2^chunk_lg samples, about RT_MK_TAIL_CPS (8) per subpixel, and at least 32 samples: every
    // chunk costs a ticket on the one global counter, whose device-scope atomics saturate when chunks turn
    // over faster (16-sample chunks: the cornell frame +1.9%, 8-sample: +5%, profiles/r05az_tail.log); 8
    // per subpixel (4 until round 5) gave an N = 8 cornell share 0.933 -> 0.939 of the full frame's rate
    static const int cps_target = std::max(1, env_int("RT_MK_TAIL_CPS", 8));
    a.chunk_lg = min_lg;
    while ((a.n_samples >> a.chunk_lg) > cps_target) ++a.chunk_lg;
    a.tail_cps = (a.n_samples + (1 << a.chunk_lg) - 1) >> a.chunk_lg;
    // chunk 0 of a split subpixel sums in place (tail_in_place): scratch only for the samples after it
    const size_t per_sub = (size_t)std::max(0, a.n_samples - (1 << a.chunk_lg)) * 3 * sizeof(double);
    long n_split = 0, want = 0;
    if (tail_env && a.n_samples >= 64 && a.tail_cps >= 2 && per_sub > 0) {
        want = std::min(split_want, nsub / std::max(1, cap_div));
        if (tail_buf) n_split = std::min(want, (long)(tail_cap / per_sub));
    }
    if (nsub > 0) t_tail_plan = TailPlan{n_split, want, 1L << a.chunk_lg};  // rt_debug_last_split
    a.n_whole = (int32_t)(nsub - n_split);
    a.tail_buf = tail_buf;
    plan_units(a, lanes, unit_samples, min_run);
}
// Split tail, per sample of a split subpixel: chunk 0 (samples [0, 2^chunk_lg)) sums its samples in
// place, acc = acc + L * inv_n from 0 exactly like a whole subpixel, and leaves its partial sum in the
// subpixel's sub_buf entry; every later chunk stores each sample's radiance for k_tail_sum_f64, which
// continues the same sequential sum from chunk 0's partial (the same bits as one lane summing all).
__device__ __forceinline__ bool tail_in_place(const RenderArgs& a, int s) { return (s >> a.chunk_lg) == 0; }
#ifndef RT_TAIL_PROBE
#define RT_TAIL_PROBE 0  // diagnostic builds only: 1 = every lane stores to one slot of its own (wrong frames; the
                         // per-sample stores' footprint without their scatter)
#endif
// tail_buf layout: subpixel-major, [j][s - c0][3] (j = id - n_whole): a chunk's lane writes one contiguous run.
// (Groups of 64 subpixels, sample-major with a row per component, made k_tail_sum's loads contiguous, 1.0 -> 0.46 ms
// at N = 8, but scattered these stores: the frame ran 0.1-0.3% slower, profiles/r06an_ab_tail_layout.log.)
__device__ __forceinline__ void tail_store(const RenderArgs& a, int id, int s, const f64::V3& L) {
#if RT_TAIL_PROBE == 1
    (void)id; (void)s;
    double* o = a.tail_buf + ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 3;
#else
    const int c0 = 1 << a.chunk_lg;
    double* o = a.tail_buf + ((size_t)(id - a.n_whole) * (size_t)(a.n_samples - c0) + (size_t)(s - c0)) * 3;
#endif
    o[0] = L.x;
    o[1] = L.y;
    o[2] = L.z;
}

// k_tail_sum_f64 for the split tail of a megakernel launch (render_f64.hip)
void launch_tail_sum_f64(const RenderArgs& a, double* sub_buf, long n_split, hipStream_t st);

}  // namespace rt
