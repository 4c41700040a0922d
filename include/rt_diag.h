/*
 * rt_diag.h — diagnostics exported by librtamd.so next to the C ABI of rt_ffi.h (not part of the
 * drop-in surface; used by tests and tools/).
 */
#ifndef RT_DIAG_H
#define RT_DIAG_H
#ifdef __cplusplus
extern "C" {
#endif
/* Device self-test of the exact-arithmetic shortcuts (path_f64.h: rcp_rn, qdiv, sqrt_rn) against
 * the IEEE operations on n pseudo-random operands on the current HIP device; writes min(n_out, 3)
 * counts: out[0] = reciprocal mismatches, out[1] = quotient mismatches, out[2] = square-root
 * mismatches (sqrt_rn's fast range [2^-767, 2^1024) against the library sqrt). Returns 0 or -1. */
int rt_selftest_arith_n(long n, unsigned long long seed, unsigned long long* out, int n_out);
/* The original entry point: out[0] reciprocal and out[1] quotient mismatches only. */
int rt_selftest_arith(long n, unsigned long long seed, unsigned long long out[2]);
/* Device round trips of the pointers every trace call rebuilds (no dereference: any 64-bit pattern is
 * safe): for each of the n addresses p = ptrs[i], a kernel launched with DevScene.ctab = p,
 * DevScene.node_slot = p + 16 and RenderArgs.tail_buf = p + 32 as its first two (kernarg) arguments
 * writes out[6i + k]: k = 0 tables() through the kernarg view, 1 tables() of the by-value argument,
 * 2 the round-4 sign-extending form (wrong whenever bit 31 of p is set: kept to show the check catches
 * it), 3 the kernarg view's ctab, 4 its node_slot, 5 the kernarg RenderArgs' tail_buf. Returns 0 or -1. */
int rt_selftest_tables(const unsigned long long* ptrs, int n, unsigned long long* out);
/* RT_QCHECK builds (-DRT_QCHECK=1): counters of LDS hand-off protocol violations in the megakernels'
 * work queues since the last call (kernels/megakernel_common.h): [0] ring slot overwritten / bad
 * entry, [1] queue over capacity, [2] outstanding-query count below zero, [3] owner/taker state
 * mismatch. Returns 0, 1 when the checks are not compiled in (zeros), -1 on a HIP error. */
int rt_debug_qcheck(unsigned long long out[4]);
/* RT_DEBUG_COUNTERS builds: octree traversal counters since the last call (zeros otherwise):
 * [0] walks [1] past the cull [2] node visits [3] leaves opened [4] triangle tests [5] walk steps;
 * interleaved mesh megakernel: [8] wave iterations [9] lanes in the vertex phase [10] walk-loop
 * wave steps [11] walking lanes summed over those steps. */
int rt_debug_counters(unsigned long long out[16]);
/* RT_DEBUG_COUNTERS builds: lane utilisation per instrumented code region (RT_DBG_REGION) since
 * the last call: out[2i] = wave entries into region i, out[2i+1] = active lanes summed over them
 * (i < 16); RT_DEBUG_TIMERS builds: out[32 + i] = s_memtime ticks of the megakernel's waves in timed
 * region i (RT_DBG_TSTART / RT_DBG_TEND), summed over waves. */
int rt_debug_regions(unsigned long long out[64]);
/* The split tail (kernels/megakernel_common.h plan_tail) of the calling thread's last f64 megakernel
 * render: out[0] = subpixels handed out as sample chunks (0: none split; only when spp / 4 >= 64),
 * out[1] = how many the kernel family wanted before the scratch buffer capped it (out[0] < out[1]: the
 * buffer was too small; the frame is the same, only the end of the launch balances worse), out[2] =
 * samples per chunk. Returns 0. */
int rt_debug_last_split(long long out[3]);
/* RT_DEBUG_TIMERS builds: per wave of the last analytic-scene megakernel launches (k_megakernel_f64), on the
 * constant 100 MHz s_memrealtime clock: out[5w] its start, out[5w + 1] when fewer than half of its lanes
 * last held work (all ones: never), out[5w + 2] its end (zeros: wave w did not run), and for the lane of it
 * that ran out of work last: out[5w + 3] when it took its last unit, out[5w + 4] that unit (ticket); then
 * cleared. For
 * n_waves <= 8192. Returns 0, 1 without the timers (zeros), -1 on a HIP error. */
int rt_debug_wave_times(unsigned long long* out, int n_waves);
#ifdef __cplusplus
}
#endif
#endif /* RT_DIAG_H */
