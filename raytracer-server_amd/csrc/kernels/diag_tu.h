// Diagnostic symbols of one kernel translation unit. Every .hip file is its own code object with its
// own copies of path_f64.h's g_dbg / g_dbg_region / g_dbg_time and megakernel_common.h's g_qcheck, so
// each kernel TU includes this header once, at its end, with RT_DIAG_TU_FN naming its reader; the
// rt_debug_* entry points (render_f64.hip) sum the readers of every TU.
// Reader: adds this TU's counters to cnt16 / reg32 / tim16 / q4 and clears them (a null output: that
// set is left alone); 0 or -1 (HIP error).
#define RT_DIAG_TAKE(sym, acc, n)                                                                         \
    do {                                                                                                  \
        if (!(acc)) break;                                                                                \
        unsigned long long v_[n] = {0}, z_[n] = {0};                                                      \
        if (hipMemcpyFromSymbol(v_, HIP_SYMBOL(sym), sizeof(v_)) != hipSuccess ||                         \
            hipMemcpyToSymbol(HIP_SYMBOL(sym), z_, sizeof(z_)) != hipSuccess)                             \
            return -1;                                                                                    \
        for (int i_ = 0; i_ < n; ++i_) acc[i_] += v_[i_];                                                 \
    } while (0)
int RT_DIAG_TU_FN(unsigned long long* cnt16, unsigned long long* reg32, unsigned long long* tim16,
                  unsigned long long* q4) {
    (void)cnt16; (void)reg32; (void)tim16; (void)q4;
#if RT_DEBUG_COUNTERS
    RT_DIAG_TAKE(g_dbg, cnt16, 16);
    RT_DIAG_TAKE(g_dbg_region, reg32, 32);
#endif
#if RT_DEBUG_TIMERS
    RT_DIAG_TAKE(g_dbg_time, tim16, 16);
#endif
#if RT_QCHECK
    RT_DIAG_TAKE(g_qcheck, q4, 4);
#endif
    return 0;
}
#undef RT_DIAG_TAKE
#undef RT_DIAG_TU_FN
