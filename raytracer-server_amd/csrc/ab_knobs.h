// A/B switches. The kernels' tuning constants (block shapes, thresholds, which kernel a scene takes)
// were chosen by A/B runs on one MI355X; those runs override them through RT_* environment
// variables, but only in A/B builds (-DRT_AB_KNOBS=1: lib/variants/ab.so, the diagnostic build). The
// product library (lib/librtamd.so) takes every default and reads no environment variable for them, so a
// stray RT_MK_* in a server's environment cannot change which kernel runs (the reference's only runtime
// configuration is argv and PORT, main.rs:20-40).
#pragma once
#include <cstdlib>

#ifndef RT_AB_KNOBS
#define RT_AB_KNOBS 0
#endif

namespace rt {
// The A/B override of `name` (an integer), or dflt; dflt in product builds.
static inline long ab_knob(const char* name, long dflt) {
#if RT_AB_KNOBS
    const char* v = std::getenv(name);
    return (v && *v) ? std::atol(v) : dflt;
#else
    (void)name;
    return dflt;
#endif
}
}  // namespace rt
