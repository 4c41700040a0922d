// Streaming wavefront pipeline (f64): host driver + workspace.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../../include/rt_ffi.h"
#include "../device/scene_layout.h"
#include "kernels.h"

namespace rt {

// SoA path stream: one entry per live sample path. Paths are compacted (wave ballot + prefix
// count, one atomic per wave) from stream A into stream B every bounce, so both the extend and
// the shade kernel read their inputs with unit stride.
struct PathStream {
    double* ox; double* oy; double* oz;   // ray origin
    double* dx; double* dy; double* dz;   // ray direction
    double* bx; double* by; double* bz;   // throughput applied to R(next)
    double* lx; double* ly; double* lz;   // path radiance so far
    double* ex; double* ey; double* ez;   // throughput for the emission at the next hit (after a mirror)
    double* wx; double* wy; double* wz;   // the `o` argument carried across mirror bounces (scene.rs:178)
    double* pdf;                          // previous BSDF pdf (MIS only)
    uint64_t* r0; uint64_t* r1;           // RNG stream state of the sample
    int32_t* sub;                         // tile-local subpixel id
    int32_t* sample;                      // sample index within the subpixel
    int32_t* dk;                          // depth << 2 | kind
};

struct Workspace {
    int device = 0;
    unsigned long long* counters = nullptr;  // 8 x u64: [0] vertices
    // stream storage
    void* blob = nullptr;
    size_t slots = 0;
    bool mis = false;
    PathStream s[2]{};
    double* hit_t = nullptr;
    int32_t* hit_obj = nullptr;
    int32_t* hit_prim = nullptr;
    uint32_t* ctrl = nullptr;  // [0],[1] stream counts, [2] next subpixel, [3] spare, [4] |Q1|, [5] |Q2|, [6],[7] Q1/Q2 read heads
    // deferred mesh queries (scenes with meshes): Q1 = paths whose extension ray may hit a mesh,
    // Q2 = shadow rays the analytic objects let through that a mesh may still block
    int32_t* q1 = nullptr;
    int32_t* q2_pos = nullptr;   // the path's index in the output stream
    double* q2 = nullptr;        // [10][slots]: origin xyz, dir xyz, dist, weighted NEE term xyz
    double* sub_buf = nullptr; // subpixel means when the caller passes none
    size_t sub_cap = 0;
    double* tail_buf = nullptr;  // megakernel split tail (bytes: tail_cap)
    size_t tail_cap = 0;
    uint32_t* host_ctrl = nullptr;  // pinned mirror of ctrl
    hipEvent_t ev = nullptr;
    // Pool bookkeeping (rt_api.cpp: take_workspace / give_workspace): `busy` is recorded on the
    // render's stream after its last launch; the workspace is handed to another render only once
    // that event has completed, or to a render on the same stream (ordered after it anyway).
    hipEvent_t busy = nullptr;
    hipStream_t last_stream = nullptr;
    bool in_flight = false;

    hipError_t ensure_counters();
    hipError_t ensure_slots(size_t n);
    hipError_t ensure_sub(size_t pixels);
    hipError_t ensure_tail(size_t bytes);
    ~Workspace();
};

// Runs the whole render on `st`. Returns RT_OK / RT_CANCELLED / RT_E_*.
int wavefront_render_f64(const DevScene& sc, const RenderArgs& a, Workspace& ws, hipStream_t st,
                         const volatile int32_t* cancel, rt_render_stats* stats, std::string* err);

}  // namespace rt
