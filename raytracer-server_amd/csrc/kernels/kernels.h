// Host-visible launchers of the HIP kernels (implemented in *.hip, called by rt_api.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device/scene_layout.h"

namespace rt {

struct RenderArgs {
    int32_t width, height, x0, y0, tw, th;
    int32_t n_samples;  // spp / 4 per subpixel
    int32_t mis;
    int32_t features;  // Cfg<F> bits: 1 mesh, 2 phong, 4 mis, 8 compact, 16 nearest-triangle meshes (BVH),
                       // 32 no mirror (specular) object (the query-pool kernel's Cfg; the others ignore it)
    int32_t mesh_nodes;  // octree nodes of the largest mesh (megakernel choice)
    int32_t row_step;    // tile row i = screen row y0 + i * row_step
    int32_t tail_cps;    // split tail: chunks per subpixel
    // split tail (megakernels): subpixels [n_whole, nsub) are handed out as chunks of 2^chunk_lg
    // samples; a chunk's lane stores each sample's radiance in tail_buf[sub - n_whole][sample][3]
    // (megakernel_common.h tail_store) and k_tail_sum adds them up in sample order afterwards (the same
    // sequential sum)
    int32_t n_whole, chunk_lg;
    // whole subpixels are handed out in runs of unit_subs consecutive subpixels per ticket (n_wunits
    // tickets): at low spp a ticket per subpixel makes the one global counter's atomics the bottleneck
    int32_t unit_subs, n_wunits;
    uint64_t seed;
    double cx[3], cy[3];  // camera frame (server.rs:330-331), computed on the host
    double inv_n;         // 1.0 / n_samples (server.rs:358)
    double* sub_out;      // optional [pix][4][3]
    uint8_t* rgb_out;     // [pix][3]
    unsigned long long* counters;  // optional [0] = path vertices
    const int32_t* cancel;         // optional device view of the host cancel flag (mapped memory)
    double* tail_buf;              // split-tail sample radiance (see n_whole)
    int32_t f32_brute;             // f32 mode: meshes of <= f32_brute triangles are tested without the BVH
    int32_t all_flat;              // every mesh is a flat octree (DevMesh::flat) and there are <= 2 of them
};

// The split tail the calling thread's last megakernel launch planned (plan_tail): subpixels split into
// chunks, the split the kernel family wanted before the scratch buffer capped it, samples per chunk.
// Thread-local: a render is planned and enqueued on its caller's thread (rt_debug_last_split, rt_diag.h).
struct TailPlan {
    long n_split = 0, want = 0, chunk = 0;
};
extern thread_local TailPlan t_tail_plan;
// Subpixels the analytic and flat-mesh megakernels split per resident lane, x2 (plan_tail's split_x2): one and a
// half per lane, two for frames of up to 4 subpixels per lane (an N = 8 rank share). The tail's chunks must outlast
// the last whole subpixels, and a subpixel can cost 1.35x the average (its paths' lengths): in a share of ~4
// subpixels per lane the last whole ones started at 2/3 of the launch and ended 6 ms after every other wave
// (profiles/r06h_end_probe_waves.log); in the full cornell frame with half a subpixel per lane split, the last
// waves ended 15 ms after the median one, each behind a whole subpixel taken 59 ms before its end
// (profiles/r06ah_end_probe_waves.log). Cornell N = 8 share: 1864.6 (0.5 per lane) -> 1903.4 (1.5,
// profiles/r06u_ab_tail.log) -> 1909.1 (2; 2.5: 1910.7, profiles/r06y_ab_tail_n8.log) Msamples/s; full frames at
// 0.5 -> 1.5 per lane: cornell 1988.3 -> 2003.8 (2: 2001.2, profiles/r06ai_ab_tail_full.log), cubes 1079.5 -> 1085.5,
// N = 2 shares cornell 1963.9 -> 1987.8 and cubes 1067.5 -> 1079.7 (profiles/r06aj_ab_tail_full.log).
// rt_api.cpp sizes the split-tail scratch with the same rule.
inline int tail_split_x2(long nsub, long lanes) { return nsub <= 4 * lanes ? 4 : 3; }
// Split-tail scratch bytes per split subpixel (megakernel_common.h plan_tail: the samples after chunk 0).
size_t tail_scratch_per_subpixel(int n_samples);
// tail_buf / tail_cap: scratch for the split tail (bytes); the launcher sizes the tail to fit it.
hipError_t launch_megakernel_f64(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                 double* tail_buf, size_t tail_cap, hipStream_t st);
// Query-pool kernel for flat-octree mesh scenes (render_flat_f64.hip); called by
// launch_megakernel_f64 after the ticket counter is reset.
hipError_t launch_megakernel_flat_f64(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                      double* tail_buf, size_t tail_cap, int refill, hipStream_t st);
// Deep-octree mesh megakernel (render_mesh_f64.hip, walk pool); called by launch_megakernel_f64 after
// the ticket counter is reset; a: the caller's args (features, sizes), planned here.
hipError_t launch_megakernel_mesh_f64(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                      long nsub, int refill, int wmin, double* tail_buf, size_t tail_cap, hipStream_t st);
// Diagnostic symbols of each kernel code object (diag_tu.h): read, add to the outputs, clear.
int diag_read_main(unsigned long long* cnt16, unsigned long long* reg32, unsigned long long* tim16, unsigned long long* q4);
int diag_read_mesh(unsigned long long* cnt16, unsigned long long* reg32, unsigned long long* tim16, unsigned long long* q4);
int diag_read_flat(unsigned long long* cnt16, unsigned long long* reg32, unsigned long long* tim16, unsigned long long* q4);
// f32 perf mode (render_f32.hip): writes the subpixel means to sub_buf like the f64 megakernel.
hipError_t launch_megakernel_f32(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                 hipStream_t st);
hipError_t launch_finalize_f64(const RenderArgs& a, const double* sub_buf, hipStream_t st);
hipError_t launch_trace_f64(const DevScene& sc, long n, const double* o, const double* d, double* t, int32_t* obj,
                            double* pos, double* nrm, bool mesh_nearest, hipStream_t st);

}  // namespace rt
