// f64 render kernels for gfx950 (CDNA4).
//
//   k_megakernel_f64  — fused path loop: one lane owns one subpixel (server.rs:335-336) and walks
//                       its spp/4 sample paths vertex by vertex; a lane whose path ends starts its
//                       next sample in the same iteration (regeneration), so a wave idles only in
//                       the final tail. Accumulation per subpixel is sequential in sample order,
//                       exactly the reference's order (server.rs:338-358).
//   k_trace_f64       — Scene::trace_ray for a batch of rays (parity tests of the intersectors).
//   wavefront kernels — see wavefront_f64.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../device/integrator_f64.h"
#include "kernels.h"

namespace rt {
using namespace f64;

// Per-pixel finalisation from the 4 subpixel means held by 4 consecutive lanes
// (server.rs:360 clamp-then-average, :366-368 gamma, :187-189 `as u8`).
__device__ __forceinline__ void finalize_pixel(V3 acc, int lane, bool valid, uint8_t* rgb, size_t pix) {
    int base = lane & ~3;
    V3 pixel = v3(0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        V3 a = v3(__shfl(acc.x, base + j, 64), __shfl(acc.y, base + j, 64), __shfl(acc.z, base + j, 64));
        pixel = pixel + clampv(a, 0., 1.) * 0.25;
    }
    if (valid && (lane & 3) == 0) {
        V3 c = clampv(pixel, 0., 1.);
        const double g = 1.0 / 2.2;
        V3 gc = v3(pow(c.x, g), pow(c.y, g), pow(c.z, g)) * 255.0 + v3(0.5, 0.5, 0.5);
        rgb[pix * 3 + 0] = as_u8(gc.x);
        rgb[pix * 3 + 1] = as_u8(gc.y);
        rgb[pix * 3 + 2] = as_u8(gc.z);
    }
}

// W = minimum waves per SIMD requested from the register allocator (0: compiler's choice).
template <int F, int W>
__global__ __launch_bounds__(256, W) void k_megakernel_f64(DevScene sc, RenderArgs a) {
    using C = Cfg<F>;
    const int lane = threadIdx.x & 63;
    const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long npix = (long)a.tw * a.th;
    const long pix = q >> 2;
    const bool valid = pix < npix;
    const SubPixel sp = subpixel_of(a, valid ? q : 0);

    V3 acc = v3(0, 0, 0);
    unsigned long long nverts = 0;
    const int n = valid ? a.n_samples : 0;
    int s = 0;
    PathState ps;
    bool fresh = true;
    while (s < n) {
        if (fresh) begin_sample(sc, a, sp, s, ps);
        HitRec hr = trace_closest<C>(sc, ps.ray);
        nverts += hr.obj >= 0;
        fresh = !shade_vertex<C>(sc, a, sp, s, ps, hr);
        if (fresh) {
            acc = acc + ps.L * a.inv_n;  // server.rs:357-358
            ++s;
        }
    }
    if (valid && a.sub_out) {
        double* so = a.sub_out + ((size_t)pix * 4 + sp.sub) * 3;
        so[0] = acc.x;
        so[1] = acc.y;
        so[2] = acc.z;
    }
    finalize_pixel(acc, lane, valid, a.rgb_out, (size_t)pix);
    if (a.counters) {
        unsigned long long v = nverts;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) atomicAdd(a.counters, v);
    }
}

__global__ __launch_bounds__(256) void k_trace_f64(DevScene sc, long n, const double* __restrict__ o,
                                                   const double* __restrict__ d, double* t, int32_t* obj,
                                                   double* pos, double* nrm) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r{v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2])};
    HitRec h = trace_closest<Cfg<1>>(sc, r);
    obj[i] = h.obj;
    t[i] = h.obj >= 0 ? h.t : 0.0;
    if (h.obj >= 0) {
        V3 p, nn;
        surface<Cfg<1>>(sc, r, h, &p, &nn);
        pos[3 * i] = p.x; pos[3 * i + 1] = p.y; pos[3 * i + 2] = p.z;
        nrm[3 * i] = nn.x; nrm[3 * i + 1] = nn.y; nrm[3 * i + 2] = nn.z;
    }
}

hipError_t launch_megakernel_f64(const DevScene& sc, const RenderArgs& a, hipStream_t st) {
    long lanes = (long)a.tw * a.th * 4;
    if (lanes <= 0) return hipSuccess;
    long blocks = (lanes + 255) / 256;
    dim3 g((unsigned)blocks), b(256);
    // 4 waves/SIMD (128 VGPRs, a few spills) measured fastest on every scene (profiles/r01_ab_waves.log);
    // RT_MK_WAVES=2 or 1 selects the compiler's own allocation for A/B runs.
    static const int waves = [] {
        const char* v = std::getenv("RT_MK_WAVES");
        return v ? std::atoi(v) : 4;
    }();
#define RT_MK_CASE(F)                                                                         \
    case F:                                                                                   \
        if (waves == 4) hipLaunchKernelGGL((k_megakernel_f64<F, 4>), g, b, 0, st, sc, a);     \
        else if (waves == 2) hipLaunchKernelGGL((k_megakernel_f64<F, 2>), g, b, 0, st, sc, a); \
        else hipLaunchKernelGGL((k_megakernel_f64<F, 1>), g, b, 0, st, sc, a);                \
        break;
    switch (a.features & 7) {
        RT_MK_CASE(0) RT_MK_CASE(1) RT_MK_CASE(2) RT_MK_CASE(3)
        RT_MK_CASE(4) RT_MK_CASE(5) RT_MK_CASE(6) RT_MK_CASE(7)
    }
#undef RT_MK_CASE
    return hipGetLastError();
}

hipError_t launch_trace_f64(const DevScene& sc, long n, const double* o, const double* d, double* t, int32_t* obj,
                            double* pos, double* nrm, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_trace_f64, dim3((unsigned)blocks), dim3(256), 0, st, sc, n, o, d, t, obj, pos, nrm);
    return hipGetLastError();
}

}  // namespace rt
