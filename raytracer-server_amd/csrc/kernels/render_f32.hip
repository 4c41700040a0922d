// f32 perf mode (RT_FLAG_FP32) for gfx950: the per-pixel sample loop of server.rs:320-364 and the
// estimator of scene.rs:152-244 in single precision, statistical parity with the f64 reference only
// (DESIGN.md §10). Same RNG streams and draw order as the f64 kernels (one xoroshiro128++ stream per
// camera sample, Philox-seeded; a draw is the top 24 bits of the same 64-bit output), so an f32
// frame tracks the f64 frame path for path until a rounding difference flips a branch.
//
// Differences from the f64 path (all inside the statistical tolerance, tests/test_gpu_parity.py):
//   * every hit point is offset by off32 * n (2^-16 of the scene's largest coordinate; the
//     reference offsets planes and triangles by 1e-5 * n and spheres not at all) — 1e-5 is about one
//     f32 ulp at the scenes' coordinates (~100) and would self-intersect;
//   * sphere roots by the cancellation-free form r^2 - |op - b d|^2 (geometry.rs:512-545 uses
//     b^2 - op.op + r^2, which loses ~all bits in f32 for rays leaving a sphere);
//   * diffuse and mirror throughput updates in closed form (kd / p, ks / p: the f cos / (pdf p) of
//     scene.rs:176-184 / :232-240 with pdf and cos cancelled);
//   * meshes are intersected with nearest-triangle semantics (geometry.rs:886-903, the
//     RT_FLAG_MESH_NEAREST branch): through the BVH with f32 boxes rounded outward, or, for meshes
//     of <= RenderArgs::f32_brute triangles, triangle by triangle from scalar loads.
// Layout of the work: a persistent resident grid, lanes pulling subpixels from one counter
// (wave-aggregated tickets); object loops over the scalar-loaded compact tables (Compact32);
// camera samples computed ahead into an LDS buffer in whole-wave passes.
// Supported: diffuse and mirror BRDFs, sphere lights, spheres / planes / meshes, MIS on or off —
// every reference scene. Phong and mesh lights are rejected on the host (rt_api.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../device/integrator_f64.h"  // Rng, subpixel_of (integer work shared with the f64 path)
#include "../ab_knobs.h"
#include "kernels.h"

#ifndef RT_F32_W
#define RT_F32_W 4       // waves/SIMD, analytic scenes
#endif
#ifndef RT_F32_REFILL
#define RT_F32_REFILL 24  // camera-buffer refill threshold (lanes per wave)
#endif
#ifndef RT_F32_W_MESH
#define RT_F32_W_MESH 8  // waves/SIMD, scenes with deep meshes
#endif

namespace rt {
namespace f32 {

#define RT_DEV32 __device__ __forceinline__

struct F3 {
    float x, y, z;
};
RT_DEV32 F3 f3(float x, float y, float z) { return F3{x, y, z}; }
RT_DEV32 F3 ld3f(const float* p) { return F3{p[0], p[1], p[2]}; }
RT_DEV32 F3 operator+(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_DEV32 F3 operator-(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_DEV32 F3 operator-(F3 a) { return f3(-a.x, -a.y, -a.z); }
RT_DEV32 F3 operator*(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }
RT_DEV32 F3 operator*(float s, F3 a) { return f3(a.x * s, a.y * s, a.z * s); }
RT_DEV32 F3 mult(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_DEV32 float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_DEV32 F3 cross(F3 a, F3 b) { return f3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
RT_DEV32 float rcp(float x) { return __builtin_amdgcn_rcpf(x); }  // 1 ulp
RT_DEV32 float sqrt_a(float x) { return __builtin_amdgcn_sqrtf(x); }  // v_sqrt_f32, 1 ulp (no denormal scaling)
RT_DEV32 F3 normalize(F3 a) { return a * __builtin_amdgcn_rsqf(dot(a, a)); }
RT_DEV32 bool is_zero(F3 a) { return a.x == 0.f && a.y == 0.f && a.z == 0.f; }

constexpr float INV_PI = 0.318309886183790671538f;
constexpr float EPS_T = 1e-4f;  // sphere / triangle t threshold (geometry.rs:518, :667)

// The object table through the constant address space: with a wave-uniform index (readfirstlane)
// the object loops read it with scalar loads instead of one vector load chain per object.
typedef const __attribute__((address_space(4))) Obj32 CObj;
RT_DEV32 CObj& obj_u(const DevScene& sc, int i) {
    return ((CObj*)sc.obj32)[__builtin_amdgcn_readfirstlane(i)];
}
RT_DEV32 F3 ld3c(const __attribute__((address_space(4))) float* p) { return F3{p[0], p[1], p[2]}; }

RT_DEV32 float uni(f64::Rng& r) { return (float)(uint32_t)(r.next() >> 40) * 0x1p-24f; }

struct Hit {
    float t;
    int obj, prim;  // prim: index into btris32 (mesh hits)
};

// Sphere::intersect (geometry.rs:512-545), cancellation-free discriminant.
RT_DEV32 bool sphere_t(CObj& o, F3 ro, F3 rd, float* t) {
    const F3 op = ld3c(o.pos) - ro;
    const float b = dot(op, rd);
    const F3 v = op - b * rd;
    const float det = o.r2 - dot(v, v);
    if (det < 0.f) return false;
    const float s = sqrt_a(det);
    float tt = b - s;
    if (tt > EPS_T) { *t = tt; return true; }
    tt = b + s;
    if (tt > EPS_T) { *t = tt; return true; }
    return false;
}
RT_DEV32 bool sphere_c(float cx, float cy, float cz, float r2, F3 ro, F3 rd, float* t) {
    const F3 op = f3(cx, cy, cz) - ro;
    const float b = dot(op, rd);
    const F3 v = op - b * rd;
    const float det = r2 - dot(v, v);
    if (det < 0.f) return false;
    const float s = sqrt_a(det);
    float tt = b - s;
    if (tt > EPS_T) { *t = tt; return true; }
    tt = b + s;
    if (tt > EPS_T) { *t = tt; return true; }
    return false;
}
// Plane::intersect (geometry.rs:547-571).
RT_DEV32 bool plane_t(CObj& o, F3 ro, F3 rd, float* t) {
    const F3 n = ld3c(o.n);
    const float dn = dot(rd, n);
    if (__builtin_fabsf(dn) < 1e-4f) return false;
    const float tt = dot(ld3c(o.pos) - ro, n) * rcp(dn);
    if (tt >= 0.f) { *t = tt; return true; }
    return false;
}
// Axis plane (n = +-e_K): dot(pos - o, n) / dot(d, n) = (pos_K - o_K) / d_K with the ray's reciprocal.
template <int K>
RT_DEV32 float comp(F3 v) { return K == 0 ? v.x : K == 1 ? v.y : v.z; }
template <int K>
RT_DEV32 bool axis_t(CObj& o, F3 ro, F3 rd, F3 inv, float* t) {
    if (__builtin_fabsf(comp<K>(rd)) < 1e-4f) return false;
    const float tt = (o.pos[K] - comp<K>(ro)) * comp<K>(inv);
    if (tt >= 0.f) { *t = tt; return true; }
    return false;
}
// Shadow segment x -> y against an axis plane: only a plane with x and y not strictly on one side
// can block (behind x its t < 0, beyond y its t > |y - x|).
template <int K>
RT_DEV32 bool axis_blocks(CObj& o, F3 x, F3 y, F3 rd, F3 inv, float lim) {
    const float sx = comp<K>(x) - o.pos[K], sy = comp<K>(y) - o.pos[K];
    if ((sx > 0.f && sy > 0.f) || (sx < 0.f && sy < 0.f)) return false;
    if (__builtin_fabsf(comp<K>(rd)) < 1e-4f) return false;
    const float tt = -sx * comp<K>(inv);
    return tt >= 0.f && tt < lim;
}
// Triangle::intersect (geometry.rs:637-670): Cramer's rule on (-d, ab, ac) as in the reference.
RT_DEV32 bool tri_t(const Tri32& tr, F3 ro, F3 rd, float* t) {
    const F3 n = ld3f(tr.n);
    if (__builtin_fabsf(dot(n, rd)) < 1e-4f) return false;
    const F3 ab = ld3f(tr.ab), ac = ld3f(tr.ac);
    const F3 b = ro - ld3f(tr.a);
    const F3 nd = -rd;
    const F3 abac = cross(ab, ac);
    const float det = dot(nd, abac);
    const float y = rcp(det);
    const float u = dot(nd, cross(b, ac)) * y;
    const float v = dot(nd, cross(ab, b)) * y;
    if (u < 0.f || u > 1.f || v < 0.f || u + v > 1.f) return false;
    const float tt = dot(b, abac) * y;
    if (tt > EPS_T) { *t = tt; return true; }
    return false;
}

struct RayF {
    F3 o, d, inv;
};
RT_DEV32 float safe_inv(float d) { return rcp(__builtin_fabsf(d) < 1e-30f ? __builtin_copysignf(1e-30f, d) : d); }
RT_DEV32 RayF make_ray(F3 o, F3 d) { return RayF{o, d, f3(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z))}; }

RT_DEV32 bool box_hit(const Bvh32& nd, const RayF& r, float tmax) {
    const float x0 = (nd.bmin[0] - r.o.x) * r.inv.x, x1 = (nd.bmax[0] - r.o.x) * r.inv.x;
    const float y0 = (nd.bmin[1] - r.o.y) * r.inv.y, y1 = (nd.bmax[1] - r.o.y) * r.inv.y;
    const float z0 = (nd.bmin[2] - r.o.z) * r.inv.z, z1 = (nd.bmax[2] - r.o.z) * r.inv.z;
    const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.f));
    const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), tmax));
    return tn <= tf;
}

// Per-lane BVH stack in LDS, one column per thread (blocks of 256).
__shared__ int32_t s_stack32[kBvhMaxDepth * 256];

// Nearest triangle of mesh m closer than *t (the Mesh::intersect `octree: None` loop,
// geometry.rs:886-903, accelerated). any_hit: stop at the first triangle closer than *t.
template <bool any_hit>
RT_DEV32 bool mesh_t(const DevScene& sc, int mesh, const RayF& r, float* t, int* prim, int brute) {
    typedef const __attribute__((address_space(4))) DevMesh CMesh;
    CMesh& m = ((CMesh*)sc.meshes)[__builtin_amdgcn_readfirstlane(mesh)];
    if (m.bvh_n <= 0) return false;
    if (m.n_tris <= brute) {
        // small mesh (the cubes' 12 triangles): root box, then every triangle, from scalar loads
        // (the same data for every lane); most rays miss the box
        typedef const __attribute__((address_space(4))) Bvh32 CBvh;
        CBvh& root = ((CBvh*)sc.bvh32)[__builtin_amdgcn_readfirstlane(m.bvh_base)];
        Bvh32 rn;
        for (int k = 0; k < 3; ++k) {
            rn.bmin[k] = root.bmin[k];
            rn.bmax[k] = root.bmax[k];
        }
        if (!box_hit(rn, r, *t)) return false;
        typedef const __attribute__((address_space(4))) Tri32 CTri;
        const int base = __builtin_amdgcn_readfirstlane(m.btri_base);
        bool found = false;
        float best = *t;
        for (int j = 0; j < m.n_tris; ++j) {
            CTri& c = ((CTri*)sc.btris32)[base + j];
            Tri32 tr;
            for (int k = 0; k < 3; ++k) {
                tr.a[k] = c.a[k];
                tr.ab[k] = c.ab[k];
                tr.ac[k] = c.ac[k];
                tr.n[k] = c.n[k];
            }
            float tt;
            if (tri_t(tr, r.o, r.d, &tt) && tt < best) {
                best = tt;
                *prim = base + j;
                found = true;
                if (any_hit) break;
            }
        }
        if (found) *t = best;
        return found;
    }
    __attribute__((address_space(3))) int32_t* stk = (__attribute__((address_space(3))) int32_t*)s_stack32 + threadIdx.x;
    int cur = m.bvh_base, sp = 0;
    bool found = false;
    float best = *t;
    while (true) {
        const Bvh32 nd = sc.bvh32[cur];
        if (box_hit(nd, r, best)) {
            const int cnt = nd.cnt_axis >> 2;
            if (cnt == 0) {
                const int axis = nd.cnt_axis & 3;
                const float dk = axis == 0 ? r.d.x : axis == 1 ? r.d.y : r.d.z;
                const int l = cur + 1, rr = nd.a;
                stk[sp * 256] = dk < 0.f ? l : rr;  // far child
                ++sp;
                cur = dk < 0.f ? rr : l;
                continue;
            }
            for (int k = 0; k < cnt; ++k) {
                float tt;
                if (tri_t(sc.btris32[nd.a + k], r.o, r.d, &tt) && tt < best) {
                    best = tt;
                    *prim = nd.a + k;
                    found = true;
                }
            }
            if (any_hit && found) break;
        }
        if (sp == 0) break;
        --sp;
        cur = stk[sp * 256];
    }
    if (found) *t = best;
    return found;
}

typedef const __attribute__((address_space(4))) Compact32 CTab32;
// Per-call view of the compact tables: the empty asm makes the pointer opaque, so their scalar
// loads are issued inside each trace call, not hoisted out of the path loop into ~60 live SGPRs.
RT_DEV32 CTab32& tables32(const DevScene& sc) {
    uint64_t p = (uint64_t)(uintptr_t)sc.ctab32;
    asm volatile("" : "+s"(p));
    return *(CTab32*)p;
}

// Nearest-hit update with the reference's tie rule (scene.rs:278: strict <, so ties go to the lower
// index) — needed because the compact tables visit objects grouped by type.
RT_DEV32 void consider(Hit& h, float t, int idx) {
    if (t < h.t || (t == h.t && idx < h.obj)) { h.t = t; h.obj = idx; h.prim = -1; }
}
template <int K>
RT_DEV32 void axis_planes(CTab32& T, const RayF& r, Hit& h) {
    if (__builtin_fabsf(comp<K>(r.d)) < 1e-4f) return;
#pragma unroll
    for (int j = 0; j < kMaxAxisPlanes; ++j) {
        if (j < T.n_ax[K]) {
            const float tt = (T.ax_pos[K][j] - comp<K>(r.o)) * comp<K>(r.inv);
            if (tt >= 0.f) consider(h, tt, T.ax_idx[K][j]);
        }
    }
}
template <int K>
RT_DEV32 bool axis_planes_block(CTab32& T, const RayF& r, F3 y, float lim) {
#pragma unroll
    for (int j = 0; j < kMaxAxisPlanes; ++j) {
        if (j < T.n_ax[K]) {
            const float p = T.ax_pos[K][j];
            const float sx = comp<K>(r.o) - p, sy = comp<K>(y) - p;
            if (!((sx > 0.f && sy > 0.f) || (sx < 0.f && sy < 0.f)) && __builtin_fabsf(comp<K>(r.d)) >= 1e-4f) {
                const float tt = -sx * comp<K>(r.inv);
                if (tt >= 0.f && tt < lim) return true;
            }
        }
    }
    return false;
}

template <bool MESH>
RT_DEV32 void generic_closest(const DevScene& sc, CObj& o, int i, const RayF& r, Hit& h, int brute);

// Scene::trace_ray (scene.rs:272-289): nearest over all objects, strict < in index order.
template <bool MESH>
RT_DEV32 Hit trace_closest(const DevScene& sc, const RayF& r, int brute) {
    Hit h{3.0e38f, -1, -1};
    CTab32& T = tables32(sc);
    if (T.ok) {  // compact scene: unrolled per-type tables (one scalar-load batch)
        axis_planes<0>(T, r, h);
        axis_planes<1>(T, r, h);
        axis_planes<2>(T, r, h);
#pragma unroll
        for (int j = 0; j < kMaxSpheres; ++j) {
            float t;
            if (j < T.n_sph && sphere_c(T.sph[j][0], T.sph[j][1], T.sph[j][2], T.sph[j][3], r.o, r.d, &t))
                consider(h, t, T.sph_idx[j]);
        }
        for (int j = 0; j < T.n_gen; ++j) {
            const int i = T.gen_idx[j];
            generic_closest<MESH>(sc, obj_u(sc, i), i, r, h, brute);
        }
        return h;
    }
    for (int i = 0; i < sc.n_objects; ++i) {
        CObj& o = obj_u(sc, i);
        float t;
        if (o.geom == GEOM_SPHERE) {
            if (sphere_t(o, r.o, r.d, &t) && t < h.t) { h.t = t; h.obj = i; }
        } else if (o.geom == GEOM_PLANE) {
            const int ax = o.axis;
            bool hit;
            if (ax == 0) hit = axis_t<0>(o, r.o, r.d, r.inv, &t);
            else if (ax == 1) hit = axis_t<1>(o, r.o, r.d, r.inv, &t);
            else if (ax == 2) hit = axis_t<2>(o, r.o, r.d, r.inv, &t);
            else hit = plane_t(o, r.o, r.d, &t);
            if (hit && t < h.t) { h.t = t; h.obj = i; }
        } else if constexpr (MESH) {
            t = h.t;
            int prim = -1;
            if (mesh_t<false>(sc, o.mesh, r, &t, &prim, brute) && t < h.t) { h.t = t; h.obj = i; h.prim = prim; }
        }
    }
    return h;
}

// Scene::mutually_visible (scene.rs:250-270) as an any-hit query: blocked iff some object's hit
// satisfies t + 0.001 < |y - x|.
template <bool MESH>
RT_DEV32 bool generic_blocks(const DevScene& sc, CObj& o, const RayF& r, float lim, int brute);

template <bool MESH>
RT_DEV32 bool visible(const DevScene& sc, const RayF& r, F3 y, float dist, int brute) {
    const float lim = dist - 0.001f;
    CTab32& T = tables32(sc);
    if (T.ok) {
        if (axis_planes_block<0>(T, r, y, lim) || axis_planes_block<1>(T, r, y, lim) ||
            axis_planes_block<2>(T, r, y, lim))
            return false;
#pragma unroll
        for (int j = 0; j < kMaxSpheres; ++j) {
            float t;
            if (j < T.n_sph && sphere_c(T.sph[j][0], T.sph[j][1], T.sph[j][2], T.sph[j][3], r.o, r.d, &t) && t < lim)
                return false;
        }
        for (int j = 0; j < T.n_gen; ++j)
            if (generic_blocks<MESH>(sc, obj_u(sc, T.gen_idx[j]), r, lim, brute)) return false;
        return true;
    }
    for (int i = 0; i < sc.n_objects; ++i) {
        CObj& o = obj_u(sc, i);
        float t;
        if (o.geom == GEOM_SPHERE) {
            if (sphere_t(o, r.o, r.d, &t) && t < lim) return false;
        } else if (o.geom == GEOM_PLANE) {
            const int ax = o.axis;
            if (ax == 0) {
                if (axis_blocks<0>(o, r.o, y, r.d, r.inv, lim)) return false;
            } else if (ax == 1) {
                if (axis_blocks<1>(o, r.o, y, r.d, r.inv, lim)) return false;
            } else if (ax == 2) {
                if (axis_blocks<2>(o, r.o, y, r.d, r.inv, lim)) return false;
            } else if (plane_t(o, r.o, r.d, &t) && t < lim) {
                return false;
            }
        } else if constexpr (MESH) {
            t = lim;
            int prim;
            if (lim > 0.f && mesh_t<true>(sc, o.mesh, r, &t, &prim, brute)) return false;
        }
    }
    return true;
}

// Objects outside the compact tables: meshes and planes that are not axis-aligned.
template <bool MESH>
RT_DEV32 void generic_closest(const DevScene& sc, CObj& o, int i, const RayF& r, Hit& h, int brute) {
    float t;
    if (o.geom == GEOM_PLANE) {
        if (plane_t(o, r.o, r.d, &t)) consider(h, t, i);
    } else if constexpr (MESH) {
        if (o.geom == GEOM_MESH) {
            t = h.t;
            int prim = -1;
            if (mesh_t<false>(sc, o.mesh, r, &t, &prim, brute) && (t < h.t || (t == h.t && i < h.obj))) {
                h.t = t;
                h.obj = i;
                h.prim = prim;
            }
        }
    }
}
template <bool MESH>
RT_DEV32 bool generic_blocks(const DevScene& sc, CObj& o, const RayF& r, float lim, int brute) {
    float t;
    if (o.geom == GEOM_PLANE) return plane_t(o, r.o, r.d, &t) && t < lim;
    if constexpr (MESH) {
        if (o.geom == GEOM_MESH && lim > 0.f) {
            t = lim;
            int prim;
            return mesh_t<true>(sc, o.mesh, r, &t, &prim, brute);
        }
    }
    return false;
}

enum : int { K_CAMERA = 0, K_SPEC = 1, K_DIFF = 2 };

struct Path {
    F3 ro, rd, beta, L, bemit, o;
    float pdf_prev;
    uint64_t r0, r1;
    uint32_t depth;
    int kind;
};

struct Cam {
    F3 pos, dir, cx, cy;
    float rw, rh;  // 1 / width, 1 / height
};

// sample_pixel's camera ray (server.rs:338-357) for sample `smp` of tile subpixel `id`: its
// direction and the sample's RNG stream after the two camera draws.
RT_DEV32 void camera_sample(const Cam& cam, const RenderArgs& a, long id, int smp, F3& rd, uint64_t& r0,
                            uint64_t& r1) {
    const f64::SubPixel sp = f64::subpixel_of(a, id);
    f64::Rng rng(a.seed, sp.pid, (uint32_t)smp, (uint32_t)sp.sub);
    const float u1 = uni(rng), u2 = uni(rng);
    const float r1f = 2.f * u1, r2f = 2.f * u2;
    const float dx = r1f < 1.f ? sqrt_a(r1f) - 1.f : 1.f - sqrt_a(2.f - r1f);
    const float dy = r2f < 1.f ? sqrt_a(r2f) - 1.f : 1.f - sqrt_a(2.f - r2f);
    const F3 d = cam.cx * ((((float)sp.sx + 0.5f + dx) * 0.5f + (float)sp.col) * cam.rw - 0.5f) +
                 cam.cy * ((((float)sp.sy + 0.5f + dy) * 0.5f + (float)sp.yref) * cam.rh - 0.5f) + cam.dir;
    rd = normalize(d);
    r0 = rng.s0;
    r1 = rng.s1;
}
RT_DEV32 void begin_path(const Cam& cam, F3 rd, uint64_t r0, uint64_t r1, Path& ps) {
    ps.ro = cam.pos;
    ps.rd = rd;
    ps.r0 = r0;
    ps.r1 = r1;
    ps.beta = f3(1.f, 1.f, 1.f);
    ps.L = f3(0.f, 0.f, 0.f);
    ps.bemit = f3(0.f, 0.f, 0.f);
    ps.o = f3(0.f, 0.f, 0.f);
    ps.pdf_prev = 0.f;
    ps.depth = 0;
    ps.kind = K_CAMERA;
}

// One path vertex (integrator_f64.h: shade_vertex, same walk and draw order). Returns true when the
// path continues with ps.ro / ps.rd.
template <bool MESH, bool MIS>
RT_DEV32 bool shade(const DevScene& sc, Path& ps, const Hit& h, float light_pdf, int brute) {
    if (h.obj < 0) return false;
    const Obj32& obj = sc.obj32[h.obj];
    F3 x = ps.ro + h.t * ps.rd, n;
    if (obj.geom == GEOM_SPHERE) n = normalize(x - ld3f(obj.pos));
    else if (obj.geom == GEOM_PLANE) n = ld3f(obj.n);
    else n = ld3f(sc.btris32[h.prim].n);
    if (dot(n, ps.rd) > 0.f) n = -n;  // normal toward the incoming side (geometry.rs:535, :566, :669)
    x = x + n * sc.off32;
    const F3 Le = ld3f(obj.emitted);
    if (ps.kind == K_CAMERA) {
        ps.L = Le;
    } else if (ps.kind == K_SPEC) {
        ps.L = ps.L + mult(ps.bemit, Le);
    } else if (MIS && h.obj == sc.light && ps.pdf_prev > 0.f) {
        const float cosl = -dot(n, ps.rd);
        const float pdf_l = light_pdf * (h.t * h.t) * rcp(cosl);
        ps.L = ps.L + mult(ps.beta, Le * (ps.pdf_prev * rcp(ps.pdf_prev + pdf_l)));
    }
    if (ps.kind != K_SPEC) ps.o = -ps.rd;
    ps.depth += 1;
    const float p = ps.depth <= (uint32_t)f64::MAX_BOUNCES ? 1.f : (float)f64::SURVIVAL_PROBABILITY;
    f64::Rng rng(ps.r0, ps.r1);
    const bool spec = obj.brdf == BRDF_SPECULAR;
    const F3 k = ld3f(obj.k);
    if (!spec) {
        // next-event estimation to the sphere light (scene.rs:217-229, geometry.rs:573-585)
        CObj& Lo = obj_u(sc, sc.light);
        const float xi1 = uni(rng), xi2 = uni(rng);
        const float z = 2.f * xi1 - 1.f;
        float sphi, cphi;
        __sincosf(6.283185307179586f * xi2, &sphi, &cphi);
        const float sz = sqrt_a(fmaxf(0.f, 1.f - z * z));
        const F3 ny = f3(sz * cphi, sz * sphi, z);
        const F3 y = ld3c(Lo.pos) + ny * Lo.r;
        const F3 diff = y - x;
        const float r_sqr = dot(diff, diff);
        const float dist = sqrt_a(r_sqr);
        const F3 i = diff * rcp(dist);
        const F3 lef = mult(ld3c(Lo.emitted), k) * INV_PI;
        if (!is_zero(lef)) {
            const bool vis = visible<MESH>(sc, make_ray(x, i), y, dist, brute);
            const float cosx = dot(n, i), cosl = -dot(ny, i);
            F3 c = f3(0.f, 0.f, 0.f);
            if (!MIS) {
                if (vis) c = lef * (cosx * cosl * rcp(r_sqr * light_pdf));
            } else {
                const float pdf_l = light_pdf * r_sqr * rcp(cosl);
                const float pdf_b = cosx * INV_PI;
                if (vis && cosl > 0.f && pdf_b > 0.f) c = lef * (cosx * rcp(pdf_l + pdf_b));
            }
            ps.L = ps.L + mult(ps.beta, c);
        }
    }
    // Russian roulette + BSDF continuation (scene.rs:173-184 / :231-242)
    if (!(uni(rng) < p)) return false;
    F3 wi;
    float pdf = 0.f;
    if (!spec) {
        const float z = sqrt_a(uni(rng));
        const float rr = sqrt_a(fmaxf(0.f, 1.f - z * z));
        float sphi, cphi;
        __sincosf(6.283185307179586f * uni(rng), &sphi, &cphi);
        // create_local_coord (scene.rs:112-123)
        const F3 base = __builtin_fabsf(n.x) > 0.1f ? f3(0.f, 1.f, 0.f) : f3(1.f, 0.f, 0.f);
        const F3 u = normalize(cross(base, n));
        const F3 v = cross(n, u);
        wi = normalize(u * (rr * cphi) + v * (rr * sphi) + n * z);
        pdf = dot(n, wi) * INV_PI;
    } else {
        wi = (2.f * dot(ps.o, n)) * n - ps.o;  // o.flip_across(n) (scene.rs:50-54)
        ps.bemit = ps.beta;
    }
    ps.r0 = rng.s0;
    ps.r1 = rng.s1;
    ps.beta = mult(ps.beta, k) * rcp(p);
    ps.ro = x;
    ps.rd = wi;
    ps.kind = spec ? K_SPEC : K_DIFF;
    ps.pdf_prev = MIS && !spec ? pdf : 0.f;
    return spec || !is_zero(ps.beta);
}

RT_DEV32 long wave_ticket(uint32_t* counter, bool want) {
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

// Persistent path loop: a resident grid whose lanes take subpixels from a global counter and walk
// their spp/4 samples vertex by vertex (a finished sample starts the next one in the next
// iteration). The subpixel mean is written in f64 for k_finalize_f64 (clamp, gamma, `as u8`).
template <bool MESH, bool MIS, int W>
__global__ __launch_bounds__(256, W) void k_megakernel_f32(DevScene sc, RenderArgs a, double* __restrict__ sub_buf,
                                                       uint32_t* next_sub, long nsub, int unit) {
    Cam cam;
    cam.pos = f3((float)sc.cam_pos[0], (float)sc.cam_pos[1], (float)sc.cam_pos[2]);
    cam.dir = f3((float)sc.cam_dir[0], (float)sc.cam_dir[1], (float)sc.cam_dir[2]);
    cam.cx = f3((float)a.cx[0], (float)a.cx[1], (float)a.cx[2]);
    cam.cy = f3((float)a.cy[0], (float)a.cy[1], (float)a.cy[2]);
    cam.rw = (float)(1.0 / a.width);
    cam.rh = (float)(1.0 / a.height);
    const float light_pdf = (float)sc.light_pdf;
    uint32_t nverts = 0;
    // a ticket is a run of `unit` consecutive subpixels (fewer atomics on the one counter at low spp,
    // render_f64.hip: plan_units)
    const long nunits = (nsub + unit - 1) / unit;
    long t0 = wave_ticket(next_sub, true);
    long id = t0 * unit, end = min(id + unit, nsub);
    bool active = t0 < nunits;
    int smp = 0;
    F3 acc = f3(0.f, 0.f, 0.f);
    Path ps;
    // Camera-sample buffer (one per lane, LDS): the next sample's ray + RNG state computed ahead in
    // a camera pass the whole wave runs once >= RT_F32_REFILL lanes have an empty slot (or some lane
    // must start a path without one), instead of a Philox + camera pass at ~7% lane utilisation in
    // almost every iteration. Off for the 8-wave deep-mesh kernel (its LDS holds the BVH stacks).
    constexpr bool BUF = W <= 6;
    __shared__ float s_cd[BUF ? 3 * 256 : 1];
    __shared__ uint64_t s_cr[BUF ? 2 * 256 : 1];
    bool nb = false;  // slot holds sample smp + 1 of subpixel id
    bool start = active;
    while (__any(active)) {
        bool finished = false;
        if (active && !start) {
            const Hit h = trace_closest<MESH>(sc, make_ray(ps.ro, ps.rd), a.f32_brute);
            nverts += h.obj >= 0;
            if (!shade<MESH, MIS>(sc, ps, h, light_pdf, a.f32_brute)) {
                acc = acc + ps.L;
                if (++smp < a.n_samples) {
                    if (BUF && nb) {
                        const int l = threadIdx.x;
                        begin_path(cam, f3(s_cd[l], s_cd[256 + l], s_cd[512 + l]), s_cr[l], s_cr[256 + l], ps);
                        nb = false;
                    } else {
                        start = true;
                    }
                } else {
                    double* o = sub_buf + (size_t)id * 3;
                    o[0] = (double)acc.x * a.inv_n;
                    o[1] = (double)acc.y * a.inv_n;
                    o[2] = (double)acc.z * a.inv_n;
                    if (++id < end) {  // the next subpixel of the run
                        smp = 0;
                        acc = f3(0.f, 0.f, 0.f);
                        start = true;
                        nb = false;
                    } else {
                        finished = true;
                    }
                }
            }
        }
        const long t = wave_ticket(next_sub, finished && !(a.cancel && *(const volatile int32_t*)a.cancel));
        if (finished) {
            if (t >= 0 && t < nunits) {
                id = t * unit;
                end = min(id + unit, nsub);
                smp = 0;
                acc = f3(0.f, 0.f, 0.f);
                start = true;
                nb = false;
            } else {
                active = false;
            }
        }
        bool fill = false;
        if constexpr (BUF) {
            fill = active && !start && !nb && smp + 1 < a.n_samples;
            if (!__any(start) && __popcll(__ballot(fill)) < RT_F32_REFILL) fill = false;
        }
        if (start || fill) {  // camera pass: paths that start now, then buffer refills
            F3 rd;
            uint64_t r0, r1;
            camera_sample(cam, a, id, start ? smp : smp + 1, rd, r0, r1);
            if (start) {
                begin_path(cam, rd, r0, r1, ps);
            } else {
                const int l = threadIdx.x;
                s_cd[l] = rd.x;
                s_cd[256 + l] = rd.y;
                s_cd[512 + l] = rd.z;
                s_cr[l] = r0;
                s_cr[256 + l] = r1;
                nb = true;
            }
            start = false;
        }
    }
    if (a.counters) {
        unsigned long long v = nverts;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (__lane_id() == 0 && v) atomicAdd(a.counters, v);
    }
}

template <bool MESH, bool MIS, int W>
static hipError_t launch_w(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                           hipStream_t st) {
    auto kern = k_megakernel_f32<MESH, MIS, W>;
    int dev = 0, ncu = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    const long blocks = std::max(1L, std::min((long)ncu * per_cu, (nsub + 255) / 256));
    // about 256 samples per ticket, at least 16 tickets per resident lane (render_f64.hip: plan_units)
    const long unit = std::max(1L, std::min((long)std::max(1, 256 / std::max(1, a.n_samples)), nsub / (blocks * 256 * 16)));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, sc, a, sub_buf, next_sub, nsub, (int)unit);
    return hipGetLastError();
}

// waves/SIMD requested from the register allocator (RT_F32_WAVES overrides for A/B runs)
template <bool MESH, bool MIS>
static hipError_t launch_k(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub, long nsub,
                           hipStream_t st) {
    static const int env = (int)ab_knob("RT_F32_WAVES", 0);
    // deep meshes (the unicorn's BVH walks) hide their node-load latency with more waves:
    // 8 waves/SIMD +12% there, cubes and cornell -20% (profiles/r01h_fp32.log)
    const int w = env ? env : (MESH && a.mesh_nodes >= 64 ? RT_F32_W_MESH : RT_F32_W);
    if (w >= 8) return launch_w<MESH, MIS, 8>(sc, a, sub_buf, next_sub, nsub, st);
    if (w >= 6) return launch_w<MESH, MIS, 6>(sc, a, sub_buf, next_sub, nsub, st);
    return launch_w<MESH, MIS, 4>(sc, a, sub_buf, next_sub, nsub, st);
}

}  // namespace f32

hipError_t launch_megakernel_f32(const DevScene& sc, const RenderArgs& a, double* sub_buf, uint32_t* next_sub,
                                 hipStream_t st) {
    const long nsub = (long)a.tw * a.th * 4;
    if (nsub <= 0 || a.n_samples <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(next_sub, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const bool mesh = (a.features & 1) != 0, mis = a.mis != 0;
    if (mesh) return mis ? f32::launch_k<true, true>(sc, a, sub_buf, next_sub, nsub, st)
                         : f32::launch_k<true, false>(sc, a, sub_buf, next_sub, nsub, st);
    return mis ? f32::launch_k<false, true>(sc, a, sub_buf, next_sub, nsub, st)
               : f32::launch_k<false, false>(sc, a, sub_buf, next_sub, nsub, st);
}

}  // namespace rt
