// f64 device path: the reference's hot path (server.rs:320-368, scene.rs:30-289,
// geometry.rs:512-670, 977-1036, 1237-1295) restated for CDNA4 lanes.
//
// Compiled with -ffp-contract=off: every expression keeps the reference's operation order, so a
// lane produces the same f64 bits as the reference's arithmetic (and the oracle) except where
// device libm (sin/cos/pow) differs by an ulp from the host's.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "scene_layout.h"

namespace rt {
namespace f64 {

#define RT_DEV __device__ __forceinline__

constexpr double PI = 3.14159265358979323846264338327950288;
constexpr double FRAC_1_PI = 0.318309886183790671537767526745028724;
constexpr int MAX_BOUNCES = 5;               // scene.rs:109
constexpr double SURVIVAL_PROBABILITY = 0.9;  // scene.rs:110

struct V3 {
    double x, y, z;
};
RT_DEV V3 v3(double x, double y, double z) { return V3{x, y, z}; }
template <class P>
RT_DEV V3 ld3(P p) { return V3{p[0], p[1], p[2]}; }  // any address space (scalar-loaded tables too)
RT_DEV V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_DEV V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_DEV V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
RT_DEV V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
RT_DEV V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
// ---- correctly rounded division with a shared divisor ----
// q = RN(a / b) from y = RN(1 / b): q0 = RN(a y), r = a - b q0 (exact, FMA), q = RN(q0 + r y)
// (Markstein's theorem; valid without overflow/underflow). Used only when |b| is in
// [2^-900, 2^900]; otherwise, and for NaN/inf, the plain IEEE division is taken. The sign of a
// zero quotient is restored from q0 (see qdiv). Bit-identical to a / b for finite a.
#ifndef RT_OPT_VOTE
#define RT_OPT_VOTE 1
#endif
RT_DEV bool rcp_safe(double b) { return fabs(b) >= 0x1p-900 && fabs(b) <= 0x1p900; }
// All active lanes satisfy p (a wave vote kept in SGPRs: ballot vs exec, no VGPR round trip).
RT_DEV bool wave_all(bool p) {
#if RT_OPT_VOTE
    return __builtin_amdgcn_ballot_w64(p) == __builtin_amdgcn_read_exec();
#else
    return __all(p);
#endif
}
// RN(1 / b) for rcp_safe(b): the compiler's own IEEE f64 division sequence for 1.0 / b (v_rcp_f64,
// two Newton steps, residual correction) without its range scaling (v_div_scale) and special-case
// fixup (v_div_fixup), both identities in that range (every intermediate stays normal). 7 VALU
// instead of 11; bit-identical to 1.0 / b (rt_selftest_arith, tests/test_gpu_parity.py).
RT_DEV double rcp_rn(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    return fma(e, r, r);
}
// 1 / b for any b: rcp_rn's sequence when every lane of the wave is in its range, else the library's
RT_DEV double rcp_any(double b) {
    if (wave_all(rcp_safe(b))) return rcp_rn(b);
    return 1.0 / b;
}
#ifndef RT_OPT_QDIV
#define RT_OPT_QDIV 1  // A/B: sign of a zero quotient by copysign (1) or by a select on r == 0 (0)
#endif
RT_DEV double qdiv(double a, double b, double y) {
    double q0 = a * y;
    double r = fma(-b, q0, a);
#if RT_OPT_QDIV
    // fma(r, y, q0) is RN(a / b); only a zero quotient (a = +-0) can come out with the wrong sign
    // (+0 + -0 = +0), and q0 = a y already carries the quotient's sign whenever a != 0 (no
    // underflow in range), so the sign bit is taken from q0 (one v_bfi_b32 instead of cmp + 2 selects).
    return __builtin_copysign(fma(r, y, q0), q0);
#else
    return r == 0.0 ? q0 : fma(r, y, q0);
#endif
}
RT_DEV V3 operator/(V3 a, double s) {
    if (wave_all(rcp_safe(s))) {  // wave-uniform: no per-lane exec juggling on the common path
        double y = rcp_rn(s);
        return v3(qdiv(a.x, s, y), qdiv(a.y, s, y), qdiv(a.z, s, y));
    }
    return v3(a.x / s, a.y / s, a.z / s);
}
#ifndef RT_OPT_SQRT
#define RT_OPT_SQRT 1  // A/B: unscaled sqrt sequence behind a wave vote (1) or the library sqrt (0)
#endif
// RN(sqrt(x)): for x in [2^-767, inf) the compiler's own f64 sqrt sequence (v_rsq_f64, one
// Goldschmidt step and two Newton corrections) without its input scaling (an identity in that
// range: ldexp by 0) and its 0/inf fixup (unreachable there); 11 VALU instead of 17. Other inputs
// (0, tiny, inf, NaN, negative) take the library sqrt.
RT_DEV double sqrt_rn(double x) {
#if RT_OPT_SQRT
    if (wave_all(x >= 0x1p-767 && x < INFINITY)) {
        const double y = __builtin_amdgcn_rsq(x);
        double g = x * y, h = y * 0.5;
        const double r = fma(-h, g, 0.5);
        g = fma(g, r, g);
        h = fma(h, r, h);
        double d = fma(-g, g, x);
        g = fma(d, h, g);
        d = fma(-g, g, x);
        return fma(d, h, g);
    }
#endif
    return sqrt(x);
}
RT_DEV double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_DEV V3 cross(V3 a, V3 b) { return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
RT_DEV V3 mult(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_DEV double mag(V3 a) { return sqrt_rn(a.x * a.x + a.y * a.y + a.z * a.z); }
RT_DEV V3 norm(V3 a) { return a / mag(a); }
RT_DEV bool equal_within(V3 a, V3 b, double e) {
    return fabs(a.x - b.x) < e && fabs(a.y - b.y) < e && fabs(a.z - b.z) < e;
}
RT_DEV V3 flip_across(V3 a, V3 axis) { return (2.0 * dot(a, axis)) * axis - a; }
RT_DEV bool is_zero(V3 a) { return a.x == 0.0 && a.y == 0.0 && a.z == 0.0; }
RT_DEV double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
RT_DEV V3 clampv(V3 a, double lo, double hi) { return v3(clampd(a.x, lo, hi), clampd(a.y, lo, hi), clampd(a.z, lo, hi)); }
RT_DEV double det3(V3 v0, V3 v1, V3 v2) {
    return v0.x * (v1.y * v2.z - v1.z * v2.y) - v1.x * (v0.y * v2.z - v0.z * v2.y) + v2.x * (v0.y * v1.z - v0.z * v1.y);
}
RT_DEV double powi(double b, int n) {
    bool neg = n < 0;
    unsigned e = neg ? (unsigned)(-n) : (unsigned)n;
    double r = 1.0;
    while (e) {
        if (e & 1u) r *= b;
        b *= b;
        e >>= 1;
    }
    return neg ? 1.0 / r : r;
}

// sin and cos of phi in [0, 2pi] (the only arguments the path uses: 2*PI*u, scene.rs:61,
// geometry.rs:580-581): Cody-Waite reduction by pi/2 (fdlibm constants) and the fdlibm kernel
// polynomials. Max error 1 ulp against glibc over 5e7 samples — the same class as
// device libm; ~50 VALU instead of ~250 for ocml's general sin+cos.
RT_DEV void sincos_2pi(double x, double* s, double* c) {
    const double INVPIO2 = 6.36619772367581382433e-01;
    const double P1 = 1.57079632673412561417e+00, P2 = 6.07710050630396597660e-11, P2T = 2.02226624879595063154e-21;
    double k = rint(x * INVPIO2);
    double t = fma(-k, P1, x);
    double w = k * P2;
    double r = t - w;
    w = k * P2T - ((t - r) - w);
    double xx = r - w;
    double yy = (r - xx) - w;
    const int q = (int)k & 3;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = xx * xx, v = z * xx;
    double rs = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    double sn = xx - ((z * (0.5 * yy - v * rs) - yy) - v * S1);
    double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double ax = fabs(xx);
    double qx;
    if (ax > 0.78125) qx = 0.28125;
    else qx = __longlong_as_double((__double_as_longlong(ax * 0.25) & (long long)0xFFFFFFFF00000000ull));
    double cs = ax < 0.3 ? 1.0 - (0.5 * z - (z * rc - xx * yy)) : (1.0 - qx) - ((0.5 * z - qx) - (z * rc - xx * yy));
    double s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
    *s = (q & 2) ? -s0 : s0;
    *c = ((q + 1) & 2) ? -c0 : c0;
}

struct Ray {
    V3 o, d;
};
RT_DEV V3 eval(const Ray& r, double t) { return r.o + t * r.d; }

// Per-ray reciprocals of the direction for the divisions x / d.{x,y,z} (box faces, axis planes).
// Bit-identical to the IEEE quotient whenever |d_k| is in [2^-900, 2^900]. Outside that range
// (d_k = 0 or subnormal-tiny) the quotient becomes NaN/inf where the reference has +-inf or a
// huge value; both only ever decide "this face/plane is not hit" (a plane needs |d_k| >= 1e-4; a
// box face at t ~ 1/d_k lies far outside the box in the other coordinates for any direction with
// |d| ~ 1), so the boolean outcomes are the reference's for every valid ray.
struct RayInv {
    double rx, ry, rz;
};
RT_DEV RayInv make_inv(const V3& d) {
    RayInv v;
    if (wave_all(rcp_safe(d.x) && rcp_safe(d.y) && rcp_safe(d.z))) {  // wave-uniform fast path
        v.rx = rcp_rn(d.x);
        v.ry = rcp_rn(d.y);
        v.rz = rcp_rn(d.z);
    } else {
        v.rx = 1.0 / d.x;
        v.ry = 1.0 / d.y;
        v.rz = 1.0 / d.z;
    }
    return v;
}
RT_DEV double div_x(double a, const Ray& r, const RayInv& v) { return qdiv(a, r.d.x, v.rx); }
RT_DEV double div_y(double a, const Ray& r, const RayInv& v) { return qdiv(a, r.d.y, v.ry); }
RT_DEV double div_z(double a, const Ray& r, const RayInv& v) { return qdiv(a, r.d.z, v.rz); }

// ---------------------------------------------------------------- RNG v2
#ifndef RT_RNG32
#define RT_RNG32 0
#endif
// One xoroshiro128++ stream per camera sample, seeded by Philox4x32-10(key = seed,
// counter = (pixel, sample, 0, subpixel)); consumed in the reference's draw order along the path.
struct Rng {
    uint64_t s0, s1;
    RT_DEV Rng() : s0(1), s1(0) {}
    RT_DEV Rng(uint64_t a, uint64_t b) : s0(a), s1(b) {}
    RT_DEV Rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t sub) {
        uint32_t c0 = pixel, c1 = sample, c2 = 0u, c3 = sub;
        uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (r) {
                k0 += 0x9E3779B9u;
                k1 += 0xBB67AE85u;
            }
            uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
            uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
            uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
            c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        }
        s0 = ((uint64_t)c0 << 32) | c1;
        s1 = ((uint64_t)c2 << 32) | c3;
        if ((s0 | s1) == 0) s0 = 1;
    }
    static RT_DEV uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
#if RT_RNG32
    // A/B (RNG v3 candidate): xoshiro128++ on the same 128 state bits (x0..x3 = the 32-bit halves of
    // s0, s1), one 32-bit output per draw, uniform = k * 2^-32
    static RT_DEV uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
    RT_DEV uint32_t next32() {
        uint32_t x0 = (uint32_t)s0, x1 = (uint32_t)(s0 >> 32), x2 = (uint32_t)s1, x3 = (uint32_t)(s1 >> 32);
        const uint32_t r = rotl32(x0 + x3, 7) + x0;
        const uint32_t t = x1 << 9;
        x2 ^= x0;
        x3 ^= x1;
        x1 ^= x2;
        x0 ^= x3;
        x2 ^= t;
        x3 = rotl32(x3, 11);
        s0 = (uint64_t)x0 | ((uint64_t)x1 << 32);
        s1 = (uint64_t)x2 | ((uint64_t)x3 << 32);
        return r;
    }
    RT_DEV double uniform() { return (double)next32() * 0x1p-32; }
    RT_DEV bool below53(uint64_t thr) { return ((uint64_t)next32() << 21) < thr; }
#endif
    RT_DEV uint64_t next() {  // xoroshiro128++
        uint64_t a = s0, b = s1;
        uint64_t r = rotl(a + b, 17) + a;
        b ^= a;
        s0 = rotl(a, 49) ^ b ^ (b << 21);
        s1 = rotl(b, 28);
        return r;
    }
#if !RT_RNG32
#ifndef RT_OPT_UNIF
#define RT_OPT_UNIF 0  // A/B: 1 = two 32-bit conversions and one FMA (same bits; measured 0.6% slower on
                       // cornell_box, profiles/r02_ab.log r02z), 0 = the u64 -> f64 conversion
#endif
    // (u64 >> 11) * 2^-53, exactly: the 53-bit value is hi * 2^32 + lo (hi < 2^21); hi * 2^-21 and
    // lo * 2^-53 are exact and so is their sum, so the FMA returns the exact product
    RT_DEV double uniform() {
#if RT_OPT_UNIF
        const uint64_t v = next() >> 11;
        return fma((double)(uint32_t)(v >> 32), 0x1p-21, (double)(uint32_t)v * 0x1p-53);
#else
        return (double)(next() >> 11) * (1.0 / 9007199254740992.0);
#endif
    }
    // uniform() < p for p = thr * 2^-53 (thr an integer <= 2^53): the draw is v * 2^-53 exactly, so
    // the comparison is v < thr, with no conversion (Russian roulette, scene.rs:173/:231)
    RT_DEV bool below53(uint64_t thr) { return (next() >> 11) < thr; }
#endif
};
// Russian-roulette thresholds as 53-bit integers: p = 1 (depth <= MAX_BOUNCES) and p = 0.9, whose
// double is M * 2^-53 for an integer M (0.9 lies in [0.5, 1))
constexpr uint64_t kP53One = 1ull << 53;
constexpr uint64_t kP53Survive = (uint64_t)(SURVIVAL_PROBABILITY * 9007199254740992.0);
static_assert((double)kP53Survive == SURVIVAL_PROBABILITY * 9007199254740992.0, "0.9 * 2^53 must be an integer");

// ---------------------------------------------------------------- primitives (geometry.rs:512-571)
RT_DEV bool sphere_t(const DevObject& o, const Ray& ray, double* tout) {
    V3 op = ld3(o.pos) - ray.o;
    const double eps = 1e-4;
    double b = dot(op, ray.d);
    double det = b * b - dot(op, op) + o.r * o.r;
    if (det < 0.) return false;
    det = sqrt_rn(det);
    double t = b - det;
    if (t > eps) { *tout = t; return true; }
    t = b + det;
    if (t > eps) { *tout = t; return true; }
    return false;
}
RT_DEV bool plane_t(const DevObject& o, const Ray& ray, const RayInv& inv, double* tout) {
    if (o.axis >= 0) {
        // n = +-e_axis exactly: dot(pos - o, n) / dot(d, n) == (pos - o)_axis / d_axis bit for bit
        // (the +-0 terms vanish and IEEE division is sign-symmetric); shares the ray reciprocal.
        double dn, num, t;
        if (o.axis == 0) { dn = ray.d.x; num = o.pos[0] - ray.o.x; }
        else if (o.axis == 1) { dn = ray.d.y; num = o.pos[1] - ray.o.y; }
        else { dn = ray.d.z; num = o.pos[2] - ray.o.z; }
        if (fabs(dn) < 0.0001) return false;
        t = o.axis == 0 ? div_x(num, ray, inv) : o.axis == 1 ? div_y(num, ray, inv) : div_z(num, ray, inv);
        if (t >= 0.) { *tout = t; return true; }
        return false;
    }
    V3 n = ld3(o.n);
    double dn = dot(ray.d, n);
    if (fabs(dn) < 0.0001) return false;
    double t = dot(ld3(o.pos) - ray.o, n) / dot(ray.d, n);
    if (t >= 0.) { *tout = t; return true; }
    return false;
}
// Triangle::intersect (geometry.rs:637-670) on the precomputed (a, ab, ac, n); TR = DevTri in any
// address space (flat_query reads its triangles through a constant-address-space pointer: s_load).
// The triangle's unit normal: stored (DevTri), or recomputed for a 72-B leaf copy with the host's own
// operations (rt_api.cpp: Triangle::normal = (c - a).cross(b - a).norm()), so the same bits.
template <class TR>
RT_DEV V3 tri_normal(const TR& tr) {
    if constexpr (sizeof(TR) == sizeof(DevTri)) {
        return ld3(tr.n);
    } else {
        const V3 ab = ld3(tr.ab), ac = ld3(tr.ac);
        const V3 cr = v3(ac.y * ab.z - ac.z * ab.y, ac.z * ab.x - ac.x * ab.z, ac.x * ab.y - ac.y * ab.x);
        const double mg = sqrt_rn(cr.x * cr.x + cr.y * cr.y + cr.z * cr.z);
        if (wave_all(rcp_safe(mg))) {
            const double y = rcp_rn(mg);
            return v3(qdiv(cr.x, mg, y), qdiv(cr.y, mg, y), qdiv(cr.z, mg, y));
        }
        return v3(cr.x / mg, cr.y / mg, cr.z / mg);
    }
}
#ifndef RT_TRI_MINORS
#define RT_TRI_MINORS 1  // tri_t's determinants through their shared minors (1), or four det3 calls (0: A/B)
#endif
template <class TR>
RT_DEV bool tri_t(const TR& tr, const Ray& ray, double* tout) {
    V3 n = tri_normal(tr);
    if (fabs(dot(n, ray.d)) < 0.0001) return false;
    V3 ab = ld3(tr.ab), ac = ld3(tr.ac);
    V3 b = ray.o - ld3(tr.a);
    V3 nd = -ray.d;
#if RT_TRI_MINORS
    // det3's cofactor expansion of the four determinants with their seven distinct 2x2 minors computed once
    // (each det3(v0, v1, v2) = v0.x M1 - v1.x M2 + v2.x M3 with the same minors, the same operations)
    const double mA = ab.y * ac.z - ab.z * ac.y, mB = nd.y * ac.z - nd.z * ac.y, mC = nd.y * ab.z - nd.z * ab.y;
    const double mD = b.y * ac.z - b.z * ac.y, mE = b.y * ab.z - b.z * ab.y, mF = nd.y * b.z - nd.z * b.y;
    const double mG = ab.y * b.z - ab.z * b.y;
    double det = nd.x * mA - ab.x * mB + ac.x * mC;  // det3(nd, ab, ac)
    double tn = b.x * mA - ab.x * mD + ac.x * mE;    // det3(b, ab, ac)
    double un = nd.x * mD - b.x * mB + ac.x * mF;    // det3(nd, b, ac)
    double vn = nd.x * mG - ab.x * mF + b.x * mC;    // det3(nd, ab, b)
#else
    double det = det3(nd, ab, ac);
    double tn = det3(b, ab, ac), un = det3(nd, b, ac), vn = det3(nd, ab, b);
#endif
    double t, u, v;
    if (wave_all(rcp_safe(det))) {  // wave-uniform
        double y = rcp_rn(det);
        t = qdiv(tn, det, y);
        u = qdiv(un, det, y);
        v = qdiv(vn, det, y);
    } else {
        t = tn / det;
        u = un / det;
        v = vn / det;
    }
    if (u < 0. || u > 1. || v < 0. || u + v > 1.) return false;
    if (t > 0.0001) { *tout = t; return true; }
    return false;
}
// BoundingBox::intersect(..).is_some() (geometry.rs:977-1036): first face in order (-x,+x,-y,+y,-z,+z).
// The six divisions use the ray's reciprocals (bit-identical quotients, see qdiv).
RT_DEV bool box_hit(const double* bx, const Ray& r, const RayInv& inv) {
    const double EPS = 0.0000001;
    const double mnx = bx[0], mny = bx[1], mnz = bx[2], mxx = bx[3], mxy = bx[4], mxz = bx[5];
    double t;
    V3 p;
    t = div_x(mnx - r.o.x, r, inv);
    if (t >= EPS) { p = eval(r, t); if (mny <= p.y && p.y <= mxy && mnz <= p.z && p.z <= mxz) return true; }
    t = div_x(mxx - r.o.x, r, inv);
    if (t >= EPS) { p = eval(r, t); if (mny <= p.y && p.y <= mxy && mnz <= p.z && p.z <= mxz) return true; }
    t = div_y(mny - r.o.y, r, inv);
    if (t >= EPS) { p = eval(r, t); if (mnx <= p.x && p.x <= mxx && mnz <= p.z && p.z <= mxz) return true; }
    t = div_y(mxy - r.o.y, r, inv);
    if (t >= EPS) { p = eval(r, t); if (mnx <= p.x && p.x <= mxx && mnz <= p.z && p.z <= mxz) return true; }
    t = div_z(mnz - r.o.z, r, inv);
    if (t >= EPS) { p = eval(r, t); if (mnx <= p.x && p.x <= mxx && mny <= p.y && p.y <= mxy) return true; }
    t = div_z(mxz - r.o.z, r, inv);
    if (t >= EPS) { p = eval(r, t); if (mnx <= p.x && p.x <= mxx && mny <= p.y && p.y <= mxy) return true; }
    return false;
}

// Conservative cull: false only if the ray (t >= 0) passes farther than `pad` from the box, in
// which case no box contained in it can pass box_hit (its face points would be within rounding,
// ~1e-11, of the ray). Exactness argument in DESIGN.md §Octree.
// tmax: the caller's bound on a useful hit (closest analytic hit so far, or the shadow distance);
// every mesh hit point lies in DevMesh::cull_box (the root box united with the vertex bounds, so it
// encloses every triangle even after the `scale` bbox quirk), so a box entered only beyond tmax
// (with margin) cannot produce a hit that would be used.
RT_DEV bool near_box(const double* bx, const Ray& r, const RayInv& inv, double pad, double tmax) {
    double t0 = 0.0, t1 = INFINITY;
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    const double rc[3] = {inv.rx, inv.ry, inv.rz};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double lo = bx[k] - pad, hi = bx[3 + k] + pad;
        if (!(fabs(d[k]) >= 0x1p-900 && fabs(d[k]) <= 0x1p900)) {
            if (!(fabs(d[k]) < 0x1p-900)) return true;  // NaN / huge: do not cull
            if (o[k] < lo || o[k] > hi) return false;  // (nearly) parallel slab: origin must lie inside it
            continue;
        }
        double ta = (lo - o[k]) * rc[k], tb = (hi - o[k]) * rc[k];
        double tn = fmin(ta, tb), tf = fmax(ta, tb);
        t0 = fmax(t0, tn - 1e-9 * fabs(tn));
        t1 = fmin(t1, tf + 1e-9 * fabs(tf));
    }
    return t0 <= t1 && t0 <= tmax * (1.0 + 1e-9) + 1e-9;
}


// The reference's child visiting order (geometry.rs:1248-1260): the 8 root octants insertion-sorted
// by mag(centre - origin), swapping only while strictly greater — a stable sort, i.e. a sort by
// (key, octant index). Done as Batcher's 19-comparator network on (key, index) pairs held in
// registers (the unrolled insertion sort indexed d2[] by runtime nibbles: select chains, ~1000
// VALU). Keys: the radicands d2 (sqrt is monotone); two radicands within 2^-50 of each other may
// round to the same sqrt, so if any neighbours of the sorted order are that close the sort is redone
// on the exact keys sqrt(d2) (rare, wave-divergent). Returns nibble q = octant visited q-th.
RT_DEV uint32_t root_order(const double d2[8]) {
    constexpr int net[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
                                {0, 4}, {3, 7}, {1, 5}, {2, 6}, {1, 4}, {3, 6}, {2, 4}, {3, 5}, {3, 4}};
    double k[8];
    int ix[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { k[i] = d2[i]; ix[i] = i; }
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int c = 0; c < 19; ++c) {
            const int a = net[c][0], b = net[c][1];
            const bool sw = k[a] > k[b] || (k[a] == k[b] && ix[a] > ix[b]);
            const double ka = k[a], kb = k[b];
            const int ia = ix[a], ib = ix[b];
            k[a] = sw ? kb : ka; k[b] = sw ? ka : kb;
            ix[a] = sw ? ib : ia; ix[b] = sw ? ia : ib;
        }
        bool close = false;
#pragma unroll
        for (int q = 0; q < 7; ++q) close |= !(k[q + 1] > k[q] * (1.0 + 0x1p-50));
        if (pass == 1 || !close) break;
#pragma unroll
        for (int i = 0; i < 8; ++i) { k[i] = sqrt(d2[i]); ix[i] = i; }  // mag() itself
    }
    uint32_t order = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) order |= (uint32_t)ix[q] << (4 * q);
    return order;
}

// root_order's result from the structure of the 8 root octant centres, a 2x2x2 grid: along axis k the
// centres take two coordinates, with squared distances e0_k, e1_k from the origin (the very values
// the radicand dv.x*dv.x + dv.y*dv.y + dv.z*dv.z sums), so up to rounding the radicand of an octant is
// the sum of its near-half terms plus delta_k = |e1_k - e0_k| for every axis where it lies in the
// far half. With the deltas sorted, da <= db <= dc, the octants in increasing radicand are: near,
// +a, +b, then +a+b and +c (in the order of da + db vs dc), +a+c, +b+c, +a+b+c. The consecutive gaps
// are da, db - da, dc - db and |dc - da - db|; when all exceed 2^-46 of the largest radicand (the
// radicands carry two roundings, <= 2^-52 of it), the radicands in this order increase by more than
// the 2^-50 that root_order requires to take its keys as distinct, so this IS root_order's result
// (a strict order, no tie to break). Returns false otherwise (the caller runs root_order). ~70 VALU
// instead of the radicands plus the 19-comparator network (~260).
#ifndef RT_ROOT_GRID
#define RT_ROOT_GRID 1  // A/B: 0 = always the sorting network
#endif
template <class MT>
RT_DEV bool root_order_grid(const MT& m, const Ray& ray, uint32_t* order) {
#if RT_ROOT_GRID
    const double o[3] = {ray.o.x, ray.o.y, ray.o.z};
    double dl[3], far[3];
    uint32_t nb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double lo = m.oct_center[0][k] - o[k], hi = m.oct_center[4 >> k][k] - o[k];  // octants 0 / 4, 2, 1
        const double e0 = lo * lo, e1 = hi * hi;
        nb[k] = e1 < e0 ? (4u >> k) : 0u;  // the nearer half's octant bit
        dl[k] = fabs(e1 - e0);
        far[k] = fmax(e0, e1);
    }
    // sort (delta, axis bit) ascending: a, b, c
    double da = dl[0], db = dl[1], dc = dl[2];
    uint32_t A = 4u, B = 2u, C = 1u;
    if (db < da) { const double t = da; da = db; db = t; const uint32_t u = A; A = B; B = u; }
    if (dc < db) { const double t = db; db = dc; dc = t; const uint32_t u = B; B = C; C = u; }
    if (db < da) { const double t = da; da = db; db = t; const uint32_t u = A; A = B; B = u; }
    const double sab = da + db;
    const double gap = fmin(fmin(da, db - da), fmin(dc - db, fabs(dc - sab)));
    const bool ok = gap > 0x1p-46 * (far[0] + far[1] + far[2]);
    const uint32_t N = nb[0] | nb[1] | nb[2];
    const bool abc = sab < dc;  // +a+b before +c
    const uint32_t x3 = abc ? (N ^ A ^ B) : (N ^ C), x4 = abc ? (N ^ C) : (N ^ A ^ B);
    *order = N | (N ^ A) << 4 | (N ^ B) << 8 | x3 << 12 | x4 << 16 | (N ^ A ^ C) << 20 | (N ^ B ^ C) << 24 |
             (N ^ A ^ B ^ C) << 28;
    return ok;
#else
    (void)m; (void)ray; (void)order;
    return false;
#endif
}

// BoundingBox::intersect(..).is_some() (geometry.rs:977-1036) for all 8 octants of the box
// [mn, mx] at once; bit i = octant i (bit2 = x, bit1 = y, bit0 = z upper half, geometry.rs:1067-1099).
// An octant's six faces lie on 9 planes (min / centre / max per axis), so each plane's crossing
// (t, and the point's two other coordinates) is computed once and shared by the 4 octants whose
// faces lie on it. Every quantity is the one box_hit computes for that octant's box (same
// division, same eval, same bounds: the octant boxes are built from exactly this centre), and
// box_hit's result is the OR over faces, so the mask equals eight box_hit calls bit for bit.
RT_DEV uint32_t octant_mask(const double* mn, const double* mx, const Ray& r, const RayInv& inv) {
    const double EPS = 0.0000001;
    const double o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    double c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = (mn[k] + mx[k]) / 2.0;  // BoundingBox::center
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // planes normal to axis k
        const int u = k == 0 ? 1 : 0, v = k == 2 ? 1 : 2;  // the other two axes, u < v
        // octant index bit of axis a: 4 >> a
        const uint32_t bk = 4u >> k, bu = 4u >> u, bv = 4u >> v;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double X = j == 0 ? mn[k] : j == 1 ? c[k] : mx[k];
            const double num = X - o[k];
            const double t = k == 0 ? div_x(num, r, inv) : k == 1 ? div_y(num, r, inv) : div_z(num, r, inv);
            if (t >= EPS) {
                const double pu = o[u] + t * d[u], pv = o[v] + t * d[v];  // Ray::eval
                const bool ul = mn[u] <= pu && pu <= c[u], uh = c[u] <= pu && pu <= mx[u];
                const bool vl = mn[v] <= pv && pv <= c[v], vh = c[v] <= pv && pv <= mx[v];
                // octants with this face, for the lower (j <= 1) and upper (j >= 1) half along k
                uint32_t q = 0;
                q |= (ul && vl) ? (1u << 0) : 0u;
                q |= (ul && vh) ? (1u << bv) : 0u;
                q |= (uh && vl) ? (1u << bu) : 0u;
                q |= (uh && vh) ? (1u << (bu + bv)) : 0u;
                if (j <= 1) m |= q;
                if (j >= 1) m |= q << bk;
            }
        }
    }
    return m;
}

// Diagnostic builds only (make EXTRA="-DRT_DEBUG_COUNTERS=1 -DRT_DEBUG_TIMERS=1", tools/dbg_mesh.py).
// Counters and timers accumulate per block in LDS (LDS atomics: global atomics from every lane on a
// few addresses serialised the instrumented kernels and distorted what they measured) and are
// flushed to the g_dbg* arrays once per block by the megakernels (RT_DBG_TINIT / RT_DBG_TFLUSH);
// other kernels' counts are dropped.
#if RT_DEBUG_COUNTERS
// 0 walks, 1 past cull, 2 node visits, 3 leaves, 4 tri tests, 5 steps; mesh megakernel (per wave):
// 8 iterations, 9 lanes in the vertex phase, 10 walk-loop steps, 11 walking lanes over those steps
__device__ unsigned long long g_dbg[16];
__shared__ unsigned long long s_dbg_cnt[16];
#define RT_DBG(i) atomicAdd(&s_dbg_cnt[i], 1ull)
#define RT_DBG_WAVE(i, pred) do { const unsigned long long m_ = __ballot(pred); if (__lane_id() == 0) atomicAdd(&s_dbg_cnt[i], (unsigned long long)__popcll(m_)); } while (0)
// lane utilisation of code region i (< 16): [2i] wave entries, [2i+1] active lanes summed over them
__device__ unsigned long long g_dbg_region[32];
__shared__ unsigned long long s_dbg_reg[32];
#define RT_DBG_REGION(i) do { const unsigned long long m_ = __ballot(1); if (__lane_id() == __ffsll((long long)m_) - 1) { atomicAdd(&s_dbg_reg[2 * (i)], 1ull); atomicAdd(&s_dbg_reg[2 * (i) + 1], (unsigned long long)__popcll(m_)); } } while (0)
#define RT_DBG_CINIT() do { if (threadIdx.x < 16) s_dbg_cnt[threadIdx.x] = 0; if (threadIdx.x < 32) s_dbg_reg[threadIdx.x] = 0; } while (0)
#define RT_DBG_CFLUSH() do { if (threadIdx.x < 16) atomicAdd(&g_dbg[threadIdx.x], s_dbg_cnt[threadIdx.x]); if (threadIdx.x < 32) atomicAdd(&g_dbg_region[threadIdx.x], s_dbg_reg[threadIdx.x]); } while (0)
#else
#define RT_DBG_REGION(i) ((void)0)
#define RT_DBG(i) ((void)0)
#define RT_DBG_WAVE(i, pred) ((void)0)
#define RT_DBG_CINIT() ((void)0)
#define RT_DBG_CFLUSH() ((void)0)
#endif
// Wave time per code region i (< 16) in s_memtime ticks, summed per wave in LDS and flushed to
// g_dbg_time at the kernel's end; blocks of up to 512 threads (8 waves).
#if RT_DEBUG_TIMERS
__device__ unsigned long long g_dbg_time[16];
__shared__ unsigned long long s_dbg_time[16 * 16];
#define RT_DBG_TSTART(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define RT_DBG_TEND(i, v) do { const uint64_t d_ = __builtin_amdgcn_s_memtime() - (v); const unsigned long long m_ = __ballot(1); if (__lane_id() == __ffsll((long long)m_) - 1) atomicAdd(&s_dbg_time[(threadIdx.x >> 6) * 16 + (i)], (unsigned long long)d_); } while (0)
#define RT_DBG_TIMERS_INIT() do { for (unsigned i_ = threadIdx.x; i_ < 16 * 16; i_ += blockDim.x) s_dbg_time[i_] = 0; } while (0)
#define RT_DBG_TIMERS_FLUSH() do { for (unsigned i_ = threadIdx.x; i_ < 16 * 16; i_ += blockDim.x) atomicAdd(&g_dbg_time[i_ & 15], s_dbg_time[i_]); } while (0)
#else
#define RT_DBG_TSTART(v) ((void)0)
#define RT_DBG_TEND(i, v) ((void)0)
#define RT_DBG_TIMERS_INIT() ((void)0)
#define RT_DBG_TIMERS_FLUSH() ((void)0)
#endif
#if RT_DEBUG_COUNTERS || RT_DEBUG_TIMERS
#define RT_DBG_TINIT() do { RT_DBG_CINIT(); RT_DBG_TIMERS_INIT(); __syncthreads(); } while (0)
#define RT_DBG_TFLUSH() do { __syncthreads(); RT_DBG_CFLUSH(); RT_DBG_TIMERS_FLUSH(); } while (0)
#else
#define RT_DBG_TINIT() ((void)0)
#define RT_DBG_TFLUSH() ((void)0)
#endif

// Octree::intersect (geometry.rs:1237-1295) as a resumable per-lane walk.
// The reference visits a node's children in one order per ray (distances from the ray origin to
// the ROOT box's octant centres, insertion-sorted with strict >, geometry.rs:1248-1260), descends
// into the first child whose box the ray hits, and returns the first subtree with any hit (a leaf:
// its nearest triangle, strict <, geometry.rs:1276-1293). The order is the same at every level, so
// the walk keeps, per level, the 8-bit mask of the children still to visit (in visiting order)
// instead of a stack of nodes, resumes at the parent through node_up, and rebuilds boxes from the
// root along the path of octant slots. Same visits, same early exit, same result bits.
// Each walk_step does one unit of work (a triangle test, a backtrack, or a child pick that either
// opens a leaf or descends and masks the new node's children), so a wave can interleave walks of
// different lengths and refill lanes whose walk ended (persistent traversal kernels).
#ifndef RT_LTRI_INDEX
#define RT_LTRI_INDEX 0  // 1: leaf triangle lists as indices into DevScene::tris (3.6 MB for the unicorn);
                         // 0: per-leaf copies (18 MB). The index adds a dependent load per triangle: 3%
                         // slower while tri_t loaded triangles one by one, 0.5% once a step's triangles
                         // are preloaded (profiles/r02_ab.log): the copies stay the default
#endif
#ifndef RT_WALK_TIGHT
#define RT_WALK_TIGHT 1  // A/B: 0 = visit every child whose octant box the ray hits (the reference's walk)
#endif
#ifndef RT_WALK_HOIST
#define RT_WALK_HOIST 1  // the slot walk loads the open leaf's triangles before its node operation (1: unicorn
                         // +2.4%, no spill at 254 VGPRs with the kernarg views), tests them first with the node
                         // operation's loads fetched ahead (2: +2.1%), or after it (0) (profiles/r04_ab.log)
#endif
struct OctWalk {
    double mn[3], mx[3];  // box of `cur`
    int32_t cur, depth;
    uint32_t path;        // octant slot taken at each level, 3 bits per level (max depth 10)
    uint32_t pm;          // children of `cur` still to visit, bit q = visiting rank q
    uint64_t stk;         // pm of the ancestors at levels 0..7, 8 bits each
    uint32_t stk8;        // level 8 (parents exist at depths 0..9; MAX_DEPTH = 10)
    uint32_t order;       // nibble q = octant visited q-th
    int32_t lpos, lend;   // leaf triangle cursor
    int32_t best;         // nearest triangle so far in the current leaf (ltri index), -1 none
    double bt;
    // The slot walk's one-leaf buffer (walk_step<true>): the next leaf in visiting order the node walk
    // found while the cursor was still busy (nlf < nle), and whether the node walk is exhausted.
    int32_t nlf, nle;
    uint32_t ndone;
    uint32_t enter;  // bit 0, slot walk: the root is still to be entered (its octant_mask runs in the first step,
                     // in the same code as every descent's); bit 1: dir_in_range of the walk's ray (walk_begin)
};

RT_DEV bool dir_in_range(const Ray& ray) {  // kid_tight_hit's `inr` on all three axes
    auto inr = [](double d) { return fabs(d) >= 0x1p-900 && fabs(d) <= 0x1p900; };
    return inr(ray.d.x) && inr(ray.d.y) && inr(ray.d.z);
}
// LDS column of a walk's ancestor node ids (walk_node_slots' `anc`)
typedef __attribute__((address_space(3))) int32_t LdsAncI32;
typedef __attribute__((address_space(3))) uint16_t LdsAncU16;  // pids < 2^16 (DevScene::n_pid): half the LDS

// Mask `cur`'s existing children whose boxes the ray hits, permuted to visiting order (the node_kids
// walk: the child table is read again by each pick, an L2 hit).
RT_DEV void walk_enter(const DevScene& sc, const Ray& ray, const RayInv& inv, OctWalk& w) {
    RT_DBG(2);
    const int4* k4 = reinterpret_cast<const int4*>(sc.node_kids + 8 * (size_t)w.cur);
    const int4 ka = k4[0], kb = k4[1];
    const int32_t kid[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
    uint32_t m = octant_mask(w.mn, w.mx, ray, inv);
#pragma unroll
    for (int i = 0; i < 8; ++i) m &= kid[i] == kKidEmpty ? ~(1u << i) : ~0u;
    uint32_t pm = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) pm |= ((m >> ((w.order >> (4 * q)) & 0xF)) & 1u) << q;
    w.pm = pm;
}
// walk_enter for the slot walk: the node's existence mask comes with its parent's slot entry
// (scene_layout.h KidSlot), so entering a node loads nothing.
RT_DEV void walk_enter_mask(const Ray& ray, const RayInv& inv, OctWalk& w, uint32_t exist) {
    RT_DBG(2);
    const uint32_t m = octant_mask(w.mn, w.mx, ray, inv) & exist;
    uint32_t pm = 0;
    // bit q of pm = bit order[q] of m: one bit-field extract at a variable offset and one shift-or per rank
#pragma unroll
    for (int q = 0; q < 8; ++q) pm |= __builtin_amdgcn_ubfe(m, (w.order >> (4 * q)) & 0xFu, 1u) << q;
    w.pm = pm;
}

// Starts a walk; false if the ray cannot produce a usable hit on this mesh (empty mesh, or the
// conservative near_box cull). tmax: see near_box.
// Slots: the walk continues with walk_step<true> (the slot walk: the root is entered in its first step),
// or with walk_step<false> (the node_kids walk: entered here). The slot walk needs DevScene::node_slot
// (absent for octrees whose node ids do not fit a KidSlot entry: rt_api.cpp pack_scene).
// cull = false: the caller already knows the ray passes near_box for this mesh (mesh_near_mask).
template <bool Slots = (RT_WALK_TIGHT != 0)>
RT_DEV bool walk_begin(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, double tmax,
                       OctWalk& w, bool cull = true) {
    if (m.n_nodes == 0) return false;
    RT_DBG(0);
    if (cull && !near_box(m.cull_box, ray, inv, m.cull_pad, tmax)) return false;
    RT_DBG(1);
    w.best = -1;
    w.bt = 0.0;
    w.nlf = w.nle = 0;
    w.ndone = 0;
    w.enter = dir_in_range(ray) ? 2u : 0u;  // bit 1: kid_tight_hit's `inr` on every axis, once per walk
    // the slot walk names parents by their row (pid); a root leaf has none, and its walk never reads `cur`
    // (no children to pick), but cur >= 0 is what marks a walk in progress (pool_round)
    w.cur = Slots ? max(m.root_pid, 0) : m.node_base;
    w.depth = 0;
    w.path = 0;
    w.stk = 0;
    w.stk8 = 0;
    w.pm = 0;
    if (m.root_leaf >= 0) {
        const int2 ls = sc.leaf_span[m.root_leaf];
        w.lpos = ls.x;
        w.lend = ls.x + ls.y;
        w.order = 0x76543210u;
        return true;
    }
    w.lpos = w.lend = 0;
    uint32_t order;
    const bool grid = root_order_grid(m, ray, &order);
    if (!wave_all(grid)) {
        // a lane near a tie (or the A/B build without the grid form): the sorting network on the radicands
        double d2[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            V3 dv = ld3(m.oct_center[i]) - ray.o;
            d2[i] = dv.x * dv.x + dv.y * dv.y + dv.z * dv.z;  // mag()'s radicand, same operation order
        }
        const uint32_t o2 = root_order(d2);
        if (!grid) order = o2;
    }
    w.order = order;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        w.mn[k] = m.root_box[k];
        w.mx[k] = m.root_box[3 + k];
    }
    if constexpr (Slots) {
        w.enter |= 1u;  // the first step enters the root (walk_node_slots)
    } else {
        walk_enter(sc, ray, inv, w);
    }
    return true;
}

enum : int { WALK_RUN = 0, WALK_HIT = 1, WALK_MISS = 2 };

// One step of the walk. On WALK_HIT, *t / *prim hold the first hit subtree's nearest triangle.
// A step tests up to kTrisPerStep triangles of the open leaf; when the leaf ends without a hit (or
// no leaf is open) it pops every exhausted level at once, then picks the next child in visiting
// order and either opens it (leaf) or descends into it and masks its children. Fewer, fuller steps
// than one unit of work per step: a walk of the unicorn takes ~18 steps instead of ~39.
#ifndef RT_TRIS_PER_STEP
#define RT_TRIS_PER_STEP 2
#endif
constexpr int kTrisPerStep = RT_TRIS_PER_STEP;
#ifndef RT_WALK_OPEN_TEST
#define RT_WALK_OPEN_TEST 0  // 1: a step that opens a leaf also tests its first triangles (measured -10%)
#endif
// Up to kTrisPerStep triangles of the open leaf: WALK_RUN (triangles left), WALK_HIT (the leaf is
// done and has a hit: the first leaf with a hit wins, geometry.rs:1267-1269), or -1 (done, no hit).
#ifndef RT_TRI_PRELOAD
#define RT_TRI_PRELOAD 1  // A/B: the step's triangles are loaded whole before any test (1), or by tri_t (0)
#endif
RT_DEV int leaf_tris(const DevScene& sc, const Ray& ray, OctWalk& w, double* t, int* prim) {
#if RT_TRI_PRELOAD
    // All of the step's triangles (96 B each) are loaded up front: tri_t reads a triangle's normal,
    // tests |n . d| and only then its other 72 B, and the next triangle only after that, i.e. four
    // dependent trips to L2 / the Infinity Cache per step. Entries past the leaf's end are clamped
    // to its last one (loaded, never tested).
    LeafTri tr[kTrisPerStep];
#pragma unroll
    for (int j = 0; j < kTrisPerStep; ++j) {
        const int e = max(0, min(w.lpos + j, w.lend - 1));
#if RT_LTRI_INDEX
        tr[j] = sc.tris[sc.ltri_id[e]];
#else
        tr[j] = sc.ltris[e];
#endif
    }
#endif
#pragma unroll
    for (int j = 0; j < kTrisPerStep; ++j) {
        if (w.lpos < w.lend) {
            RT_DBG(4);
            double tt;
#if RT_TRI_PRELOAD
            if (tri_t(tr[j], ray, &tt) && (w.best < 0 || tt < w.bt)) {
#else
#if RT_LTRI_INDEX
            const DevTri& trj = sc.tris[sc.ltri_id[w.lpos]];  // leaf list = triangle indices (3.6 MB table)
#else
            const LeafTri& trj = sc.ltris[w.lpos];  // leaf list = triangle copies (18 MB for the unicorn)
#endif
            if (tri_t(trj, ray, &tt) && (w.best < 0 || tt < w.bt)) {
#endif
                w.bt = tt;
                w.best = w.lpos;
            }
            ++w.lpos;
        }
    }
    if (w.lpos < w.lend) return WALK_RUN;
    if (w.best >= 0) {
        *t = w.bt;
        *prim = sc.ltri_id[w.best];
        return WALK_HIT;
    }
    return -1;
}
// The tests of leaf_tris on triangles already loaded (the slot walk's hoisted loads, walk_step<true>).
// tid (RT_LTRI_ID_HOIST): the triangles' global ids, loaded with them; w.best then holds the best
// triangle's id itself, so a hit needs no dependent ltri_id load at the leaf's end.
RT_DEV int leaf_tris_loaded(const DevScene& sc, const Ray& ray, OctWalk& w, const LeafTri* tr, double* t, int* prim,
                            const int32_t* tid = nullptr) {
#pragma unroll
    for (int j = 0; j < kTrisPerStep; ++j) {
        if (w.lpos < w.lend) {
            RT_DBG(4);
            double tt;
            if (tri_t(tr[j], ray, &tt) && (w.best < 0 || tt < w.bt)) {
                w.bt = tt;
                w.best = tid ? tid[j] : w.lpos;
            }
            ++w.lpos;
        }
    }
    if (w.lpos < w.lend) return WALK_RUN;
    if (w.best >= 0) {
        *t = w.bt;
        *prim = tid ? w.best : sc.ltri_id[w.best];
        return WALK_HIT;
    }
    return -1;
}
// Could any triangle below the child of slot `ks` (scene_layout.h KidSlot) return tri_intersect ==
// true for this ray? false only if the ray (t >= 0) passes farther than the padding from the child
// subtree's triangle bounds: the same conservative slab test as near_box. Skipping such a child leaves
// the walk's result unchanged: the reference would descend, test every triangle below it, find none,
// and go on with the next child in visiting order.
// The bound codes decode as base + q * step: rt_api.cpp make_slot keeps the scene's slot tables only when no
// code was clamped to the 16-bit range, so every decoded bound encloses its subtree's padded triangle bounds.
// (RT_TIGHT_INF=1: round 4's decode, codes 0 / kTightTop as -inf / +inf, which that guarantee makes dead.)
#ifndef RT_TIGHT_INF
#define RT_TIGHT_INF 0
#endif
RT_DEV double tight_lo(uint32_t q, double step, double base) {
    return (RT_TIGHT_INF && q == 0u) ? -INFINITY : fma((double)q, step, base);
}
RT_DEV double tight_hi(uint32_t q, double step, double base) {
    return (RT_TIGHT_INF && q == (uint32_t)kTightTop) ? INFINITY : fma((double)q, step, base);
}
// The slab test's final comparison with its 1e-9 relative padding. RT_TIGHT_PAD1: the padding applied once, to
// the interval ends t0 = max(0, tn_k), t1 = min(inf, tf_k), instead of to every axis' tn_k / tf_k before the max /
// min: x -> RN(x - RN(1e-9 |x|)) and x -> RN(x + RN(1e-9 |x|)) are non-decreasing in x (between adjacent doubles x
// moves by an ulp, the padding by 1e-9 of that), so they commute with max and min (and map 0 to 0, inf to inf),
// and the comparison is the per-axis form's, bit for bit, with 4 VALU instead of 12.
#ifndef RT_TIGHT_PAD1
#define RT_TIGHT_PAD1 1
#endif
RT_DEV bool tight_padded_le(double t0, double t1) {
#if RT_TIGHT_PAD1
    return t0 - 1e-9 * fabs(t0) <= t1 + 1e-9 * fabs(t1);
#else
    return t0 <= t1;
#endif
}
RT_DEV bool kid_tight_hit(const DevMesh& m, const int4& ks, const Ray& ray, const RayInv& inv) {
    const double step = m.tight_step;
    double t0 = 0.0, t1 = INFINITY;
    bool keep = true, force = false;
    // one axis of near_box's slab test (branch-free: no private arrays, no early exits)
    auto axis = [&](uint32_t ql, uint32_t qh, double base, double o, double d, double rc) {
        const double lo = tight_lo(ql, step, base);
        const double hi = tight_hi(qh, step, base);
        const bool inr = fabs(d) >= 0x1p-900 && fabs(d) <= 0x1p900;
        const bool tiny = fabs(d) < 0x1p-900;
        force |= !inr && !tiny;                      // NaN / huge: do not cull
        keep &= !tiny || (o >= lo && o <= hi);       // (nearly) parallel slab: origin must lie inside it
        const double ta = (lo - o) * rc, tb = (hi - o) * rc;
        const double tn = fmin(ta, tb), tf = fmax(ta, tb);
#if RT_TIGHT_PAD1
        t0 = inr ? fmax(t0, tn) : t0;
        t1 = inr ? fmin(t1, tf) : t1;
#else
        t0 = inr ? fmax(t0, tn - 1e-9 * fabs(tn)) : t0;
        t1 = inr ? fmin(t1, tf + 1e-9 * fabs(tf)) : t1;
#endif
    };
    axis((uint32_t)ks.y & 0xFFFFu, (uint32_t)ks.z >> 16, m.tight_base[0], ray.o.x, ray.d.x, inv.rx);
    axis((uint32_t)ks.y >> 16, (uint32_t)ks.w & 0xFFFFu, m.tight_base[1], ray.o.y, ray.d.y, inv.ry);
    axis((uint32_t)ks.z & 0xFFFFu, (uint32_t)ks.w >> 16, m.tight_base[2], ray.o.z, ray.d.z, inv.rz);
    return force || (keep && tight_padded_le(t0, t1));
}
// kid_tight_hit for rays whose direction components all lie in [2^-900, 2^900] in magnitude (every ray of
// the wave: walk_node_slots' wave vote), where its `inr` holds on every axis, so `force` and `keep` keep
// their initial values and every axis updates t0 / t1: the same operations on the same values, hence the
// same result, without the per-axis range logic.
#ifndef RT_TIGHT_FAST
#define RT_TIGHT_FAST 1  // A/B: 0 = always the general form
#endif
RT_DEV bool kid_tight_hit_inr(const DevMesh& m, const int4& ks, const Ray& ray, const RayInv& inv) {
    const double step = m.tight_step;
    double t0 = 0.0, t1 = INFINITY;
    auto axis = [&](uint32_t ql, uint32_t qh, double base, double o, double rc) {
        const double lo = tight_lo(ql, step, base);
        const double hi = tight_hi(qh, step, base);
        const double ta = (lo - o) * rc, tb = (hi - o) * rc;
        const double tn = fmin(ta, tb), tf = fmax(ta, tb);
#if RT_TIGHT_PAD1
        t0 = fmax(t0, tn);
        t1 = fmin(t1, tf);
#else
        t0 = fmax(t0, tn - 1e-9 * fabs(tn));
        t1 = fmin(t1, tf + 1e-9 * fabs(tf));
#endif
    };
    axis((uint32_t)ks.y & 0xFFFFu, (uint32_t)ks.z >> 16, m.tight_base[0], ray.o.x, inv.rx);
    axis((uint32_t)ks.y >> 16, (uint32_t)ks.w & 0xFFFFu, m.tight_base[1], ray.o.y, inv.ry);
    axis((uint32_t)ks.z & 0xFFFFu, (uint32_t)ks.w >> 16, m.tight_base[2], ray.o.z, inv.rz);
    return tight_padded_le(t0, t1);
}
// The slot of child octant oi of node `cur` (one 16-byte load: entry + bounds).
RT_DEV int4 kid_slot(const DevScene& sc, int32_t cur, uint32_t oi) {
    return *reinterpret_cast<const int4*>(sc.node_slot + 8 * (size_t)cur + oi);
}
// The node part of a walk step through the child slots (RT_WALK_TIGHT): as walk_node below, but a
// pick reads the child's 16-byte slot (entry + subtree triangle bounds) and skips children whose
// bounds the ray misses (up to two picks per step), and a descent takes the new node's existence
// mask from the entry (no load). `anc` (or null: the pid_up chain): this walk's LDS column of
// ancestor node ids at depths 0 .. kSlotAncLevels - 1 (stride 256 threads), written at each descent,
// so a pop reads the node it resumes at from LDS.
constexpr int kSlotAncLevels = 9;
#ifndef RT_POP_BOXLOAD
#define RT_POP_BOXLOAD 1  // A/B: a pop reloads the ancestor's box (1) or rebuilds it from the root (0)
#endif
#ifndef RT_SLOT_CULL
#define RT_SLOT_CULL 1  // A/B: 0 = the slot walk without the subtree-bounds test
#endif
#ifndef RT_LTRI_ID_HOIST
#define RT_LTRI_ID_HOIST 1  // the hoisted triangle loads also load the triangles' ids (leaf_tris_loaded: unicorn +1.5%, r04o), or not (0)
#endif
#ifndef RT_SLOT_PAIR
#define RT_SLOT_PAIR 1  // a pick loads the slots of the next two candidates together (1: unicorn +0.7%, r04j) or one by one (0)
#endif  // the deepest parents sit at depth 8 (MAX_DEPTH 10, root depth 1)
// What the next node operation will load, fetched ahead (RT_WALK_HOIST=2: at the start of the step,
// before its triangle tests): kind 1 = a pick at `cur` (its first candidate's slot), kind 2 = a pop to
// the ancestor `cur` at level `lv` (its box and its first candidate's slot), 0 = nothing (the root still
// to be entered, or exhausted). The node state this reads is not touched by the triangle tests, so the
// node operation after them starts from the same state and uses these values instead of loading.
// The deepest ancestor level lv < w.depth whose remaining-children mask pm (stk byte lv; level 8 in stk8) is
// non-zero, pm = 0 if none: branch-free (RT_POP_CLZ: the highest non-zero byte of the live part of stk by a
// count of leading zeros) instead of a loop over the levels, whose trip count is the largest over the wave's
// popping lanes. Parents sit at depths 0..8 of a walk (MAX_DEPTH 10), so w.depth <= 9 and lv <= 8.
#ifndef RT_POP_CLZ
#define RT_POP_CLZ 1
#endif
RT_DEV void pop_level(const OctWalk& w, int& lv, uint32_t& pm) {
#if RT_POP_CLZ
    const int d = w.depth;
    const int nb = min(d, 8);
    const uint64_t live = nb >= 8 ? w.stk : (w.stk & ((1ull << (8 * nb)) - 1ull));
    const int hb = 63 - __clzll((long long)(live | 1ull));  // (| 1: defined for live == 0, then byte 0 below)
    const int lb = hb >> 3;
    const uint32_t pb = (uint32_t)(live >> (8 * lb)) & 0xFFu;
    const bool at8 = d > 8 && w.stk8 != 0u;
    lv = at8 ? 8 : lb;
    pm = at8 ? w.stk8 : pb;
#else
    lv = w.depth;
    pm = 0;
    while (pm == 0 && lv > 0) {
        --lv;
        pm = lv < 8 ? (uint32_t)(w.stk >> (8 * lv)) & 0xFFu : w.stk8;
    }
#endif
}
struct SlotPF {
    int4 ks;
    double2 b0, b1, b2;
    int32_t cur, lv;
    uint32_t pm;
    int kind;
};
template <int AS = 256, class Anc = LdsAncI32>
RT_DEV void slot_prefetch(const DevScene& sc, const OctWalk& w, const Anc* anc, SlotPF& pf) {
    pf.kind = 0;
    if (w.enter & 1u) return;
    uint32_t pm = w.pm;
    int32_t cur = w.cur;
    if (pm == 0) {
        int lv = w.depth;
        while (pm == 0 && lv > 0) {
            --lv;
            pm = lv < 8 ? (uint32_t)(w.stk >> (8 * lv)) & 0xFFu : w.stk8;
        }
        if (pm == 0) return;
        if (anc) {
            cur = (int32_t)anc[lv * AS];
        } else {
            for (int l = w.depth; l > lv; --l) cur = sc.pid_up[cur];
        }
        const double2* nb = reinterpret_cast<const double2*>(sc.node_box + 6 * (size_t)cur);
        pf.b0 = nb[0];
        pf.b1 = nb[1];
        pf.b2 = nb[2];
        pf.lv = lv;
        pf.kind = 2;
    } else {
        pf.kind = 1;
    }
    pf.cur = cur;
    pf.pm = pm;
    pf.ks = *reinterpret_cast<const int4*>(sc.node_slot + 8 * (size_t)cur + ((w.order >> (4 * __builtin_ctz(pm))) & 0xF));
}
template <int AS = 256, class Anc = LdsAncI32>  // `anc`'s stride (the block's threads) and element type
RT_DEV int walk_node_slots(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, OctWalk& w,
                           Anc* anc = nullptr, const SlotPF* pf = nullptr) {
    RT_DBG_TSTART(t_pop);
    uint32_t exist = 0;  // a node to enter: its existence mask (the root at a walk's start, or a descent)
    if (w.enter & 1u) {
        w.enter &= ~1u;
        exist = (uint32_t)m.root_exist;
    } else {
    if (pf && pf->kind == 2) {  // the pop, its box fetched ahead (slot_prefetch)
        w.cur = pf->cur;
        w.depth = pf->lv;
        w.pm = pf->pm;
        w.path &= (1u << (3 * pf->lv)) - 1u;
        w.mn[0] = pf->b0.x; w.mn[1] = pf->b0.y; w.mn[2] = pf->b1.x;
        w.mx[0] = pf->b1.y; w.mx[1] = pf->b2.x; w.mx[2] = pf->b2.y;
    } else if (w.pm == 0) {  // `cur` exhausted: resume at the nearest ancestor with children left
        int lv;
        uint32_t pm;
        pop_level(w, lv, pm);
        if (pm == 0) {  // the root is exhausted
            RT_DBG_TEND(13, t_pop);
            return WALK_MISS;
        }
        if (anc) {
            w.cur = (int32_t)anc[lv * AS];
        } else {  // the parent chain by pid (rows of node_slot / node_box)
            int32_t cur = w.cur;
            for (int l = w.depth; l > lv; --l) cur = sc.pid_up[cur];
            w.cur = cur;
        }
        w.depth = lv;
        w.pm = pm;
        w.path &= (1u << (3 * lv)) - 1u;
#if RT_POP_BOXLOAD
        // the ancestor's box (DevScene::node_box: the same arithmetic as the descents); only a descent
        // from it reads the box, so the load overlaps the pick's slot load
        const double2* nb = reinterpret_cast<const double2*>(sc.node_box + 6 * (size_t)w.cur);
        const double2 b0 = nb[0], b1 = nb[1], b2 = nb[2];
        w.mn[0] = b0.x; w.mn[1] = b0.y; w.mn[2] = b1.x;
        w.mx[0] = b1.y; w.mx[1] = b2.x; w.mx[2] = b2.y;
#else
        // the ancestor's box, rebuilt from the root along the path (the build's own arithmetic)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            w.mn[k] = m.root_box[k];
            w.mx[k] = m.root_box[3 + k];
        }
        for (int l = 0; l < lv; ++l) {
            const uint32_t oi = (w.path >> (3 * l)) & 7u;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double c = (w.mn[k] + w.mx[k]) / 2.0;
                if ((oi >> (2 - k)) & 1u) w.mn[k] = c; else w.mx[k] = c;
            }
        }
#endif
    }
    RT_DBG_TEND(13, t_pop);
    RT_DBG_TSTART(t_pick);
    // the next child in visiting order whose subtree's triangle bounds the ray comes near; up to two
    // picks per step (a culled pick is as if the reference found nothing below that child)
    int32_t c = kKidEmpty;
    uint32_t oi = 0;
    // wave-uniform: one form of the test per step (each lane's dir_in_range from its walk's start, OctWalk::enter)
    const bool inr = RT_TIGHT_FAST && wave_all((w.enter & 2u) != 0u);
    auto tight = [&](const int4& ks) { return inr ? kid_tight_hit_inr(m, ks, ray, inv) : kid_tight_hit(m, ks, ray, inv); };
#if RT_SLOT_PAIR
    if (!pf) {
        // both candidates' slots loaded at once (one row of node_slot: the same 128-byte line), so a
        // culled first pick does not wait a second memory latency for the second
        const uint32_t pm1 = w.pm & (w.pm - 1u);
        const uint32_t oi1 = (w.order >> (4 * __builtin_ctz(w.pm))) & 0xF;
        const uint32_t oi2 = pm1 ? (w.order >> (4 * __builtin_ctz(pm1))) & 0xF : oi1;
        const int4 ks1 = kid_slot(sc, w.cur, oi1);
        const int4 ks2 = kid_slot(sc, w.cur, oi2);
        w.pm = pm1;
        oi = oi1;
        if (!RT_SLOT_CULL || tight(ks1)) {
            c = ks1.x;
        } else {
            RT_DBG(6);
            if (w.pm == 0) {  // nothing picked in this step
                RT_DBG_TEND(14, t_pick);
                return WALK_RUN;
            }
            w.pm &= w.pm - 1u;
            oi = oi2;
            if (!tight(ks2)) {
                RT_DBG(6);
                RT_DBG_TEND(14, t_pick);
                return WALK_RUN;
            }
            c = ks2.x;
        }
    } else
#endif
    for (int tries = 0; tries < 2; ++tries) {
        const int q = __builtin_ctz(w.pm);
        w.pm &= w.pm - 1u;
        oi = (w.order >> (4 * q)) & 0xF;
        const int4 ks = (pf && pf->kind != 0 && tries == 0) ? pf->ks : kid_slot(sc, w.cur, oi);
        if (!RT_SLOT_CULL || tight(ks)) {
            c = ks.x;
            break;
        }
        RT_DBG(6);
        if (w.pm == 0 || tries == 1) {  // nothing picked in this step
            RT_DBG_TEND(14, t_pick);
            return WALK_RUN;
        }
    }
    if (c <= -2) {  // open a leaf
        RT_DBG(3);
        const int32_t e = -2 - c;  // the leaf's range inline (kid_leaf), or its id behind the escape count
        int32_t first = e >> 6, cnt = e & 63;
        if (cnt == kKidCountEscape) {
            const int2 ls = sc.leaf_span[first];
            first = ls.x;
            cnt = ls.y;
        }
        if (w.lpos >= w.lend) {  // the triangle cursor is free: test this leaf next
            w.lpos = first;
            w.lend = first + cnt;
            w.best = -1;
        } else {  // the cursor is still on an earlier leaf: buffer this one (walk_step<true>)
            w.nlf = first;
            w.nle = first + cnt;
        }
        RT_DBG_TEND(14, t_pick);
        return WALK_RUN;
    }
    // descend: push the remaining mask of `cur`, take the octant's box
    const int lv = w.depth;
    if (anc) anc[lv * AS] = w.cur;  // (a pid: < 2^16 for a 16-bit column)
    if (lv < 8) w.stk = (w.stk & ~(0xFFull << (8 * lv))) | ((uint64_t)w.pm << (8 * lv));
    else w.stk8 = w.pm;
    w.path |= oi << (3 * lv);
    w.depth = lv + 1;
    w.cur = slot_node(c);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double cc = (w.mn[k] + w.mx[k]) / 2.0;
        if ((oi >> (2 - k)) & 1u) w.mn[k] = cc; else w.mx[k] = cc;
    }
    exist = slot_exist(c);
    RT_DBG_TEND(14, t_pick);
    }
    walk_enter_mask(ray, inv, w, exist);  // one octant_mask for the descents and the walks' starts
    return WALK_RUN;
}
// The node part of a walk step through node_kids (the reference's visiting order without the slot
// walk's subtree-bounds culls; RT_WALK_TIGHT=0 builds, the wavefront's walk kernels, scenes without
// slot tables): pops every exhausted level (the ancestor through the node_up links, its box rebuilt
// from the root), then picks the next child in visiting order and either opens it (a leaf: its
// triangle range in w.lpos / w.lend) or descends into it and masks its children (walk_enter).
// WALK_RUN, or WALK_MISS once the root is exhausted.
RT_DEV int walk_node(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, OctWalk& w) {
    RT_DBG_TSTART(t_pop);
    if (w.pm == 0) {  // `cur` exhausted: resume at the nearest ancestor with children left
        int lv = w.depth;
        uint32_t pm = 0;
        while (pm == 0 && lv > 0) {
            --lv;
            pm = lv < 8 ? (uint32_t)(w.stk >> (8 * lv)) & 0xFFu : w.stk8;
        }
        if (pm == 0) {  // the root is exhausted
            RT_DBG_TEND(13, t_pop);
            return WALK_MISS;
        }
        int32_t cur = w.cur;
        for (int l = w.depth; l > lv; --l) cur = sc.node_up[cur].x;
        w.cur = cur;
        w.depth = lv;
        w.pm = pm;
        w.path &= (1u << (3 * lv)) - 1u;
        // the ancestor's box, rebuilt from the root along the path (the build's own arithmetic)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            w.mn[k] = m.root_box[k];
            w.mx[k] = m.root_box[3 + k];
        }
        for (int l = 0; l < lv; ++l) {
            const uint32_t oi = (w.path >> (3 * l)) & 7u;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double c = (w.mn[k] + w.mx[k]) / 2.0;
                if ((oi >> (2 - k)) & 1u) w.mn[k] = c; else w.mx[k] = c;
            }
        }
    }
    RT_DBG_TEND(13, t_pop);
    RT_DBG_TSTART(t_pick);
    const int q = __builtin_ctz(w.pm);
    w.pm &= w.pm - 1u;
    const uint32_t oi = (w.order >> (4 * q)) & 0xF;
    const int32_t c = sc.node_kids[8 * (size_t)w.cur + oi];
    if (c <= -2) {  // open a leaf
        RT_DBG(3);
        const int32_t e = -2 - c;  // the leaf's range inline (kid_leaf), or its id behind the escape count
        int32_t first = e >> 6, cnt = e & 63;
        if (cnt == kKidCountEscape) {
            const int2 ls = sc.leaf_span[first];
            first = ls.x;
            cnt = ls.y;
        }
        w.lpos = first;
        w.lend = first + cnt;
        w.best = -1;
        RT_DBG_TEND(14, t_pick);
        return WALK_RUN;
    }
    // descend: push the remaining mask of `cur`, take the octant's box
    const int lv = w.depth;
    if (lv < 8) w.stk = (w.stk & ~(0xFFull << (8 * lv))) | ((uint64_t)w.pm << (8 * lv));
    else w.stk8 = w.pm;
    w.path |= oi << (3 * lv);
    w.depth = lv + 1;
    w.cur = c;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double cc = (w.mn[k] + w.mx[k]) / 2.0;
        if ((oi >> (2 - k)) & 1u) w.mn[k] = cc; else w.mx[k] = cc;
    }
    walk_enter(sc, ray, inv, w);
    RT_DBG_TEND(14, t_pick);
    return WALK_RUN;
}
// Slots = the slot walk (walk_node_slots, RT_WALK_TIGHT) or the node_kids walk (walk_node); both give
// the reference's result. (The wavefront's persistent walk kernels use the node_kids walk: the slot
// walk inlined there trips an AMDGPU backend error, "illegal VGPR to SGPR copy", in ROCm 7.2.)
// Hoist: RT_WALK_HOIST's modes (below); the Phong / mesh-light instances of the walk pool pass 0, where
// the hoisted triangles' registers would spill.
template <bool Slots = (RT_WALK_TIGHT != 0), int AS = 256, int Hoist = RT_WALK_HOIST, class Anc = LdsAncI32>
RT_DEV int walk_step(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, OctWalk& w, double* t,
                     int* prim, Anc* anc = nullptr) {
    RT_DBG(5);
    if constexpr (Slots) {
        // The node walk and the triangle tests run in the same step, one leaf apart: the node walk
        // advances (pop / pick / descend) while no found leaf waits in the buffer, and the open leaf's
        // next triangles are tested. Leaves are still tested in visiting order and the first leaf with
        // a hit ends the walk (a leaf the node walk found beyond it is dropped): the same result, in
        // fewer steps, with both parts of a step busy in most lanes.
        // Hoist 1: the open leaf's triangles (and their ids, RT_LTRI_ID_HOIST) are loaded BEFORE the node
        // operation: while a leaf is open the node walk only fills the one-leaf buffer (nlf / nle), so the
        // cursor stays as loaded and the slot load of the pick and the triangle loads are in flight
        // together (one memory latency per step instead of two in a row). A leaf the node walk opens into
        // a free cursor is tested from the next step: the same leaves in the same order, the same result.
        // Hoist 2: triangle tests first, with the next node operation's loads issued before them (the
        // pick's slot and a pop's box, slot_prefetch). Hoist 0: node operation, then leaf_tris.
        const bool open = w.lpos < w.lend;
        LeafTri tr[kTrisPerStep];
        int32_t tid[kTrisPerStep];
        if (Hoist != 0 && open) {
#pragma unroll
            for (int j = 0; j < kTrisPerStep; ++j) {
#if RT_LTRI_INDEX
                // leaf lists as triangle ids only (no ltris uploaded): the triangle from the 3.6 MB table, one
                // dependent load later (round 6: C4 -2.2%, C5 -3.7% against the copies, profiles/r06aa_ab_oct_ltidx.log)
                tid[j] = sc.ltri_id[min(w.lpos + j, w.lend - 1)];
                tr[j] = sc.tris[tid[j]];
#else
                tr[j] = sc.ltris[min(w.lpos + j, w.lend - 1)];
                if (RT_LTRI_ID_HOIST) tid[j] = sc.ltri_id[min(w.lpos + j, w.lend - 1)];
#endif
            }
        }
        SlotPF pf;
        pf.kind = 0;
        if constexpr (Hoist == 2) {
            if (!w.ndone) slot_prefetch<AS, Anc>(sc, w, anc, pf);
        } else {
            if (!w.ndone && w.nlf >= w.nle && walk_node_slots<AS, Anc>(sc, m, ray, inv, w, anc) == WALK_MISS) w.ndone = 1;
        }
        RT_DBG_TSTART(t_lt);
        if (Hoist != 0 ? open : w.lpos < w.lend) {
            const int st = Hoist != 0 ? leaf_tris_loaded(sc, ray, w, tr, t, prim, (RT_LTRI_ID_HOIST || RT_LTRI_INDEX) ? tid : nullptr)
                                      : leaf_tris(sc, ray, w, t, prim);
            if (st == WALK_HIT) {
                RT_DBG_TEND(12, t_lt);
                return WALK_HIT;
            }
            if (st < 0 && w.nlf < w.nle) {  // leaf done without a hit: the buffered one is next
                w.lpos = w.nlf;
                w.lend = w.nle;
                w.best = -1;
                w.nle = w.nlf;
            }
        }
        RT_DBG_TEND(12, t_lt);
        if constexpr (Hoist == 2) {
            if (!w.ndone && w.nlf >= w.nle && walk_node_slots<AS, Anc>(sc, m, ray, inv, w, anc, &pf) == WALK_MISS) w.ndone = 1;
        }
        return w.ndone && w.lpos >= w.lend && w.nlf >= w.nle ? WALK_MISS : WALK_RUN;
    }
    int st = -1;
    RT_DBG_TSTART(t_lt);
    if (w.lpos < w.lend) st = leaf_tris(sc, ray, w, t, prim);  // triangles of the open leaf
    RT_DBG_TEND(12, t_lt);
    if (st >= 0) return st;
    (void)anc;
    st = walk_node(sc, m, ray, inv, w);
#if RT_WALK_OPEN_TEST
    if (st == WALK_RUN && w.lpos < w.lend) {  // a leaf was just opened: its first triangles in this step
        const int s2 = leaf_tris(sc, ray, w, t, prim);
        return s2 >= 0 ? s2 : WALK_RUN;
    }
#endif
    return st;
}

// Mesh::intersect's `octree: None` branch (geometry.rs:886-903): the nearest triangle hit, strict <
// in triangle order (ties go to the lower index), found through the mesh's BVH: near child first
// (by the ray's direction along the split axis), far child on a per-lane stack in LDS. Boxes are
// culled with the padded slab test against the best t so far, so a triangle that could win is
// never skipped; the tie rule makes the result independent of the visiting order. tmax: a hit
// beyond it cannot be used by the caller (closest other object / shadow distance); hits at exactly
// tmax are kept (the caller's tie rule decides).
// bvh_step does one node per call (resumable, for the interleaved mesh kernel): WALK_RUN, or
// WALK_HIT with the nearest triangle in w.bt / w.best, or WALK_MISS. With shadow_dist >= 0 it
// returns as soon as a triangle blocks the shadow ray (t + 0.001 < dist, mutually_visible).
struct BvhWalk {
    int32_t cur, sp, best;
    double bt;
};
RT_DEV void bvh_begin(const DevMesh& m, double tmax, BvhWalk& w) {
    w.cur = m.bvh_base;
    w.sp = 0;
    w.best = -1;
    w.bt = tmax;
}
template <class Stack>
RT_DEV int bvh_step(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, BvhWalk& w,
                    const Stack& stk, double shadow_dist) {
    const DevBvhNode& nd = sc.bvh[w.cur];
    const double bx[6] = {nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2]};
    if (near_box(bx, ray, inv, m.cull_pad, w.bt)) {
        if (nd.count == 0) {
            const double dk = nd.axis == 0 ? ray.d.x : nd.axis == 1 ? ray.d.y : ray.d.z;
            const int l = w.cur + 1, r = nd.a;
            stk.at(w.sp) = dk < 0. ? l : r;  // far child
            ++w.sp;
            w.cur = dk < 0. ? r : l;
            return 0;  // WALK_RUN
        }
        for (int k = 0; k < nd.count; ++k) {
            double tt;
            const int id = sc.btri_id[nd.a + k];
            if (tri_t(sc.btris[nd.a + k], ray, &tt) && (tt < w.bt || (tt == w.bt && (w.best < 0 || id < w.best)))) {
                w.bt = tt;
                w.best = id;
            }
        }
        if (shadow_dist >= 0. && w.best >= 0 && !(w.bt + 0.001 >= shadow_dist)) return 1;  // blocked
    }
    if (w.sp == 0) return w.best >= 0 ? 1 : 2;  // WALK_HIT / WALK_MISS
    --w.sp;
    w.cur = stk.at(w.sp);
    return 0;
}
// Fused traversal (analytic megakernel, trace kernel): the stack in its own LDS array.
__shared__ int32_t s_bvh_stack[kBvhMaxDepth * 256];  // blocks of 256 threads
struct BvhLdsStack {
    typedef __attribute__((address_space(3))) int32_t LdsI32;
    LdsI32* p;
    RT_DEV LdsI32& at(int e) const { return p[e * 256]; }
};
RT_DEV bool mesh_hit_bvh(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, double tmax,
                         double* t, int* prim) {
    if (m.bvh_n <= 0) return false;
    const BvhLdsStack stk{(BvhLdsStack::LdsI32*)s_bvh_stack + threadIdx.x};
    BvhWalk w;
    bvh_begin(m, tmax, w);
    int st;
    while ((st = bvh_step(sc, m, ray, inv, w, stk, -1.0)) == 0) {
    }
    if (st != 1) return false;
    *t = w.bt;
    *prim = w.best;
    return true;
}

// Whole traversal in one call (megakernel / trace kernel).
template <bool Slots>
RT_DEV bool mesh_hit_walk(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, double tmax,
                          double* t, int* prim) {
    OctWalk w;
    if (!walk_begin<Slots>(sc, m, ray, inv, tmax, w)) return false;
    int st;
    while ((st = walk_step<Slots>(sc, m, ray, inv, w, t, prim)) == WALK_RUN) {
    }
    return st == WALK_HIT;
}
// The slot walk when the scene has its tables (DevScene::node_slot), else the node_kids walk.
RT_DEV bool mesh_hit(const DevScene& sc, const DevMesh& m, const Ray& ray, const RayInv& inv, double tmax, double* t,
                     int* prim) {
    if (RT_WALK_TIGHT && sc.node_slot) return mesh_hit_walk<true>(sc, m, ray, inv, tmax, t, prim);
    return mesh_hit_walk<false>(sc, m, ray, inv, tmax, t, prim);
}

// Kernel specialisation by scene features (chosen on the host per scene/flags): code paths a
// scene cannot reach are not compiled into its kernels, which keeps register pressure down.
template <int F>
struct Cfg {
    static constexpr bool mesh = (F & 1) != 0;   // scene has triangle meshes (octree traversal)
    static constexpr bool phong = (F & 2) != 0;  // scene has a Phong BRDF
    static constexpr bool mis = (F & 4) != 0;    // RT_FLAG_MIS
    static constexpr bool compact = (F & 8) != 0;  // scene fits the compact tables (DevScene)
    static constexpr bool bvh = (F & 16) != 0;     // RT_FLAG_MESH_NEAREST: nearest-triangle meshes via the BVH
    static constexpr bool nospec = (F & 32) != 0;  // no specular (mirror) object: the mirror paths compile out
    static constexpr bool ldsobj = (F & 64) != 0;  // the kernel holds the object table in LDS (rt_lds_objects)
};
constexpr int kCfgLdsObj = 64;

// The object table of compact scenes in LDS (16 x 208 B): a megakernel instantiated with Cfg bit 64
// copies DevScene::objects here at its start (lds_objects_fill), so the shading's per-lane object reads
// (hit object, light) are ds_reads instead of global loads. Only the kernels that reference it get it
// allocated.
__shared__ DevObject rt_lds_objects[kMaxCompactObjects];
template <class C>
RT_DEV const DevObject& object_at(const DevScene& sc, int i) {
    if constexpr (C::ldsobj) return rt_lds_objects[i];
    else return sc.objects[i];
}
RT_DEV void lds_objects_fill(const DevScene& sc) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(sc.objects);
    uint64_t* dst = reinterpret_cast<uint64_t*>(rt_lds_objects);
    const int nw = sc.n_objects * (int)(sizeof(DevObject) / 8);
    for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// Per-call view of the compact tables (scene_layout.h: CompactTab). The empty asm makes the pointer
// opaque, so the scalar loads through it are issued inside each trace call instead of being
// hoisted to the kernel entry, where the tables would hold ~100 SGPRs across the path loop.
// kSext = true is the round-4 first build's reconstruction, in which the builtin's int result of the low
// word sign-extended into the high word (an illegal address whenever hipMalloc placed the table at a low
// word with bit 31 set: profiles/r04_ab.log). Only rt_selftest_tables instantiates it, to show that its
// round-trip check catches that form; every trace call uses kSext = false.
template <bool kSext = false>
RT_DEV CTab* tables_form(const DevScene& sc) {
    uint64_t p = (uint64_t)(uintptr_t)sc.ctab;
    // (uniform: readfirstlane keeps the asm's SGPR operand legal where the compiler holds it in a VGPR)
    // (the builtin returns int: through uint32_t, or the low word's sign would fill the high word)
    if constexpr (kSext)
        p = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)) << 32);
    else
        p = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)) << 32);
    asm volatile("" : "+s"(p));
    return (CTab*)p;
}
RT_DEV CTab* tables(const DevScene& sc) { return tables_form<false>(sc); }

// One object's Geometry::intersect, reporting t (and the triangle for meshes).
template <class C>
RT_DEV bool object_t(const DevScene& sc, const DevObject& o, const Ray& ray, const RayInv& inv, double* t, int* prim,
                     double tmax = INFINITY) {
    if (o.geom == GEOM_SPHERE) return sphere_t(o, ray, t);
    if (o.geom == GEOM_PLANE) return plane_t(o, ray, inv, t);
    if constexpr (C::mesh && C::bvh) return mesh_hit_bvh(sc, sc.meshes[o.mesh], ray, inv, tmax, t, prim);
    if constexpr (C::mesh && !C::bvh) return mesh_hit(sc, sc.meshes[o.mesh], ray, inv, tmax, t, prim);
    return false;
}

// Geometry::intersect of a sphere or plane only (the analytic halves of the deferred queries: no
// octree walk is compiled in, which the generic object_t would inline for a non-sphere/plane geom).
RT_DEV bool analytic_t(const DevObject& o, const Ray& ray, const RayInv& inv, double* t) {
    if (o.geom == GEOM_SPHERE) return sphere_t(o, ray, t);
    if (o.geom == GEOM_PLANE) return plane_t(o, ray, inv, t);
    return false;
}

struct HitRec {
    double t;
    int obj;   // -1: no hit
    int prim;  // triangle (meshes)
};

// Scene::trace_ray (scene.rs:272-289): nearest over all objects, ties to the lower index.
RT_DEV void consider(HitRec& h, double t, int idx, int prim) {
    if (h.obj < 0 || t < h.t || (t == h.t && idx < h.obj)) { h.t = t; h.obj = idx; h.prim = prim; }
}
// Sphere test on the compact table (same operations as sphere_t; r*r precomputed exactly).
// (Conservative culls of spheres beyond tmax / below eps before the square root measured 4% slower
// on cornell_box: the extra compares cost more than the divergent roots they skip.)
template <class P>
RT_DEV bool sphere_c(P c, const Ray& ray, double* tout) {
    V3 op = v3(c[0], c[1], c[2]) - ray.o;
    double b = dot(op, ray.d);
    double det = b * b - dot(op, op) + c[3];
    if (det < 0.) return false;
    RT_DBG_REGION(11);
    det = sqrt_rn(det);
    double t = b - det;
    if (t > 1e-4) { *tout = t; return true; }
    t = b + det;
    if (t > 1e-4) { *tout = t; return true; }
    return false;
}
// Axis planes of axis K: one |d_K| test and one reciprocal serve all of them (plane_t's axis path).
template <int K, class Visit>
RT_DEV void axis_planes(const DevScene& sc, CTab* T, const Ray& ray, const RayInv& inv, Visit&& visit) {
    const int n = T->n_ax[K];
    if (n == 0) return;
    const double dk = K == 0 ? ray.d.x : K == 1 ? ray.d.y : ray.d.z;
    if (fabs(dk) < 0.0001) return;
    const double ok = K == 0 ? ray.o.x : K == 1 ? ray.o.y : ray.o.z;
#pragma unroll
    for (int i = 0; i < kMaxAxisPlanes; ++i) {
        if (i < n) {
            double num = T->ax_pos[K][i] - ok;
            double t = K == 0 ? div_x(num, ray, inv) : K == 1 ? div_y(num, ray, inv) : div_z(num, ray, inv);
            if (t >= 0.) visit(t, T->ax_idx[K][i], -1);
        }
    }
}

template <class C>
RT_DEV HitRec trace_closest(const DevScene& sc, const Ray& ray) {
    RT_DBG_REGION(12);
    CTab* T = tables(sc);
    HitRec h{0.0, -1, -1};
    RT_DBG_TSTART(t_pl);
    const RayInv inv = make_inv(ray.d);
    if constexpr (C::compact) {
        auto visit = [&](double t, int idx, int prim) { consider(h, t, idx, prim); };
        axis_planes<0>(sc, T, ray, inv, visit);
        axis_planes<1>(sc, T, ray, inv, visit);
        axis_planes<2>(sc, T, ray, inv, visit);
        RT_DBG_TEND(13, t_pl);
        RT_DBG_TSTART(t_sp);
#pragma unroll
        for (int i = 0; i < kMaxSpheres; ++i) {
            double t;
            if (i < T->n_sph && sphere_c(T->sph[i], ray, &t)) consider(h, t, T->sph_idx[i], -1);
        }
        RT_DBG_TEND(14, t_sp);
        for (int i = 0; i < T->n_gen; ++i) {
            const int idx = T->gen_idx[i];
            double t;
            int prim = -1;
            const double tmax = h.obj >= 0 ? h.t : INFINITY;
            if (object_t<C>(sc, object_at<C>(sc, idx), ray, inv, &t, &prim, tmax)) consider(h, t, idx, prim);
        }
        return h;
    }
    for (int i = 0; i < sc.n_objects; ++i) {
        const DevObject& o = object_at<C>(sc, i);
        double t;
        int prim = -1;
        if (object_t<C>(sc, o, ray, inv, &t, &prim)) {
            if (h.obj < 0 || t < h.t) { h.t = t; h.obj = i; h.prim = prim; }
        }
    }
    return h;
}

// Hit position and facing normal, computed exactly as the intersect routines build their Hit.
template <class C>
RT_DEV void surface(const DevScene& sc, const Ray& ray, const HitRec& h, V3* pos, V3* n) {
    const DevObject& o = object_at<C>(sc, h.obj);
    if (o.geom == GEOM_SPHERE) {
        V3 p = eval(ray, h.t);
        V3 nn = norm(p - ld3(o.pos));
        *pos = p;
        *n = dot(nn, -ray.d) >= 0. ? nn : -nn;
    } else if (o.geom == GEOM_PLANE) {
        V3 pn = ld3(o.n);
        V3 nn = dot(pn, -ray.d) >= 0. ? pn : -pn;
        *pos = eval(ray, h.t) + nn * 0.00001;
        *n = nn;
    } else if constexpr (C::mesh) {
        V3 tn = ld3(sc.tris[h.prim].n);
        V3 nn = dot(tn, -ray.d) >= 0. ? tn : -tn;
        *pos = eval(ray, h.t) + 0.00001 * nn;
        *n = nn;
    }
}

// Scene::mutually_visible (scene.rs:258-270) as an any-hit query: occluded iff some object's
// intersect t satisfies t + 0.001 < |y - x| (equivalent to the nearest-hit test because x + 0.001
// rounds monotonically). Analytic objects are tested before meshes (order-free for a boolean).
// r = {x, norm(y - x)} and dist = mag(y - x) as the caller computed them (visible() below, or the
// NEE term's own values: same bits).
//
// Axis planes: a plane with both endpoints strictly on one side cannot block (exact; DESIGN.md §2:
// behind x its t < 0, beyond y its t >= |y - x| (1 - 2^-52) and t + 0.001 >= |y - x| for
// |y - x| < 1e9), so the exact plane test (and the ray reciprocals it needs) runs only for lanes
// whose segment crosses or touches a plane.
template <int K>
RT_DEV bool planes_clear(CTab* T, double xk, double yk) {
    bool c = true;
#pragma unroll
    for (int i = 0; i < kMaxAxisPlanes; ++i) {
        if (i < T->n_ax[K]) {
            const double p = T->ax_pos[K][i];
            c &= (xk < p && yk < p) || (xk > p && yk > p);
        }
    }
    return c;
}
template <class C>
RT_DEV bool visible_ray(const DevScene& sc, V3 y, const Ray& r, double dist) {
    RT_DBG_REGION(13);
    CTab* T = tables(sc);
    const double ERR_MARGIN = 0.001;
    if constexpr (C::compact) {
        bool occluded = false;
        auto visit = [&](double t, int, int) { occluded |= !(t + ERR_MARGIN >= dist); };
        const bool clear = dist < 1e9 && planes_clear<0>(T, r.o.x, y.x) && planes_clear<1>(T, r.o.y, y.y) &&
                           planes_clear<2>(T, r.o.z, y.z);
        RayInv inv;
        const bool gen = T->n_gen > 0;  // the generic intersectors use the reciprocals too
        if (gen) inv = make_inv(r.d);
        if (!clear) {
            if (!gen) inv = make_inv(r.d);
            axis_planes<0>(sc, T, r, inv, visit);
            axis_planes<1>(sc, T, r, inv, visit);
            axis_planes<2>(sc, T, r, inv, visit);
        }
#pragma unroll
        for (int i = 0; i < kMaxSpheres; ++i) {
            double t;
            if (i < T->n_sph && sphere_c(T->sph[i], r, &t)) occluded |= !(t + ERR_MARGIN >= dist);
        }
        if (occluded) return false;
        for (int i = 0; i < T->n_gen; ++i) {
            double t;
            int prim;
            if (object_t<C>(sc, object_at<C>(sc, T->gen_idx[i]), r, inv, &t, &prim, dist) && !(t + ERR_MARGIN >= dist))
                return false;
        }
        return true;
    }
    const RayInv inv = make_inv(r.d);
    for (int pass = 0; pass < (C::mesh ? 2 : 1); ++pass) {
        for (int i = 0; i < sc.n_objects; ++i) {
            const DevObject& o = object_at<C>(sc, i);
            if ((o.geom == GEOM_MESH) != (pass == 1)) continue;
            double t;
            int prim;
            if (object_t<C>(sc, o, r, inv, &t, &prim, dist) && !(t + ERR_MARGIN >= dist)) return false;
        }
    }
    return true;
}

template <class C>
RT_DEV bool visible(const DevScene& sc, V3 x, V3 y) {
    V3 diff = y - x;
    double dist = mag(diff);
    return visible_ray<C>(sc, y, Ray{x, diff / dist}, dist);  // norm(diff), sharing the magnitude
}

// ---- pieces of trace_ray / mutually_visible for the wavefront's deferred mesh queries ----
// (compact scenes only: analytic objects = axis planes, spheres, and non-mesh generic objects)
template <class C>
RT_DEV HitRec trace_analytic(const DevScene& sc, const Ray& ray, const RayInv& inv) {
    CTab* T = tables(sc);
    HitRec h{0.0, -1, -1};
    auto visit = [&](double t, int idx, int prim) { consider(h, t, idx, prim); };
    axis_planes<0>(sc, T, ray, inv, visit);
    axis_planes<1>(sc, T, ray, inv, visit);
    axis_planes<2>(sc, T, ray, inv, visit);
#pragma unroll
    for (int i = 0; i < kMaxSpheres; ++i) {
        double t;
        if (i < T->n_sph && sphere_c(T->sph[i], ray, &t)) consider(h, t, T->sph_idx[i], -1);
    }
    for (int i = 0; i < T->n_gen; ++i) {
        if (!((T->gen_analytic >> i) & 1u)) continue;  // a mesh: analytic_t cannot hit it
        const int idx = T->gen_idx[i];
        const DevObject& o = object_at<C>(sc, idx);
        double t;
        if (analytic_t(o, ray, inv, &t)) consider(h, t, idx, -1);
    }
    return h;
}
// Adds the meshes' hits to an analytic closest hit (Scene::trace_ray's loop over the mesh objects).
template <class C>
RT_DEV void trace_meshes(const DevScene& sc, const Ray& ray, const RayInv& inv, HitRec& h) {
    CTab* T = tables(sc);
    for (int i = 0; i < T->n_gen; ++i) {
        const int idx = T->gen_idx[i];
        const DevObject& o = object_at<C>(sc, idx);
        if (o.geom != GEOM_MESH) continue;
        double t;
        int prim = -1;
        if (mesh_hit(sc, sc.meshes[o.mesh], ray, inv, h.obj >= 0 ? h.t : INFINITY, &t, &prim)) consider(h, t, idx, prim);
    }
}
// near_box's cull in single precision, padded so that it passes every ray near_box passes (a cull may
// only let more rays through: a mesh walk or query for a ray it could have skipped returns the
// reference's result anyway). The ray is rounded to f32 (|o32 - o| <= 2^-24 |o|, |d32 - d| <= 2^-24
// for |d| = 1) and the slab arithmetic adds a few f32 roundings; within the distances where the ray
// can meet the box (t <= |o| + 4 S for a box inside [-S, S]^3) all of it moves the ray's points by less
// than 2^-21 (|o| + S). The box is padded by pad = 2^-16 (max |o_k| + S), 16x that (and 30x the f64
// test's own 1e-7 S pad), and the interval ends are compared with the same slack.
// c: the cull32 box (6 floats, any address space), s: cull32_s.
template <class CP>
RT_DEV bool near_cull32(CP c, float s, const Ray& ray, double tmax) {
    const float o[3] = {(float)ray.o.x, (float)ray.o.y, (float)ray.o.z};
    const float d[3] = {(float)ray.d.x, (float)ray.d.y, (float)ray.d.z};
    const float pad = 0x1p-16f * (fmaxf(fabsf(o[0]), fmaxf(fabsf(o[1]), fabsf(o[2]))) + s);
    float t0 = 0.0f, t1 = INFINITY;
    bool keep = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float lo = c[k] - pad, hi = c[3 + k] + pad;
        const bool tiny = !(fabsf(d[k]) >= 0x1p-60f);  // (nearly) parallel slab (or NaN): origin inside it
        keep &= !tiny || !(o[k] < lo || o[k] > hi);
        const float rc = __builtin_amdgcn_rcpf(d[k]);
        const float ta = (lo - o[k]) * rc, tb = (hi - o[k]) * rc;
        t0 = tiny ? t0 : fmaxf(t0, fminf(ta, tb));
        t1 = tiny ? t1 : fminf(t1, fmaxf(ta, tb));
    }
    const float tm = (float)tmax;
    return keep && !(t0 > t1 + 0x1p-16f * fabsf(t1) + pad) && !(t0 > tm + 0x1p-16f * tm + pad);
}
RT_DEV bool near_mesh32(const DevMesh& m, const Ray& ray, double tmax) { return near_cull32(m.cull32, m.cull32_s, ray, tmax); }
#ifndef RT_NEAR32
#define RT_NEAR32 1  // A/B: the meshes' near test in f32 (near_mesh32) or f64 (near_box)
#endif
// Which meshes could change this ray's result (closest hit so far at tmax / shadow distance tmax)?
// Bit m: mesh m (non-empty octree) passes the near test against its cull box.
template <class C>
RT_DEV uint32_t mesh_near_mask(const DevScene& sc, const Ray& ray, const RayInv& inv, double tmax) {
    CTab* T = tables(sc);
    uint32_t mask = 0;
    for (int i = 0; i < T->n_gen; ++i) {
#if RT_NEAR32
        // the slot's mesh and its f32 cull box from the compact table (no object / mesh reads)
        (void)inv;
        const int mm = T->gen_mesh[i];
        if (mm >= 0) mask |= near_cull32(T->gen_cull32[i], T->gen_cull32[i][6], ray, tmax) ? 1u << mm : 0u;
#else
        const DevObject& o = object_at<C>(sc, T->gen_idx[i]);
        if (o.geom == GEOM_MESH && sc.meshes[o.mesh].n_nodes > 0) {
            const DevMesh& m = sc.meshes[o.mesh];
            mask |= near_box(m.cull_box, ray, inv, m.cull_pad, tmax) ? 1u << o.mesh : 0u;
        }
#endif
    }
    return mask;
}
template <class C>
RT_DEV bool mesh_candidate(const DevScene& sc, const Ray& ray, const RayInv& inv, double tmax) {
    return mesh_near_mask<C>(sc, ray, inv, tmax) != 0;
}
// mutually_visible split: the analytic objects here, the meshes later (mesh_occludes).
template <class C>
RT_DEV bool visible_analytic(const DevScene& sc, V3 y, const Ray& r, double dist) {
    CTab* T = tables(sc);
    const double ERR_MARGIN = 0.001;
    bool occluded = false;
    auto visit = [&](double t, int, int) { occluded |= !(t + ERR_MARGIN >= dist); };
    const bool clear = dist < 1e9 && planes_clear<0>(T, r.o.x, y.x) && planes_clear<1>(T, r.o.y, y.y) &&
                       planes_clear<2>(T, r.o.z, y.z);
    // the ray reciprocals only where they are used (make_inv's wave vote makes it a convergent call
    // the compiler cannot sink into these branches itself; its result is the same bits either way)
    if (!clear) {
        const RayInv inv = make_inv(r.d);
        axis_planes<0>(sc, T, r, inv, visit);
        axis_planes<1>(sc, T, r, inv, visit);
        axis_planes<2>(sc, T, r, inv, visit);
    }
#pragma unroll
    for (int i = 0; i < kMaxSpheres; ++i) {
        double t;
        if (i < T->n_sph && sphere_c(T->sph[i], r, &t)) occluded |= !(t + ERR_MARGIN >= dist);
    }
    if (occluded) return false;
    if (T->gen_analytic) {
        const RayInv inv = make_inv(r.d);
        for (int i = 0; i < T->n_gen; ++i) {
            if (!((T->gen_analytic >> i) & 1u)) continue;  // a mesh: analytic_t cannot hit it
            const DevObject& o = object_at<C>(sc, T->gen_idx[i]);
            double t;
            if (analytic_t(o, r, inv, &t) && !(t + ERR_MARGIN >= dist)) return false;
        }
    }
    return true;
}
template <class C>
RT_DEV bool mesh_occludes(const DevScene& sc, const Ray& r, const RayInv& inv, double dist) {
    CTab* T = tables(sc);
    const double ERR_MARGIN = 0.001;
    for (int i = 0; i < T->n_gen; ++i) {
        const DevObject& o = object_at<C>(sc, T->gen_idx[i]);
        if (o.geom != GEOM_MESH) continue;
        double t;
        int prim;
        if (mesh_hit(sc, sc.meshes[o.mesh], r, inv, dist, &t, &prim) && !(t + ERR_MARGIN >= dist)) return true;
    }
    return false;
}

// ---------------------------------------------------------------- BRDF (scene.rs:30-123)
template <class C>
RT_DEV V3 brdf_eval(const DevObject& o, V3 n, V3 out, V3 in) {
#ifndef RT_OPT_KPI
#define RT_OPT_KPI 1  // A/B: diffuse f = kd * FRAC_1_PI read from the object (host-evaluated, same bits)
#endif
    // (every object of a scene without Phong or mirror objects is diffuse)
    if ((C::nospec && !C::phong) || o.brdf == BRDF_DIFFUSE) return RT_OPT_KPI ? ld3(o.kpi) : ld3(o.k) * FRAC_1_PI;
    if (!C::phong || o.brdf == BRDF_SPECULAR) {
        if (equal_within(in, flip_across(out, n), 0.001)) return ld3(o.k) / dot(n, in);
        return v3(0, 0, 0);
    }
    V3 refl = flip_across(in, n);
    double c = fmax(dot(out, refl), 0.);
    return ld3(o.color_d) * o.ph_kd * FRAC_1_PI +
           ld3(o.color_s) * o.ph_ks * (double)(o.ph_power + 2) / (2. * PI) * powi(c, o.ph_power);
}
RT_DEV void local_coord(V3 n, V3* u, V3* v, V3* w) {
    *w = n;
    V3 base = fabs(w->x) > 0.1 ? v3(0., 1., 0.) : v3(1., 0., 0.);
    *u = norm(cross(base, *w));
    *v = cross(*w, *u);
}
// sample_incoming (scene.rs:56-98); draws: u1 = d[3], u2 = d[4], u3 = d[5].
template <class C>
RT_DEV void brdf_sample(const DevObject& o, V3 n, V3 out, Rng& rng, V3* in, double* pdf) {
    if ((C::nospec && !C::phong) || o.brdf == BRDF_DIFFUSE) {
        double z = sqrt_rn(rng.uniform());
        double r = sqrt_rn(1.0 - z * z);
        double phi = 2.0 * PI * rng.uniform();
        double sphi, cphi;
        sincos_2pi(phi, &sphi, &cphi);
        double x = r * cphi, y = r * sphi;
        V3 u, v, w;
        local_coord(n, &u, &v, &w);
        V3 i = norm(u * x + v * y + w * z);
        *in = i;
        *pdf = dot(n, i) * FRAC_1_PI;
        return;
    }
    if (!C::phong || o.brdf == BRDF_SPECULAR) {
        *in = flip_across(out, n);
        *pdf = 1.0;
        return;
    }
    double p = (double)o.ph_power;
    double u = rng.uniform();
    if (u < o.ph_kd) {
        double xi1 = rng.uniform(), xi2 = rng.uniform();
        double sp, cp;
        sincos_2pi(2. * PI * xi2, &sp, &cp);
        V3 i = v3(sqrt(1. - xi1) * cp, sqrt(1. - xi1) * sp, sqrt(xi1));
        *in = i;
        *pdf = dot(n, i) * FRAC_1_PI;
    } else if (o.ph_kd <= u && u < o.ph_kd + o.ph_ks) {
        double xi1 = rng.uniform(), xi2 = rng.uniform();
        double sp, cp;
        sincos_2pi(2. * PI * xi2, &sp, &cp);
        V3 i = v3(sqrt(1. - pow(xi1, 2. / (p + 1.))) * cp, sqrt(1. - pow(xi1, 2. / (p + 1.))) * sp,
                  pow(xi1, 1. / (p + 1.)));
        *in = i;
        *pdf = (p + 1.) / (2. * PI) * powi(i.z, o.ph_power);
    } else {
        *in = v3(0, 0, 0);
        *pdf = 1.0;
    }
}

// ---------------------------------------------------------------- light (geometry.rs:573-595)
template <class C>
RT_DEV void light_sample(const DevScene& sc, Rng& rng, V3* y, V3* ny, double* pdf) {
    const DevObject& L = object_at<C>(sc, sc.light);
    if (!C::mesh || L.geom == GEOM_SPHERE) {
        double xi1 = rng.uniform(), xi2 = rng.uniform();
        double z = 2. * xi1 - 1.;
        double sp, cp;
        sincos_2pi(2. * PI * xi2, &sp, &cp);
        const double sz = sqrt_rn(1.0 - z * z);
        double x = sz * cp;
        double yy = sz * sp;
        V3 n = norm(v3(x, yy, z));
        *y = ld3(L.pos) + n * L.r;
        *ny = n;
        *pdf = sc.light_pdf;  // 1.0 / (4.0 * PI * L.r * L.r), same bits (host, rt_api.cpp: upload)
        return;
    }
    // mesh light: area-weighted pick + Triangle::sample with the reference's missing `+ a`
    const DevMesh& m = sc.meshes[L.mesh];
    double u = rng.uniform() * m.total_weight;
    int lo = 0, hi = m.n_tris - 1;  // first triangle whose cumulative area > u
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (sc.tri_cum_area[m.tri_base + mid] > u) hi = mid;
        else lo = mid + 1;
    }
    const DevTri& t = sc.tris[m.tri_base + lo];
    double b0 = 1. - sqrt(rng.uniform());
    double b1 = (1. - b0) * rng.uniform();
    V3 ab = norm(ld3(t.ab)), ac = norm(ld3(t.ac));
    *y = ab * b0 + ac * b1;
    *ny = ld3(t.n);
    *pdf = 1. / m.surface_area;
}
RT_DEV double light_pdf_area(const DevScene& sc) { return sc.light_pdf; }

// Camera ray of server.rs:339-357 for subpixel (sx, sy) of pixel (x, y_ref).
RT_DEV Ray camera_ray(const DevScene& sc, V3 cx, V3 cy, double w, double h, int x, int y, int sx, int sy, double u1,
                      double u2) {
    // the tent filter's two square roots, one per branch in the reference, as one sqrt_rn of the selected
    // radicand per axis (sqrt_rn == sqrt bit for bit; the library form only where a wave holds a 0 or tiny one)
    double r1 = 2. * u1;
    const double q1 = sqrt_rn(r1 < 1. ? r1 : 2. - r1);
    double dx = r1 < 1. ? q1 - 1. : 1. - q1;
    double r2 = 2. * u2;
    const double q2 = sqrt_rn(r2 < 1. ? r2 : 2. - r2);
    double dy = r2 < 1. ? q2 - 1. : 1. - q2;
    // w, h are image sizes in [1, 2^32]: the shared-divisor division is exact (qdiv)
    V3 d = cx * (qdiv(((double)sx + 0.5 + dx) / 2. + (double)x, w, rcp_rn(w)) - 0.5) +
           cy * (qdiv(((double)sy + 0.5 + dy) / 2. + (double)y, h, rcp_rn(h)) - 0.5) + ld3(sc.cam_dir);
    return Ray{ld3(sc.cam_pos), norm(d)};
}

RT_DEV uint8_t as_u8(double v) {  // Rust `as u8`: saturating, NaN -> 0
    if (!(v > 0.)) return 0;
    if (v >= 255.) return 255;
    return (uint8_t)v;
}

}  // namespace f64
}  // namespace rt
