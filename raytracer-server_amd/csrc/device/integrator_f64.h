// Per-vertex integrator shared by the megakernel and the wavefront shade kernel.
//
// The reference's recursion (scene.rs:152-244) restated as a forward walk with throughput:
//   received_radiance(r)  = Le(x1) + R(x1, -d, 1)                                   (:152-159)
//   R(x, o, k), mirror    = [u < p] ( Le(x') + R(x', o, k+1) * f cos / (pdf p) )    (:170-185)
//   R(x, o, k), diffuse   = NEE(x, o) + [u < p] R(x', -i, k+1) * f cos / (pdf p)    (:217-242)
// so, walking forward with beta = product of the weights so far:
//   camera hit:  L  = Le(x1)
//   mirror:      L += beta (.) Le(x'),  beta (.)= f cos / (pdf p)   (Le(x') is NOT weighted by
//                this vertex's f cos / (pdf p) — exactly as in the reference expression)
//   diffuse:     L += beta (.) NEE,     beta (.)= f cos / (pdf p)
// `o` stays unchanged across a mirror bounce (the reference passes the same `o`, scene.rs:178).
// Sums are taken in a different association than the recursion, so f64 results agree with the
// recursive oracle to ~1e-15 relative, not bit for bit.
#pragma once

#include "../kernels/kernels.h"
#include "path_f64.h"

// A/B switches of the shading restructure (1 = on)
#ifndef RT_OPT_SPEC
#define RT_OPT_SPEC 1  // mirror vertices share the RR + continuation code of diffuse vertices
#endif
#ifndef RT_OPT_VIS
#define RT_OPT_VIS 1   // the shadow ray reuses norm(y - x) and |y - x| of the NEE term
#endif
#ifndef RT_OPT_LEF
#define RT_OPT_LEF 1   // diffuse NEE: Le * f precomputed per object (DevObject::lef)
#endif
#ifndef RT_OPT_RR
#define RT_OPT_RR 1    // Russian roulette as an integer comparison of the draw (Rng::below53)
#endif
#ifndef RT_OPT_NEE
#define RT_OPT_NEE 1   // the NEE term's scalar factors through one reciprocal (MIS: the weight cancelled)
#endif
#ifndef RT_OPT_BETA
#define RT_OPT_BETA 1  // continuation weight f cos / (pdf p) as k / p (diffuse and mirror vertices)
#endif

namespace rt {
namespace f64 {

enum : int { K_CAMERA = 0, K_SPEC = 1, K_DIFF = 2 };
constexpr double kInvSurvival = 1.0 / SURVIVAL_PROBABILITY;

struct PathState {
    Ray ray;
    V3 beta, L, bemit, o;
    double pdf_prev;
    uint64_t r0, r1;  // this sample's RNG stream (xoroshiro128++ state)
    uint32_t depth;
    int kind;
};

// Tile-local subpixel id -> pixel coordinates (RenderJob::run flips y, server.rs:181).
struct SubPixel {
    uint32_t pid;  // global pixel id (RNG key)
    int col, yref, sx, sy, sub;
};
RT_DEV SubPixel subpixel_of(const RenderArgs& a, long p) {
    const uint32_t pix = (uint32_t)(p >> 2);  // < width * height < 2^32 (rt_api.cpp: check_params)
    const uint32_t tw = (uint32_t)a.tw;
    const uint32_t r = pix / tw;
    SubPixel s;
    s.sub = (int)(p & 3);
    s.col = a.x0 + (int)(pix - r * tw);
    int row = a.y0 + (int)r * a.row_step;
    s.yref = a.height - row - 1;
    s.pid = (uint32_t)row * (uint32_t)a.width + (uint32_t)s.col;
    s.sx = s.sub & 1;
    s.sy = s.sub >> 1;
    return s;
}

// Camera ray of sample `smp` of subpixel `sp` (server.rs:338-357): its direction and the sample's
// RNG stream after the two camera draws.
struct CameraSample {
    V3 d;
    uint64_t r0, r1;
};
RT_DEV CameraSample camera_sample(const DevScene& sc, const RenderArgs& a, const SubPixel& sp, int smp) {
    Rng rng(a.seed, sp.pid, (uint32_t)smp, (uint32_t)sp.sub);
    double u1 = rng.uniform(), u2 = rng.uniform();
    const Ray r = camera_ray(sc, ld3(a.cx), ld3(a.cy), (double)a.width, (double)a.height, sp.col, sp.yref, sp.sx, sp.sy,
                             u1, u2);
    return CameraSample{r.d, rng.s0, rng.s1};
}
// New camera path from a camera sample.
RT_DEV void begin_path(const DevScene& sc, const CameraSample& cs, PathState& ps) {
    ps.r0 = cs.r0;
    ps.r1 = cs.r1;
    ps.ray = Ray{ld3(sc.cam_pos), cs.d};
    ps.beta = v3(1, 1, 1);
    ps.L = v3(0, 0, 0);
    ps.bemit = v3(0, 0, 0);
    ps.o = v3(0, 0, 0);
    ps.pdf_prev = 0.0;
    ps.depth = 0;
    ps.kind = K_CAMERA;
}
// New camera path for sample `smp` of subpixel `sp` (server.rs:338-357).
RT_DEV void begin_sample(const DevScene& sc, const RenderArgs& a, const SubPixel& sp, int smp, PathState& ps) {
    Rng rng(a.seed, sp.pid, (uint32_t)smp, (uint32_t)sp.sub);
    double u1 = rng.uniform(), u2 = rng.uniform();
    ps.r0 = rng.s0;
    ps.r1 = rng.s1;
    ps.ray = camera_ray(sc, ld3(a.cx), ld3(a.cy), (double)a.width, (double)a.height, sp.col, sp.yref, sp.sx, sp.sy, u1, u2);
    ps.beta = v3(1, 1, 1);
    ps.L = v3(0, 0, 0);
    ps.bemit = v3(0, 0, 0);
    ps.o = v3(0, 0, 0);
    ps.pdf_prev = 0.0;
    ps.depth = 0;
    ps.kind = K_CAMERA;
}

// A shadow ray whose mesh test is deferred to the wavefront's k_wf_shadow_mesh (the analytic
// objects already let it through). `c` is the NEE term already weighted by the path throughput.
struct ShadowDefer {
    bool pending;
    V3 o, d, c;
    double dist;
    uint32_t meshes;  // the meshes near the shadow segment (mesh_near_mask): the ones that could block it
    RayInv inv;       // make_inv(d), for the deferred query
};

// Where a deferred shadow query's ray goes (ShadowDefer): NoSink returns it in the ShadowDefer (o, d,
// dist, inv); a column sink writes o, d and dist straight into the owner's LDS query columns the moment
// shade_vertex finds the query pending, so the six doubles are not held in registers through the rest
// of the vertex (the query-pool kernel: its only VGPR spill). The caller must own the columns then (no
// query of this lane outstanding: the kernel shades only lanes whose s_pend reads 0).
struct NoSink {
    static constexpr bool lds = false;
    RT_DEV void put(const V3&, const V3&, double) const {}
};
struct LdsQuerySink {
    static constexpr bool lds = true;
    __attribute__((address_space(3))) double* o;  // this lane's origin column: [3][stride]
    __attribute__((address_space(3))) double* d;  // direction + distance: [4][stride]
    int stride;
    RT_DEV void put(const V3& org, const V3& dir, double dist) const {
        o[0] = org.x; o[stride] = org.y; o[2 * stride] = org.z;
        d[0] = dir.x; d[stride] = dir.y; d[2 * stride] = dir.z; d[3 * stride] = dist;
    }
};

// Where a path keeps the two values only a mirror bounce hands on to the next vertex (read there only
// when ps.kind == K_SPEC): `o`, the direction the reference passes on unchanged (scene.rs:178), and
// the throughput before the bounce (Le(x') weight). RegCold: PathState's registers. LdsCold: a column
// of LDS per thread (the analytic megakernel: 12 VGPRs of loop-carried state less; written only at
// mirror bounces, read only after them).
struct RegCold {
    RT_DEV V3 o(const PathState& ps) const { return ps.o; }
    RT_DEV void set_o(PathState& ps, V3 v) const { ps.o = v; }
    RT_DEV V3 bemit(const PathState& ps) const { return ps.bemit; }
    RT_DEV void set_bemit(PathState& ps, V3 v) const { ps.bemit = v; }
};
struct LdsCold {
    __attribute__((address_space(3))) double* p;  // this thread's column of [6][256]
    RT_DEV V3 o(const PathState&) const { return v3(p[0], p[256], p[512]); }
    RT_DEV void set_o(PathState&, V3 v) const { p[0] = v.x; p[256] = v.y; p[512] = v.z; }
    RT_DEV V3 bemit(const PathState&) const { return v3(p[768], p[1024], p[1280]); }
    RT_DEV void set_bemit(PathState&, V3 v) const { p[768] = v.x; p[1024] = v.y; p[1280] = v.z; }
};

// Shades the hit `hr` of ps.ray. Returns true when the path continues (ps.ray is the next ray to
// trace), false when this sample's radiance ps.L is final. The shadow ray of next-event estimation
// is traced inline.
template <class C, class Cold = RegCold, class Sink = NoSink>
RT_DEV bool shade_vertex(const DevScene& sc, const RenderArgs& a, PathState& ps,
                         const HitRec& hr, ShadowDefer* defer = nullptr, const Cold& cold = Cold(),
                         const Sink& sink = Sink()) {
    if (hr.obj < 0) return false;  // no hit: R = 0 (scene.rs:157, :175, :233)
    RT_DBG_REGION(6);
    const DevObject& obj = object_at<C>(sc, hr.obj);
    V3 x, nrm;
    RT_DBG_TSTART(t_sf);
    surface<C>(sc, ps.ray, hr, &x, &nrm);
    RT_DBG_TEND(7, t_sf);
    if (ps.kind == K_CAMERA) {
        ps.L = ld3(obj.emitted);
    } else if (!C::nospec && ps.kind == K_SPEC) {
        ps.L = ps.L + mult(cold.bemit(ps), ld3(obj.emitted));
    } else if (C::mis && hr.obj == sc.light && ps.pdf_prev > 0.0) {
        // MIS, BSDF strategy: emitted radiance with the balance-heuristic weight
        double cosl = dot(nrm, -ps.ray.d);
#if RT_OPT_NEE
        // pdf_prev / (pdf_prev + pdf_l) with pdf_l = pdfA t^2 / cosl: numerator and denominator times cosl
        // (one division; cosl == 0 gives 0 like the reference's pdf_l = inf)
        const double pc = ps.pdf_prev * cosl;
        double wgt = pc / (pc + light_pdf_area(sc) * (hr.t * hr.t));
#else
        double pdf_l = light_pdf_area(sc) * (hr.t * hr.t) / cosl;
        double wgt = ps.pdf_prev / (ps.pdf_prev + pdf_l);
#endif
        ps.L = ps.L + mult(ps.beta, ld3(obj.emitted) * wgt);
    }
    V3 o = -ps.ray.d;  // the out direction, except after a mirror bounce (which keeps the previous one)
    if (!C::nospec && ps.kind == K_SPEC) o = cold.o(ps);
    ps.depth += 1;
    const double p = ps.depth <= (uint32_t)MAX_BOUNCES ? 1.0 : SURVIVAL_PROBABILITY;
    Rng rng(ps.r0, ps.r1);
    const bool spec = !C::nospec && obj.brdf == BRDF_SPECULAR;
#if !RT_OPT_SPEC
    if (spec) {
        RT_DBG_REGION(7);
        const bool survive = rng.uniform() < p;  // scene.rs:173
        ps.r0 = rng.s0;
        ps.r1 = rng.s1;
        if (!survive) return false;
        V3 i;
        double pdf;
        brdf_sample<C>(obj, nrm, o, rng, &i, &pdf);
        V3 f = brdf_eval<C>(obj, nrm, o, i);
        cold.set_bemit(ps, ps.beta);
        cold.set_o(ps, o);
        ps.beta = mult(ps.beta, f) * dot(nrm, i) / (pdf * p);
        ps.ray = Ray{x, i};
        ps.kind = K_SPEC;
        return true;
    }
#endif
    const bool use_mis = C::mis && obj.brdf == BRDF_DIFFUSE;
    // next-event estimation (scene.rs:217-229); a mirror vertex has none (scene.rs:170-185)
    if (!spec) {
        RT_DBG_REGION(8);
        V3 y, ny;
        double pdfA;
        RT_DBG_TSTART(t_ls);
        light_sample<C>(sc, rng, &y, &ny, &pdfA);
        RT_DBG_TEND(9, t_ls);
        const V3 diff = y - x;
        const double r_sqr = dot(diff, diff);
#if RT_OPT_VIS
        // norm(y - x) and |y - x| exactly as mutually_visible computes them (scene.rs:258-262): the
        // shadow ray reuses them
        const double dist = sqrt_rn(r_sqr);  // == mag(diff)
        const V3 i = diff / dist;          // == norm(diff)
#else
        const V3 i = norm(diff);
#endif
        // Le * f: for a diffuse vertex Le_light * (kd / pi), evaluated once per object on the host
        // (mirror vertices have no NEE)
        V3 lef = (RT_OPT_LEF && (!C::phong || obj.brdf == BRDF_DIFFUSE))
                     ? ld3(obj.lef)
                     : mult(ld3(object_at<C>(sc, sc.light).emitted), brdf_eval<C>(obj, nrm, o, i));
        if (!is_zero(lef)) {  // a zero Le*f makes the term exactly 0: skip the shadow ray
            RT_DBG_REGION(9);
            double vis;
#if RT_OPT_VIS
            const Ray sr{x, i};
#else
            const double dist = mag(diff);
            const Ray sr{x, diff / dist};
#endif
            if constexpr (C::mesh && C::compact) {
                if (defer) {
                    // mutually_visible (scene.rs:258-270) split: analytic objects now, meshes deferred
                    // (the reciprocals only where used: the plane tests, f64 near tests, the deferral)
                    vis = visible_analytic<C>(sc, y, sr, dist) ? 1. : 0.;
#if RT_NEAR32
                    const RayInv ninv{};  // near_cull32 takes its own f32 reciprocals
#else
                    const RayInv ninv = make_inv(sr.d);
#endif
                    const uint32_t near = vis > 0. ? mesh_near_mask<C>(sc, sr, ninv, dist) : 0u;
                    if (near) {
                        defer->pending = true;
                        defer->meshes = near;
                        if constexpr (Sink::lds) {
                            sink.put(sr.o, sr.d, dist);
                        } else {
                            defer->inv = make_inv(sr.d);
                            defer->o = sr.o;
                            defer->d = sr.d;
                            defer->dist = dist;
                        }
                    }
                } else {
                    vis = visible_ray<C>(sc, y, sr, dist) ? 1. : 0.;
                }
            } else {
                RT_DBG_TSTART(t_vi);
                vis = visible_ray<C>(sc, y, sr, dist) ? 1. : 0.;
                RT_DBG_TEND(10, t_vi);
            }
            V3 c;
            if (!use_mis) {
#if RT_OPT_NEE
                // one scalar weight, one reciprocal (magnitude only: the same value up to the last bits)
                c = lef * (vis * dot(nrm, i) * dot(ny, -i) * rcp_any(r_sqr * pdfA));
#else
                c = lef * vis * dot(nrm, i) * dot(ny, -i) / (r_sqr * pdfA);
#endif
            } else {
                double cosl = dot(ny, -i);
                double pdf_l = pdfA * r_sqr / cosl;
                double pdf_b = dot(nrm, i) * FRAC_1_PI;
                c = v3(0, 0, 0);
#if RT_OPT_NEE
                // (pdf_l / (pdf_l + pdf_b)) / pdf_l == 1 / (pdf_l + pdf_b)
                if (vis > 0. && cosl > 0. && pdf_b > 0.) c = lef * (dot(nrm, i) * rcp_any(pdf_l + pdf_b));
#else
                if (vis > 0. && cosl > 0. && pdf_b > 0.) c = lef * dot(nrm, i) * ((pdf_l / (pdf_l + pdf_b)) / pdf_l);
#endif
            }
            if (defer && defer->pending) defer->c = mult(ps.beta, c);  // added later iff no mesh occludes
            else ps.L = ps.L + mult(ps.beta, c);
        }
    }
    // Russian roulette (scene.rs:173 / :231) + BSDF continuation (scene.rs:176-184 / :232-240): one
    // code path for mirror and diffuse vertices
#if RT_OPT_RR
    if (!rng.below53(ps.depth <= (uint32_t)MAX_BOUNCES ? kP53One : kP53Survive)) return false;  // uniform() < p
#else
    if (!(rng.uniform() < p)) return false;
#endif
    RT_DBG_REGION(10);
    V3 wi;
    double pdf;
    RT_DBG_TSTART(t_bs);
    brdf_sample<C>(obj, nrm, o, rng, &wi, &pdf);
    RT_DBG_TEND(11, t_bs);
    ps.r0 = rng.s0;
    ps.r1 = rng.s1;
    if (spec) {  // Le(x') after a mirror bounce is weighted by the beta before it; o goes on unchanged
        cold.set_bemit(ps, ps.beta);
        cold.set_o(ps, o);
    }
#if RT_OPT_BETA
    // f cos / (pdf p) with cos and pdf cancelled: diffuse f = kd / pi, pdf = cos / pi (scene.rs:41-43,
    // 56-70); mirror f = ks / cos (wi is exactly flip_across(o, n), so Specular::eval's equal_within
    // holds), pdf = 1 (scene.rs:44-55, 71-74) — both k / p. Same value up to the last bits; cos == 0
    // (the reference's 0 / 0) and Phong take the general form.
    const double cw = dot(nrm, wi);
    if ((!C::phong || obj.brdf != BRDF_PHONG) && cw != 0.0) {
        ps.beta = mult(ps.beta, ld3(obj.k)) * (ps.depth <= (uint32_t)MAX_BOUNCES ? 1.0 : kInvSurvival);
    } else {
        ps.beta = mult(ps.beta, brdf_eval<C>(obj, nrm, o, wi)) * cw / (pdf * p);
    }
#else
    V3 f = brdf_eval<C>(obj, nrm, o, wi);
    ps.beta = mult(ps.beta, f) * dot(nrm, wi) / (pdf * p);
#endif
    ps.ray = Ray{x, wi};
    ps.kind = spec ? K_SPEC : K_DIFF;
    ps.pdf_prev = use_mis ? pdf : 0.0;
    // zero throughput: every later term is exactly 0 (a mirror bounce's Le(x') still counts, with the
    // beta before it), and with a counter-based RNG no draws need to be kept in step — end the path
    // (same result, less work)
    return spec || !is_zero(ps.beta);
}

}  // namespace f64
}  // namespace rt
