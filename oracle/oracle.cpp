// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU f64 restatement of SuneelFreimuth/raytracer-server's render hot path and of the host
// scene preparation it depends on. Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / CPU baseline. The product
// (raytracer-server_amd/) never links, loads or calls anything in oracle/.
//
// Parity pins:
//   * geometry.rs:1115-1131 `test_octants` — the reference's only unit test (known answer),
//   * examples/cornell_box.png region means (statistical golden, tests/golden/),
//   * Random123 Philox4x32-10 known-answer vectors for the RNG spec below.
// The reference draws from rand::thread_rng (OS-seeded ChaCha12, rand 0.8.5 / rand_chacha
// 0.3.1), which cannot be replayed: per-sample values are therefore "parity unpinned" against
// the reference itself; the oracle and the HIP kernels share the counter-based RNG spec.
//
// Build: oracle/Makefile (-O3 -ffp-contract=off, no fast-math: every expression keeps the
// reference's evaluation order so results are IEEE-identical to a Rust f64 build except for
// libm sin/cos/pow ulps).
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace orc {

static const double PI = 3.14159265358979323846264338327950288;
static const double FRAC_1_PI = 0.318309886183790671537767526745028724;

// ---- Vec3: geometry.rs:21-134 (evaluation order kept operator by operator) ----
struct V3 {
    double x, y, z;
};
static inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline V3 operator/(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // :65
static inline V3 cross(V3 a, V3 b) {                                                  // :69
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V3 mult(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }  // :77
static inline double mag(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  // :57
static inline V3 norm(V3 a) { return a / mag(a); }                                     // :61
static inline bool equal_within(V3 a, V3 b, double e) {                                 // :85
    return std::fabs(a.x - b.x) < e && std::fabs(a.y - b.y) < e && std::fabs(a.z - b.z) < e;
}
static inline V3 flip_across(V3 a, V3 axis) { return (2.0 * dot(a, axis)) * axis - a; }  // :99
static inline double clampd(double x, double lo, double hi) {                          // :11
    if (x < lo) return lo;
    if (x > hi) return hi;
    return x;
}
static inline V3 clampv(V3 a, double lo, double hi) {
    return v3(clampd(a.x, lo, hi), clampd(a.y, lo, hi), clampd(a.z, lo, hi));
}
static inline V3 rot_x(V3 a, double ang) {  // :111
    return v3(a.x, a.y * std::cos(ang) - a.z * std::sin(ang), a.y * std::sin(ang) + a.z * std::cos(ang));
}
static inline V3 rot_y(V3 a, double ang) {  // :119
    return v3(a.x * std::cos(ang) + a.z * std::sin(ang), a.y, a.z * std::cos(ang) - a.x * std::sin(ang));
}
static inline V3 rot_z(V3 a, double ang) {  // :127
    return v3(a.x * std::cos(ang) - a.y * std::sin(ang), a.x * std::sin(ang) + a.y * std::cos(ang), a.z);
}
static inline double determinant3(V3 v0, V3 v1, V3 v2) {  // :136
    return v0.x * (v1.y * v2.z - v1.z * v2.y) - v1.x * (v0.y * v2.z - v0.z * v2.y) +
           v2.x * (v0.y * v1.z - v0.z * v1.y);
}
// Rust f64::powi (llvm.powi): binary exponentiation. Only the unused Phong BRDF reaches it.
static inline double powi(double b, int n) {
    bool neg = n < 0;
    unsigned e = neg ? (unsigned)(-(long)n) : (unsigned)n;
    double r = 1.0;
    while (e) {
        if (e & 1u) r *= b;
        b *= b;
        e >>= 1;
    }
    return neg ? 1.0 / r : r;
}

struct Ray {
    V3 pos, dir;
};
static inline V3 eval(const Ray& r, double t) { return r.pos + t * r.dir; }  // :382

struct Hit {
    double t;
    V3 pos, n;
    int id;
};

// ---- RNG spec v2 (shared with the HIP kernels) ----
// One stream per camera sample: Philox4x32-10 (Salmon et al., SC'11; Random123 constants) keyed
// by the 64-bit seed with counter (pixel, sample, 0, subpixel) seeds xoroshiro128++, whose outputs
// are consumed in the reference's own draw order along the path (thread_rng is likewise consumed
// sequentially): camera r1, r2 (server.rs:339,346); per diffuse vertex light xi1, xi2
// (geometry.rs:576-577; a mesh light draws its triangle pick first, :589), RR (scene.rs:231),
// BSDF u1, u2 (scene.rs:59,61; Phong u, xi1, xi2); per mirror vertex RR (scene.rs:173).
// uniform = (u64 >> 11) * 2^-53 (rand 0.8's f64 conversion).
static inline void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Rng {
    uint64_t s0, s1;
    Rng() : s0(1), s1(0) {}
    Rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t sub) {
        uint32_t ctr[4] = {pixel, sample, 0u, sub};
        uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
        uint32_t o[4];
        philox4x32_10(ctr, key, o);
        s0 = ((uint64_t)o[0] << 32) | o[1];
        s1 = ((uint64_t)o[2] << 32) | o[3];
        if ((s0 | s1) == 0) s0 = 1;
    }
    static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {  // xoroshiro128++ (Blackman & Vigna 2019)
        uint64_t a = s0, b = s1;
        uint64_t r = rotl(a + b, 17) + a;
        b ^= a;
        s0 = rotl(a, 49) ^ b ^ (b << 21);
        s1 = rotl(b, 28);
        return r;
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// ---- geometry.rs:916-1113 BoundingBox ----
struct BBox {
    V3 min, max;
};
static BBox enclose(const std::vector<V3>& pts) {  // :927
    V3 mn = v3(INFINITY, INFINITY, INFINITY), mx = v3(-INFINITY, -INFINITY, -INFINITY);
    for (const V3& p : pts) {
        if (p.x < mn.x) mn.x = p.x;
        if (p.x > mx.x) mx.x = p.x;
        if (p.y < mn.y) mn.y = p.y;
        if (p.y > mx.y) mx.y = p.y;
        if (p.z < mn.z) mn.z = p.z;
        if (p.z > mx.z) mx.z = p.z;
    }
    return BBox{mn, mx};
}
static inline bool contains(const BBox& b, V3 p) {  // :968
    return b.min.x <= p.x && p.x <= b.max.x && b.min.y <= p.y && p.y <= b.max.y && b.min.z <= p.z &&
           p.z <= b.max.z;
}
// :977 — first face (−x,+x,−y,+y,−z,+z) whose plane hit at t >= 1e-7 lies inside the face.
static bool box_intersect(const BBox& b, const Ray& r, double* tout) {
    const double EPS = 0.0000001;
    double t;
    V3 p;
    t = (b.min.x - r.pos.x) / r.dir.x;
    if (t >= EPS) { p = eval(r, t); if (b.min.y <= p.y && p.y <= b.max.y && b.min.z <= p.z && p.z <= b.max.z) { *tout = t; return true; } }
    t = (b.max.x - r.pos.x) / r.dir.x;
    if (t >= EPS) { p = eval(r, t); if (b.min.y <= p.y && p.y <= b.max.y && b.min.z <= p.z && p.z <= b.max.z) { *tout = t; return true; } }
    t = (b.min.y - r.pos.y) / r.dir.y;
    if (t >= EPS) { p = eval(r, t); if (b.min.x <= p.x && p.x <= b.max.x && b.min.z <= p.z && p.z <= b.max.z) { *tout = t; return true; } }
    t = (b.max.y - r.pos.y) / r.dir.y;
    if (t >= EPS) { p = eval(r, t); if (b.min.x <= p.x && p.x <= b.max.x && b.min.z <= p.z && p.z <= b.max.z) { *tout = t; return true; } }
    t = (b.min.z - r.pos.z) / r.dir.z;
    if (t >= EPS) { p = eval(r, t); if (b.min.x <= p.x && p.x <= b.max.x && b.min.y <= p.y && p.y <= b.max.y) { *tout = t; return true; } }
    t = (b.max.z - r.pos.z) / r.dir.z;
    if (t >= EPS) { p = eval(r, t); if (b.min.x <= p.x && p.x <= b.max.x && b.min.y <= p.y && p.y <= b.max.y) { *tout = t; return true; } }
    return false;
}
static inline V3 center(const BBox& b) { return (b.min + b.max) / 2.0; }  // :1063
static BBox octant(const BBox& b, int i) {                                // :1067
    V3 c = center(b);
    const V3 &mn = b.min, &mx = b.max;
    switch (i) {
        case 0: return BBox{mn, c};
        case 1: return BBox{v3(mn.x, mn.y, c.z), v3(c.x, c.y, mx.z)};
        case 2: return BBox{v3(mn.x, c.y, mn.z), v3(c.x, mx.y, c.z)};
        case 3: return BBox{v3(mn.x, c.y, c.z), v3(c.x, mx.y, mx.z)};
        case 4: return BBox{v3(c.x, mn.y, mn.z), v3(mx.x, c.y, c.z)};
        case 5: return BBox{v3(c.x, mn.y, c.z), v3(mx.x, c.y, mx.z)};
        case 6: return BBox{v3(c.x, c.y, mn.z), v3(mx.x, mx.y, c.z)};
        default: return BBox{c, mx};
    }
}

// ---- geometry.rs:598-670 Triangle ----
struct Tri {
    V3 a, b, c;
};
static inline V3 tri_normal(const Tri& t) { return norm(cross(t.c - t.a, t.b - t.a)); }  // :606
static double tri_area(const Tri& t) {                                                  // :614 Heron
    double ab = mag(t.a - t.b), bc = mag(t.b - t.c), ca = mag(t.c - t.a);
    double s = (ab + bc + ca) / 2.0;
    return std::sqrt(s * (s - ab) * (s - bc) * (s - ca));
}
static bool tri_intersect(const Tri& tr, const Ray& ray, Hit* h) {  // :637
    V3 n = tri_normal(tr);
    if (std::fabs(dot(n, ray.dir)) < 0.0001) return false;
    V3 ab = tr.b - tr.a, ac = tr.c - tr.a, b = ray.pos - tr.a;
    V3 nd = -ray.dir;
    double det = determinant3(nd, ab, ac);
    double t = determinant3(b, ab, ac) / det;
    double u = determinant3(nd, b, ac) / det;
    double v = determinant3(nd, ab, b) / det;
    if (u < 0. || u > 1. || v < 0. || u + v > 1.) return false;
    if (t > 0.0001) {
        V3 nn = dot(n, -ray.dir) >= 0. ? n : -n;
        h->t = t;
        h->pos = eval(ray, t) + 0.00001 * nn;
        h->n = nn;
        return true;
    }
    return false;
}
// :1038 / :1049
static bool seg_intersect(const BBox& b, V3 a, V3 c) {
    Ray r{a, norm(c - a)};
    double t;
    if (box_intersect(b, r, &t)) {
        if (t <= mag(c - a)) return true;
    }
    return false;
}
static bool overlaps_triangle(const BBox& b, const Tri& t) {
    if (contains(b, t.a) || contains(b, t.b) || contains(b, t.c)) return true;
    return seg_intersect(b, t.a, t.b) || seg_intersect(b, t.a, t.c) || seg_intersect(b, t.b, t.c);
}

// ---- geometry.rs:1133-1300 Octree ----
struct Node {
    bool leaf;
    int children[8];
    std::vector<int> tris;  // leaf: triangle indices, in push order
};
struct Mesh {
    std::vector<V3> vertices;
    std::vector<int> indices;
    BBox bbox;
    double surface_area;
    std::vector<double> areas;  // triangle_selector weights (computed at Mesh::new, pre-transform)
    std::vector<Node> nodes;
    BBox oct_bbox;
    bool accelerated = false;
    size_t num_triangles() const { return indices.size() / 3; }
    Tri tri(size_t i) const { return Tri{vertices[indices[3 * i]], vertices[indices[3 * i + 1]], vertices[indices[3 * i + 2]]}; }
};
static const int OCT_MAX_DEPTH = 10, OCT_SMALL_NODE = 9;  // :1146-1147
static int oct_build(const Mesh& m, BBox box, const std::vector<int>& tris, std::vector<Node>& nodes, int depth) {
    if (tris.empty()) return -1;
    if ((int)tris.size() <= OCT_SMALL_NODE || depth >= OCT_MAX_DEPTH) {
        Node n;
        n.leaf = true;
        for (int k = 0; k < 8; ++k) n.children[k] = -1;
        n.tris = tris;
        nodes.push_back(std::move(n));
        return (int)nodes.size() - 1;
    }
    BBox oct[8];
    for (int i = 0; i < 8; ++i) oct[i] = octant(box, i);
    std::vector<int> ot[8];
    for (int id : tris) {
        Tri t = m.tri(id);
        for (int i = 0; i < 8; ++i)
            if (overlaps_triangle(oct[i], t)) ot[i].push_back(id);
    }
    Node p;
    p.leaf = false;
    for (int k = 0; k < 8; ++k) p.children[k] = -1;
    nodes.push_back(p);
    int inew = (int)nodes.size() - 1;
    int ch[8];
    for (int i = 0; i < 8; ++i) ch[i] = oct_build(m, oct[i], ot[i], nodes, depth + 1);
    for (int i = 0; i < 8; ++i) nodes[inew].children[i] = ch[i];
    return inew;
}
static void accelerate(Mesh& m) {  // :835, :1149
    m.nodes.clear();
    std::vector<int> all(m.num_triangles());
    for (size_t i = 0; i < all.size(); ++i) all[i] = (int)i;
    oct_build(m, m.bbox, all, m.nodes, 1);
    m.oct_bbox = m.bbox;
    m.accelerated = true;
}
// :1245 — ordered DFS; child order from the ROOT box's octant centres; first subtree with a hit wins.
static bool oct_recurse(const Mesh& m, int ni, BBox box, const Ray& ray, Hit* h) {
    const Node& node = m.nodes[ni];
    if (!node.leaf) {
        int order[8] = {0, 1, 2, 3, 4, 5, 6, 7};
        BBox roct[8];
        for (int i = 0; i < 8; ++i) roct[i] = octant(m.oct_bbox, i);
        auto dist = [&](int o) { return mag(center(roct[o]) - ray.pos); };
        for (int i = 1; i < 8; ++i) {
            int j = i;
            while (j > 0 && dist(order[j - 1]) > dist(order[j])) {
                int tmp = order[j]; order[j] = order[j - 1]; order[j - 1] = tmp;
                --j;
            }
        }
        for (int k = 0; k < 8; ++k) {
            int i = order[k];
            BBox oc = octant(box, i);
            if (node.children[i] >= 0) {
                double t;
                if (box_intersect(oc, ray, &t)) {
                    if (oct_recurse(m, node.children[i], oc, ray, h)) return true;
                }
            }
        }
        return false;
    }
    bool any = false;
    for (int id : node.tris) {
        Hit hh;
        if (tri_intersect(m.tri(id), ray, &hh)) {
            if (!any || hh.t < h->t) { *h = hh; any = true; }
        }
    }
    return any;
}
static bool mesh_intersect(const Mesh& m, const Ray& ray, Hit* h) {  // :883
    if (m.accelerated) {
        if (m.nodes.empty()) return false;
        return oct_recurse(m, 0, m.oct_bbox, ray, h);
    }
    bool any = false;
    for (size_t i = 0; i < m.num_triangles(); ++i) {
        Hit hh;
        if (tri_intersect(m.tri(i), ray, &hh)) {
            if (!any || hh.t < h->t) { *h = hh; any = true; }
        }
    }
    return any;
}

// ---- scene.rs:10-141 objects / BRDF ----
enum { BRDF_DIFFUSE = 0, BRDF_SPECULAR = 1, BRDF_PHONG = 2 };
enum { GEOM_SPHERE = 0, GEOM_PLANE = 1, GEOM_MESH = 2 };
struct Object {
    V3 emitted;
    int brdf;
    V3 k;  // kd (diffuse) / ks (specular)
    double ph_kd, ph_ks;
    int ph_power;
    V3 color_d, color_s;
    int geom;
    V3 pos;
    double r;
    V3 n;
    int mesh;
};
struct Scene {
    Ray camera;
    std::vector<Object> objects;
    std::vector<Mesh> meshes;
    int light = -1;
};

static V3 brdf_eval(const Object& o, V3 n, V3 out, V3 in) {  // scene.rs:31
    switch (o.brdf) {
        case BRDF_DIFFUSE: return o.k * FRAC_1_PI;
        case BRDF_SPECULAR:
            if (equal_within(in, flip_across(out, n), 0.001)) return o.k / dot(n, in);
            return v3(0, 0, 0);
        default: {
            V3 refl = flip_across(in, n);
            double c = std::fmax(dot(out, refl), 0.);  // f64::max ignores NaN like fmax
            return o.color_d * o.ph_kd * FRAC_1_PI +
                   o.color_s * o.ph_ks * (double)(o.ph_power + 2) / (2. * PI) * powi(c, o.ph_power);
        }
    }
}
static void create_local_coord(V3 n, V3* u, V3* v, V3* w) {  // scene.rs:112
    *w = n;
    V3 base = std::fabs(w->x) > 0.1 ? v3(0., 1., 0.) : v3(1., 0., 0.);
    *u = norm(cross(base, *w));
    *v = cross(*w, *u);
}
static void brdf_sample(const Object& o, V3 n, V3 out, Rng& rng, V3* in, double* pdf) {  // scene.rs:56
    switch (o.brdf) {
        case BRDF_DIFFUSE: {
            double z = std::sqrt(rng.uniform());
            double r = std::sqrt(1.0 - z * z);
            double phi = 2.0 * PI * rng.uniform();
            double x = r * std::cos(phi), y = r * std::sin(phi);
            V3 u, v, w;
            create_local_coord(n, &u, &v, &w);
            V3 i = norm(u * x + v * y + w * z);
            *in = i;
            *pdf = dot(n, i) * FRAC_1_PI;
            return;
        }
        case BRDF_SPECULAR:
            *in = flip_across(out, n);
            *pdf = 1.0;
            return;
        default: {
            double p = (double)o.ph_power;
            double u = rng.uniform();
            if (u < o.ph_kd) {
                double xi1 = rng.uniform(), xi2 = rng.uniform();
                V3 i = v3(std::sqrt(1. - xi1) * std::cos(2. * PI * xi2), std::sqrt(1. - xi1) * std::sin(2. * PI * xi2), std::sqrt(xi1));
                *in = i;
                *pdf = dot(n, i) * FRAC_1_PI;
            } else if (o.ph_kd <= u && u < o.ph_kd + o.ph_ks) {
                double xi1 = rng.uniform(), xi2 = rng.uniform();
                V3 i = v3(std::sqrt(1. - std::pow(xi1, 2. / (p + 1.))) * std::cos(2. * PI * xi2),
                          std::sqrt(1. - std::pow(xi1, 2. / (p + 1.))) * std::sin(2. * PI * xi2),
                          std::pow(xi1, 1. / (p + 1.)));
                *in = i;
                *pdf = (p + 1.) / (2. * PI) * powi(i.z, o.ph_power);
            } else {
                *in = v3(0, 0, 0);
                *pdf = 1.0;
            }
            return;
        }
    }
}

static bool geom_intersect(const Scene& s, const Object& o, const Ray& ray, Hit* h) {  // geometry.rs:512
    if (o.geom == GEOM_SPHERE) {
        V3 op = o.pos - ray.pos;
        double eps = 1e-4;
        double b = dot(op, ray.dir);
        double det = b * b - dot(op, op) + o.r * o.r;
        if (det < 0.) return false;
        det = std::sqrt(det);
        double t = b - det;
        if (t > eps) {
            V3 pos = eval(ray, t);
            V3 n = norm(pos - o.pos);
            h->t = t; h->pos = pos; h->n = dot(n, -ray.dir) >= 0. ? n : -n;
            return true;
        }
        t = b + det;
        if (t > eps) {
            V3 pos = eval(ray, t);
            V3 n = norm(pos - o.pos);
            h->t = t; h->pos = pos; h->n = dot(n, -ray.dir) >= 0. ? n : -n;
            return true;
        }
        return false;
    }
    if (o.geom == GEOM_PLANE) {
        double dn = dot(ray.dir, o.n);
        if (std::fabs(dn) < 0.0001) return false;
        double t = dot(o.pos - ray.pos, o.n) / dot(ray.dir, o.n);
        if (t >= 0.) {
            V3 n = dot(o.n, -ray.dir) >= 0. ? o.n : -o.n;
            h->t = t;
            h->pos = eval(ray, t) + n * 0.00001;
            h->n = n;
            return true;
        }
        return false;
    }
    return mesh_intersect(s.meshes[o.mesh], ray, h);
}

static bool trace_ray(const Scene& s, const Ray& ray, Hit* nh) {  // scene.rs:272
    bool any = false;
    for (size_t i = 0; i < s.objects.size(); ++i) {
        Hit h;
        if (geom_intersect(s, s.objects[i], ray, &h)) {
            h.id = (int)i;
            if (!any || h.t < nh->t) { *nh = h; any = true; }
        }
    }
    return any;
}

// geometry.rs:573 Geometry::sample
static void light_sample(const Scene& s, Rng& rng, V3* y, V3* ny, double* pdf) {
    const Object& L = s.objects[s.light];
    if (L.geom == GEOM_SPHERE) {
        double xi1 = rng.uniform(), xi2 = rng.uniform();
        double z = 2. * xi1 - 1.;
        double x = std::sqrt(1.0 - z * z) * std::cos(2. * PI * xi2);
        double yy = std::sqrt(1.0 - z * z) * std::sin(2. * PI * xi2);
        V3 n = norm(v3(x, yy, z));
        *y = L.pos + n * L.r;
        *ny = n;
        *pdf = 1.0 / (4.0 * PI * L.r * L.r);
        return;
    }
    if (L.geom == GEOM_MESH) {  // :588 WeightedIndex pick + Triangle::sample (missing +a: :622-635)
        const Mesh& m = s.meshes[L.mesh];
        double total = 0;
        for (double a : m.areas) total += a;
        double u = rng.uniform() * total;
        double acc = 0;
        size_t idx = m.areas.size() - 1;
        for (size_t i = 0; i < m.areas.size(); ++i) {
            acc += m.areas[i];
            if (acc > u) { idx = i; break; }
        }
        Tri t = m.tri(idx);
        double b0 = 1. - std::sqrt(rng.uniform());
        double b1 = (1. - b0) * rng.uniform();
        V3 ab = norm(t.b - t.a), ac = norm(t.c - t.a);
        *y = ab * b0 + ac * b1;
        *ny = tri_normal(t);
        *pdf = 1. / m.surface_area;
        return;
    }
    // Plane light: geometry.rs:593 unimplemented!() — flagged at scene finalise.
    *y = v3(0, 0, 0); *ny = v3(0, 0, 1); *pdf = 1.0;
}

// Area pdf of the light (sphere: 1/(4 pi r^2), geometry.rs:585; mesh: 1/surface_area, :591).
static double light_pdf_area(const Scene& s) {
    const Object& L = s.objects[s.light];
    if (L.geom == GEOM_SPHERE) return 1.0 / (4.0 * PI * L.r * L.r);
    if (L.geom == GEOM_MESH) return 1. / s.meshes[L.mesh].surface_area;
    return 1.0;
}

static bool mutually_visible(const Scene& s, V3 x, V3 y) {  // scene.rs:258
    const double ERR_MARGIN = 0.001;
    V3 diff = y - x;
    Ray r{x, norm(diff)};
    Hit h;
    if (trace_ray(s, r, &h)) return h.t + ERR_MARGIN >= mag(diff);
    return true;
}

struct Ctx {
    const Scene* s;
    Rng rng;  // this sample's stream
    bool mis;
    uint64_t vertices, casts;
};

static const uint64_t MAX_BOUNCES = 5;         // scene.rs:109
static const double SURVIVAL_PROBABILITY = 0.9;  // scene.rs:110

// scene.rs:161 reflected_radiance (MIS branch scene.rs:188 is `if false` in the reference: the
// live estimator is NEE with area sampling, restated here). `mis` selects the build-defined
// balance-heuristic estimator, not a reference behaviour.
static V3 reflected(Ctx& c, const Hit& hit, V3 o, uint64_t depth) {
    const Scene& s = *c.s;
    c.vertices++;
    V3 x = hit.pos, n = hit.n;
    const Object& obj = s.objects[hit.id];
    double p = depth <= MAX_BOUNCES ? 1.0 : SURVIVAL_PROBABILITY;
    Rng& rng = c.rng;
    if (obj.brdf == BRDF_SPECULAR) {
        V3 rad = v3(0, 0, 0);
        if (rng.uniform() < p) {
            V3 i; double pdf;
            brdf_sample(obj, n, o, rng, &i, &pdf);
            Hit h2;
            c.casts++;
            if (trace_ray(s, Ray{x, i}, &h2)) {
                rad = s.objects[h2.id].emitted + mult(reflected(c, h2, o, depth + 1), brdf_eval(obj, n, o, i)) * dot(n, i) / (pdf * p);
            }
        }
        return rad;
    }
    V3 rad;
    const Object& L = s.objects[s.light];
    const bool use_mis = c.mis && obj.brdf == BRDF_DIFFUSE;  // MIS defined for the diffuse lobe only
    {
        V3 y, ny; double pdf;
        light_sample(s, rng, &y, &ny, &pdf);
        V3 i = norm(y - x);
        double r_sqr = dot(y - x, y - x);
        c.casts++;
        double vis = mutually_visible(s, x, y) ? 1. : 0.;
        if (!use_mis) {
            rad = mult(L.emitted, brdf_eval(obj, n, o, i)) * vis * dot(n, i) * dot(ny, -i) / (r_sqr * pdf);
        } else {
            // light strategy, balance heuristic with the BSDF pdf of direction i (solid angle)
            double cosl = dot(ny, -i);
            double pdf_l = pdf * r_sqr / cosl;      // area -> solid angle
            double pdf_b = dot(n, i) * FRAC_1_PI;   // cosine lobe (diffuse) pdf of i
            if (vis > 0. && cosl > 0. && pdf_b > 0.) {
                double w = pdf_l / (pdf_l + pdf_b);
                rad = mult(L.emitted, brdf_eval(obj, n, o, i)) * dot(n, i) * (w / pdf_l);
            } else {
                rad = v3(0, 0, 0);
            }
        }
    }
    if (rng.uniform() < p) {
        V3 i; double pdf_brdf;
        brdf_sample(obj, n, o, rng, &i, &pdf_brdf);
        Hit h2;
        c.casts++;
        if (trace_ray(s, Ray{x, i}, &h2)) {
            V3 rec = reflected(c, h2, -i, depth + 1);
            if (use_mis && h2.id == s.light) {
                // BSDF strategy hitting the light: emitted radiance weighted by the balance heuristic
                const Object& Lo = s.objects[s.light];
                double cosl = dot(h2.n, -i);
                double t2 = h2.t;
                double pdf_l = light_pdf_area(s) * (t2 * t2) / cosl;
                double w = pdf_brdf / (pdf_brdf + pdf_l);
                rec = rec + Lo.emitted * w;
            }
            rad = rad + mult(rec, brdf_eval(obj, n, o, i)) * dot(n, i) / (pdf_brdf * p);
        }
    }
    return rad;
}

static V3 received(Ctx& c, const Ray& r) {  // scene.rs:152
    Hit h;
    c.casts++;
    if (trace_ray(*c.s, r, &h)) {
        return c.s->objects[h.id].emitted + reflected(c, h, -r.dir, 1);
    }
    return v3(0, 0, 0);
}

// server.rs:320 sample_pixel; writes the 4 subpixel means (before clamp) to sub_out[12].
static V3 sample_pixel(const Scene& s, int x, int y, int width, int height, int spp, uint64_t seed,
                       uint32_t pixel_id, bool mis, double* sub_out, uint64_t* verts, uint64_t* casts) {
    double w = (double)width, h = (double)height;
    V3 cx = v3(w * 0.5135 / h, 0., 0.);
    V3 cy = norm(cross(cx, s.camera.dir)) * 0.5135;
    int num_samples = spp / 4;
    V3 pixel = v3(0, 0, 0);
    Ctx c{&s, Rng(), mis, 0, 0};
    for (int sy = 0; sy < 2; ++sy) {
        for (int sx = 0; sx < 2; ++sx) {
            V3 rad = v3(0, 0, 0);
            const uint32_t sub = (uint32_t)(sy * 2 + sx);
            for (int smp = 0; smp < num_samples; ++smp) {
                c.rng = Rng(seed, pixel_id, (uint32_t)smp, sub);
                double r1 = 2. * c.rng.uniform();
                double dx = r1 < 1. ? std::sqrt(r1) - 1. : 1. - std::sqrt(2. - r1);
                double r2 = 2. * c.rng.uniform();
                double dy = r2 < 1. ? std::sqrt(r2) - 1. : 1. - std::sqrt(2. - r2);
                V3 d = cx * ((((double)sx + 0.5 + dx) / 2. + (double)x) / w - 0.5) +
                       cy * ((((double)sy + 0.5 + dy) / 2. + (double)y) / h - 0.5) + s.camera.dir;
                rad = rad + received(c, Ray{s.camera.pos, norm(d)}) * (1. / (double)num_samples);
            }
            if (sub_out) {
                sub_out[(sy * 2 + sx) * 3 + 0] = rad.x;
                sub_out[(sy * 2 + sx) * 3 + 1] = rad.y;
                sub_out[(sy * 2 + sx) * 3 + 2] = rad.z;
            }
            pixel = pixel + clampv(rad, 0., 1.) * 0.25;
        }
    }
    if (verts) *verts += c.vertices;
    if (casts) *casts += c.casts;
    return pixel;
}

static inline uint8_t as_u8(double v) {  // Rust `f64 as u8`: saturating, NaN -> 0
    if (v != v) return 0;
    if (v <= 0.) return 0;
    if (v >= 255.) return 255;
    return (uint8_t)v;
}
static inline V3 gamma_correct(V3 v) {  // server.rs:366
    V3 c = clampv(v, 0., 1.);
    double g = 1.0 / 2.2;
    return v3(std::pow(c.x, g), std::pow(c.y, g), std::pow(c.z, g)) * 255.0 + v3(0.5, 0.5, 0.5);
}

// ---- host prep: geometry.rs:426-510 transforms, :753-913 mesh ----
static Mesh mesh_new(std::vector<V3> verts, std::vector<int> idx) {  // :754
    Mesh m;
    m.vertices = std::move(verts);
    m.indices = std::move(idx);
    m.areas.resize(m.num_triangles());
    double sum = 0;
    for (size_t i = 0; i < m.num_triangles(); ++i) {
        m.areas[i] = tri_area(m.tri(i));
        sum += m.areas[i];
    }
    m.surface_area = sum;
    m.bbox = enclose(m.vertices);
    return m;
}
static Mesh mesh_prism(V3 p, double w, double h, double d) {  // :839
    std::vector<V3> v = {v3(p.x, p.y, p.z), v3(p.x, p.y, p.z + d), v3(p.x, p.y + h, p.z), v3(p.x, p.y + h, p.z + d),
                         v3(p.x + w, p.y, p.z), v3(p.x + w, p.y, p.z + d), v3(p.x + w, p.y + h, p.z), v3(p.x + w, p.y + h, p.z + d)};
    std::vector<int> idx = {1, 3, 7, 1, 5, 7, 0, 2, 6, 0, 4, 6, 0, 1, 3, 0, 2, 3,
                            4, 5, 7, 4, 6, 7, 2, 3, 7, 2, 6, 7, 0, 1, 5, 0, 4, 5};
    return mesh_new(v, idx);
}
// Rust's `usize::from_str` (geometry.rs:698-701 parse_face): one optional leading '+', then at
// least one ASCII digit and nothing else; a value above usize::MAX is an error (PosOverflow).
static bool parse_u64(const std::string& s, uint64_t* out) {
    size_t i = (!s.empty() && s[0] == '+') ? 1 : 0;
    if (i == s.size()) return false;
    uint64_t v = 0;
    for (; i < s.size(); ++i) {
        const char ch = s[i];
        if (ch < '0' || ch > '9') return false;
        const uint64_t d = (uint64_t)(ch - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = v;
    return true;
}
static bool mesh_load(const char* path, Mesh* out, std::string* err) {  // :777
    std::ifstream f(path);
    if (!f) { *err = std::string("cannot open ") + path; return false; }
    std::vector<V3> verts;
    std::vector<int> idx;
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string cmd;
        if (!(ss >> cmd)) continue;
        if (cmd == "v" || cmd == "vn") {
            double xyz[3];
            for (int k = 0; k < 3; ++k) {
                std::string tok;
                if (!(ss >> tok)) { *err = "unexpected end of file"; return false; }
                char* end = nullptr;
                xyz[k] = std::strtod(tok.c_str(), &end);
                if (end == tok.c_str() || *end) { *err = "Ill-formed float " + tok; return false; }
            }
            if (cmd == "v") verts.push_back(v3(xyz[0], xyz[1], xyz[2]));
        } else if (cmd == "f") {
            for (int k = 0; k < 3; ++k) {
                std::string tok;
                if (!(ss >> tok)) { *err = "unexpected end of file"; return false; }
                // parse_face: split on '/', every present part must parse as usize
                size_t start = 0;
                uint64_t first = 0;
                int part = 0;
                while (part < 3) {
                    size_t sl = tok.find('/', start);
                    std::string p = tok.substr(start, sl == std::string::npos ? std::string::npos : sl - start);
                    uint64_t val;
                    if (!parse_u64(p, &val)) { *err = "Ill-formed integer " + p; return false; }
                    if (part == 0) first = val;
                    ++part;
                    if (sl == std::string::npos) break;
                    start = sl + 1;
                }
                if (first == 0) { *err = "face index 0 (usize underflow in the reference)"; return false; }
                idx.push_back((int)(first - 1));
            }
        }
    }
    for (int i : idx)
        if (i < 0 || (size_t)i >= verts.size()) { *err = "face index out of range"; return false; }
    *out = mesh_new(std::move(verts), std::move(idx));
    return true;
}

}  // namespace orc

using namespace orc;

// ============================== C ABI (ctypes) ==============================
extern "C" {

struct orc_scene_t {
    Scene s;
    std::string err;
};

orc_scene_t* orc_scene_new(const double cam_pos[3], const double cam_dir[3]) {
    orc_scene_t* sc = new orc_scene_t();
    sc->s.camera = Ray{v3(cam_pos[0], cam_pos[1], cam_pos[2]), v3(cam_dir[0], cam_dir[1], cam_dir[2])};
    return sc;
}
void orc_scene_free(orc_scene_t* sc) { delete sc; }
const char* orc_scene_error(orc_scene_t* sc) { return sc->err.c_str(); }

// brdf_kind: 0 diffuse(k=kd), 1 specular(k=ks), 2 phong(ph = {kd, ks, power}, cd, cs)
// geom_kind: 0 sphere(g = pos3, r), 1 plane(g = pos3, n3), 2 mesh(path), 3 cube(g = pos3, size), 4 prism(g = pos3, size3)
// transforms: kinds 0 translate(xyz) 1 scale(s) 2 rot_x 3 rot_y 4 rot_z; vals: 3 doubles per transform
int orc_add_object(orc_scene_t* sc, const double emitted[3], int brdf_kind, const double k[3], const double ph[3],
                   const double cd[3], const double cs[3], int geom_kind, const double g[6], const char* mesh_path,
                   int n_tf, const int* tf_kind, const double* tf_val) {
    Object o{};
    o.emitted = v3(emitted[0], emitted[1], emitted[2]);
    o.brdf = brdf_kind;
    o.k = v3(k[0], k[1], k[2]);
    o.ph_kd = ph[0]; o.ph_ks = ph[1]; o.ph_power = (int)ph[2];
    o.color_d = v3(cd[0], cd[1], cd[2]);
    o.color_s = v3(cs[0], cs[1], cs[2]);
    o.mesh = -1;
    Mesh m;
    bool is_mesh = false;
    switch (geom_kind) {
        case 0: o.geom = GEOM_SPHERE; o.pos = v3(g[0], g[1], g[2]); o.r = g[3]; break;
        case 1: o.geom = GEOM_PLANE; o.pos = v3(g[0], g[1], g[2]); o.n = v3(g[3], g[4], g[5]); break;
        case 2: {
            std::string err;
            if (!mesh_load(mesh_path, &m, &err)) { sc->err = err; return -1; }
            is_mesh = true;
            break;
        }
        case 3: m = mesh_prism(v3(g[0], g[1], g[2]), g[3], g[3], g[3]); is_mesh = true; break;
        case 4: m = mesh_prism(v3(g[0], g[1], g[2]), g[3], g[4], g[5]); is_mesh = true; break;
        default: sc->err = "bad geometry kind"; return -1;
    }
    if (is_mesh) o.geom = GEOM_MESH;
    for (int t = 0; t < n_tf; ++t) {  // scene.rs:411-429, geometry.rs:427-510
        const double* v = tf_val + 3 * t;
        switch (tf_kind[t]) {
            case 0: {
                V3 tr = v3(v[0], v[1], v[2]);
                if (o.geom == GEOM_SPHERE || o.geom == GEOM_PLANE) o.pos = o.pos + tr;
                else {
                    for (V3& p : m.vertices) p = p + tr;
                    m.bbox.min = m.bbox.min + tr;
                    m.bbox.max = m.bbox.max + tr;
                }
                break;
            }
            case 1: {
                double s = v[0];
                if (o.geom == GEOM_SPHERE) o.r *= s;
                else if (o.geom == GEOM_MESH) {
                    V3 c = center(m.bbox);
                    for (V3& p : m.vertices) p = c + (p - c) * s;
                    m.bbox.min = m.bbox.min + (m.bbox.min - c) * s;  // :503 (quirk kept)
                    m.bbox.max = m.bbox.max + (m.bbox.max - c) * s;
                }
                break;
            }
            case 2: case 3: case 4: {
                double a = v[0];
                int kk = tf_kind[t];
                if (o.geom == GEOM_PLANE) o.n = kk == 2 ? rot_x(o.n, a) : kk == 3 ? rot_y(o.n, a) : rot_z(o.n, a);
                else if (o.geom == GEOM_MESH) {
                    V3 c = center(m.bbox);
                    for (V3& p : m.vertices) p = c + (kk == 2 ? rot_x(p - c, a) : kk == 3 ? rot_y(p - c, a) : rot_z(p - c, a));
                    m.bbox = enclose(m.vertices);
                }
                break;
            }
            default: sc->err = "bad transform kind"; return -1;
        }
    }
    if (o.geom == GEOM_MESH) {
        accelerate(m);
        o.mesh = (int)sc->s.meshes.size();
        sc->s.meshes.push_back(std::move(m));
    }
    sc->s.objects.push_back(o);
    return (int)sc->s.objects.size() - 1;
}

// scene.rs:126-141: light = first object whose emission is not within 1e-5 of zero.
int orc_scene_finalize(orc_scene_t* sc) {
    sc->s.light = -1;
    for (size_t i = 0; i < sc->s.objects.size(); ++i) {
        if (!equal_within(sc->s.objects[i].emitted, v3(0, 0, 0), 0.00001)) { sc->s.light = (int)i; break; }
    }
    if (sc->s.light < 0) { sc->err = "scene has no emitting object (scene.rs:136 unreachable!)"; return -1; }
    if (sc->s.objects[sc->s.light].geom == GEOM_PLANE) { sc->err = "plane light (geometry.rs:593 unimplemented!)"; return -1; }
    return sc->s.light;
}

// Mesh::intersect without the octree (geometry.rs:886-903, `octree: None`: brute-force nearest
// triangle, strict <) for every mesh of the scene when accel == 0; the octree walk again when 1.
void orc_scene_set_mesh_accel(orc_scene_t* sc, int accel) {
    for (Mesh& m : sc->s.meshes) m.accelerated = accel != 0;
}

// Octree shape: out[0]=nodes, out[1]=parents, out[2]=leaves, out[3]=tri refs, out[4]=max leaf size, out[5]=max leaf depth
int orc_mesh_stats(orc_scene_t* sc, int obj, int64_t out[6], double bbox[6], double* surface_area, int64_t* ntris, int64_t* nverts) {
    const Object& o = sc->s.objects[obj];
    if (o.geom != GEOM_MESH) return -1;
    const Mesh& m = sc->s.meshes[o.mesh];
    int64_t parents = 0, leaves = 0, refs = 0, maxleaf = 0, maxdepth = 0;
    std::vector<int> depth(m.nodes.size(), 0);
    if (!m.nodes.empty()) depth[0] = 1;
    for (size_t i = 0; i < m.nodes.size(); ++i) {
        const Node& n = m.nodes[i];
        if (n.leaf) {
            leaves++;
            refs += (int64_t)n.tris.size();
            if ((int64_t)n.tris.size() > maxleaf) maxleaf = (int64_t)n.tris.size();
            if (depth[i] > maxdepth) maxdepth = depth[i];
        } else {
            parents++;
            for (int c : n.children) if (c >= 0) depth[c] = depth[i] + 1;
        }
    }
    out[0] = (int64_t)m.nodes.size(); out[1] = parents; out[2] = leaves; out[3] = refs; out[4] = maxleaf; out[5] = maxdepth;
    bbox[0] = m.bbox.min.x; bbox[1] = m.bbox.min.y; bbox[2] = m.bbox.min.z;
    bbox[3] = m.bbox.max.x; bbox[4] = m.bbox.max.y; bbox[5] = m.bbox.max.z;
    *surface_area = m.surface_area;
    *ntris = (int64_t)m.num_triangles();
    *nverts = (int64_t)m.vertices.size();
    return 0;
}

// Dump octree in DFS pre-order: node_kind[i] (0 parent, 1 leaf), child[8*i], leaf_off/leaf_cnt, refs.
int64_t orc_mesh_octree(orc_scene_t* sc, int obj, int32_t* kind, int32_t* child, int32_t* leaf_off, int32_t* leaf_cnt, int32_t* refs) {
    const Object& o = sc->s.objects[obj];
    if (o.geom != GEOM_MESH) return -1;
    const Mesh& m = sc->s.meshes[o.mesh];
    int64_t r = 0;
    for (size_t i = 0; i < m.nodes.size(); ++i) {
        const Node& n = m.nodes[i];
        if (kind) kind[i] = n.leaf ? 1 : 0;
        for (int k = 0; k < 8; ++k) if (child) child[8 * i + k] = n.children[k];
        if (leaf_off) leaf_off[i] = n.leaf ? (int32_t)r : -1;
        if (leaf_cnt) leaf_cnt[i] = n.leaf ? (int32_t)n.tris.size() : 0;
        if (n.leaf) for (int t : n.tris) { if (refs) refs[r] = t; ++r; }
    }
    return r;
}

int orc_mesh_vertices(orc_scene_t* sc, int obj, double* verts, int32_t* idx) {
    const Object& o = sc->s.objects[obj];
    if (o.geom != GEOM_MESH) return -1;
    const Mesh& m = sc->s.meshes[o.mesh];
    for (size_t i = 0; i < m.vertices.size(); ++i) { verts[3*i] = m.vertices[i].x; verts[3*i+1] = m.vertices[i].y; verts[3*i+2] = m.vertices[i].z; }
    for (size_t i = 0; i < m.indices.size(); ++i) idx[i] = m.indices[i];
    return 0;
}

// geometry.rs:1115 test_octants (known answer): returns the 8 octants of box (min,max) as 48 doubles.
void orc_octants(const double mn[3], const double mx[3], double out[48]) {
    BBox b{v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2])};
    for (int i = 0; i < 8; ++i) {
        BBox o = octant(b, i);
        double* p = out + 6 * i;
        p[0] = o.min.x; p[1] = o.min.y; p[2] = o.min.z; p[3] = o.max.x; p[4] = o.max.y; p[5] = o.max.z;
    }
}

void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { philox4x32_10(ctr, key, out); }
void orc_draws(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t sub, int n, double* out) {
    Rng r(seed, pixel, sample, sub);
    for (int k = 0; k < n; ++k) out[k] = r.uniform();
}

// Scene::trace_ray for a batch of rays: t, object id (-1 miss), hit pos[3], n[3].
void orc_trace(orc_scene_t* sc, int64_t n, const double* o, const double* d, double* t, int32_t* id, double* pos, double* nrm) {
    for (int64_t i = 0; i < n; ++i) {
        Ray r{v3(o[3*i], o[3*i+1], o[3*i+2]), v3(d[3*i], d[3*i+1], d[3*i+2])};
        Hit h;
        if (trace_ray(sc->s, r, &h)) {
            t[i] = h.t; id[i] = h.id;
            if (pos) { pos[3*i] = h.pos.x; pos[3*i+1] = h.pos.y; pos[3*i+2] = h.pos.z; }
            if (nrm) { nrm[3*i] = h.n.x; nrm[3*i+1] = h.n.y; nrm[3*i+2] = h.n.z; }
        } else {
            t[i] = 0; id[i] = -1;
        }
    }
}

// RenderJob::run (server.rs:157-199) over a tile of screen rows [y0, y0+th) x [x0, x0+tw):
// the pixel at screen row `row` is sample_pixel(x, height-row-1, ...). Pixel id for the RNG is
// row*width + x (global, so output is independent of tiling). rgb: th*tw*3 (row-major, top row
// first); sub: th*tw*12 subpixel means (may be NULL). Returns vertices traced (path vertices).
int64_t orc_render(orc_scene_t* sc, int width, int height, int x0, int y0, int tw, int th, int spp, uint64_t seed,
                   int mis, int nthreads, uint8_t* rgb, double* sub, int64_t* casts_out) {
    std::atomic<int> next_row{0};
    std::atomic<int64_t> verts{0}, casts{0};
    auto worker = [&]() {
        uint64_t v = 0, c = 0;
        for (;;) {
            int r = next_row.fetch_add(1);
            if (r >= th) break;
            int row = y0 + r;
            for (int i = 0; i < tw; ++i) {
                int x = x0 + i;
                uint32_t pid = (uint32_t)row * (uint32_t)width + (uint32_t)x;
                double* so = sub ? sub + ((size_t)r * tw + i) * 12 : nullptr;
                V3 px = sample_pixel(sc->s, x, height - row - 1, width, height, spp, seed, pid, mis != 0, so, &v, &c);
                V3 g = gamma_correct(px);
                uint8_t* o = rgb + ((size_t)r * tw + i) * 3;
                o[0] = as_u8(g.x); o[1] = as_u8(g.y); o[2] = as_u8(g.z);
            }
        }
        verts += (int64_t)v;
        casts += (int64_t)c;
    };
    if (nthreads <= 1) worker();
    else {
        std::vector<std::thread> ts;
        for (int t = 0; t < nthreads; ++t) ts.emplace_back(worker);
        for (auto& t : ts) t.join();
    }
    if (casts_out) *casts_out = casts.load();
    return verts.load();
}

}  // extern "C"
