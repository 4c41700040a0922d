// Design probe (CPU, test infrastructure): how much octree-walk work in the unicorn scene could be
// skipped without changing a single result, and how often a single-precision octant classification
// would be ambiguous. Builds the flying_unicorn scene with the oracle's own code (oracle/oracle.cpp,
// included here: this is a diagnostic, never product code), generates mesh queries shaped like a
// render's (camera rays, cosine bounces from the first hits, shadow rays to the light), and walks
// each with the reference's traversal (geometry.rs:1245-1295) three ways:
//   base   — the reference walk, counting octant box tests, descents, leaf openings, triangle tests;
//   tight  — the same walk, but a child is skipped when the ray (t >= 0) passes farther than a pad
//            from the bounding box of every triangle in the child's subtree (no triangle there can
//            return tri_intersect == true, so the reference's walk would find nothing in it);
//   f32    — per octant test, whether a slab test in f32 with a relative margin could decide
//            box_intersect without the exact f64 face tests.
// Asserts that `tight` returns the same (hit, triangle, t bits) as `base` on every query.
// g++ -O3 -std=c++17 -ffp-contract=off -o /tmp/wcp tools/walk_cull_probe.cpp && /tmp/wcp [N]
#include "../oracle/oracle.cpp"

#include <cstdio>
#include <cstring>

namespace {

struct Counts {
    long box_tests = 0, descents = 0, leaves = 0, tris = 0, queries = 0, hits = 0;
    long f32_amb = 0, f32_tests = 0, culled = 0, visits = 0, dead_visits = 0, survivors = 0, tri_culled = 0;
};

struct Tight {
    std::vector<BBox> box;  // per node: union of its subtree's triangle bounds, padded
    bool after = false;     // test only children whose octant box the ray hits
    int qbits = 0;          // > 0: boxes quantized to qbits per coordinate over the parent box +- its extent
    const BBox* qref = nullptr;  // quantise against this box (the mesh's) instead of the parent's
    bool tri_cull = false;       // also skip a leaf triangle whose own (quantized) bounds the ray passes far from
};
// conservative quantization of child box c inside parent box b's range [b.min - e, b.max + e]
BBox quant(const BBox& c, const BBox& b, int bits) {
    const double top = (double)((1 << bits) - 1);
    auto q = [&](double v, double lo, double hi, bool up) {
        const double e = hi - lo, base = lo - e, step = 3 * e / top;
        double k = (v - base) / step;
        if (!up) { k = std::floor(k) - 1; if (k <= 0) return (double)-INFINITY; return base + k * step; }
        k = std::ceil(k) + 1;
        if (k >= top) return (double)INFINITY;
        return base + k * step;
    };
    return BBox{v3(q(c.min.x, b.min.x, b.max.x, false), q(c.min.y, b.min.y, b.max.y, false), q(c.min.z, b.min.z, b.max.z, false)),
                v3(q(c.max.x, b.min.x, b.max.x, true), q(c.max.y, b.min.y, b.max.y, true), q(c.max.z, b.min.z, b.max.z, true))};
}

BBox tight_of(const Mesh& m, int ni, Tight& T) {
    const Node& n = m.nodes[ni];
    BBox b{v3(INFINITY, INFINITY, INFINITY), v3(-INFINITY, -INFINITY, -INFINITY)};
    auto grow = [&](V3 p) {
        b.min = v3(std::fmin(b.min.x, p.x), std::fmin(b.min.y, p.y), std::fmin(b.min.z, p.z));
        b.max = v3(std::fmax(b.max.x, p.x), std::fmax(b.max.y, p.y), std::fmax(b.max.z, p.z));
    };
    if (n.leaf) {
        for (int id : n.tris) {
            Tri t = m.tri(id);
            grow(t.a); grow(t.b); grow(t.c);
        }
    } else {
        for (int k = 0; k < 8; ++k)
            if (n.children[k] >= 0) {
                BBox c = tight_of(m, n.children[k], T);
                grow(c.min); grow(c.max);
            }
    }
    T.box[ni] = b;
    return b;
}

// conservative: false only if the ray (t >= 0) passes farther than pad from the box
bool near(const BBox& b, const Ray& r, double pad) {
    double t0 = 0, t1 = INFINITY;
    const double o[3] = {r.pos.x, r.pos.y, r.pos.z}, d[3] = {r.dir.x, r.dir.y, r.dir.z};
    const double lo[3] = {b.min.x - pad, b.min.y - pad, b.min.z - pad}, hi[3] = {b.max.x + pad, b.max.y + pad, b.max.z + pad};
    for (int k = 0; k < 3; ++k) {
        if (std::fabs(d[k]) < 1e-300) {
            if (o[k] < lo[k] || o[k] > hi[k]) return false;
            continue;
        }
        double ta = (lo[k] - o[k]) / d[k], tb = (hi[k] - o[k]) / d[k];
        double tn = std::fmin(ta, tb), tf = std::fmax(ta, tb);
        t0 = std::fmax(t0, tn - 1e-9 * std::fabs(tn));
        t1 = std::fmin(t1, tf + 1e-9 * std::fabs(tf));
    }
    return t0 <= t1;
}

// f32 slab classification of box_intersect: 1 hit, 0 miss, -1 ambiguous (relative margin eps of the
// box's extent in t).
int f32_class(const BBox& b, const Ray& r, float eps) {
    const float o[3] = {(float)r.pos.x, (float)r.pos.y, (float)r.pos.z};
    const float d[3] = {(float)r.dir.x, (float)r.dir.y, (float)r.dir.z};
    const float lo[3] = {(float)b.min.x, (float)b.min.y, (float)b.min.z};
    const float hi[3] = {(float)b.max.x, (float)b.max.y, (float)b.max.z};
    float t0 = -INFINITY, t1 = INFINITY;
    float ext = 0;
    for (int k = 0; k < 3; ++k) ext = std::fmax(ext, hi[k] - lo[k]);
    for (int k = 0; k < 3; ++k) {
        const float inv = 1.0f / d[k];
        float ta = (lo[k] - o[k]) * inv, tb = (hi[k] - o[k]) * inv;
        t0 = std::fmax(t0, std::fmin(ta, tb));
        t1 = std::fmin(t1, std::fmax(ta, tb));
    }
    const float m = eps * ext;  // |d| = 1: t is a distance
    if (t1 < 1e-7f - m || t0 > t1 + m) return 0;
    if (t1 > 1e-7f + m && t0 < t1 - m) return 1;
    return -1;
}

bool walk(const Mesh& m, int ni, BBox box, const Ray& ray, Hit* h, int* tri, Counts& c, const Tight* T, double pad,
          const BBox* rocts) {
    const Node& node = m.nodes[ni];
    if (!node.leaf) {
        ++c.visits;
        int surv = 0;
        int order[8] = {0, 1, 2, 3, 4, 5, 6, 7};
        auto dist = [&](int o) { return mag(center(rocts[o]) - ray.pos); };
        for (int i = 1; i < 8; ++i) {
            int j = i;
            while (j > 0 && dist(order[j - 1]) > dist(order[j])) {
                std::swap(order[j], order[j - 1]);
                --j;
            }
        }
        for (int k = 0; k < 8; ++k) {
            int i = order[k];
            if (node.children[i] < 0) continue;
            BBox oc = octant(box, i);
            auto tcull = [&]() {
                if (!T) return false;
                const BBox tb = T->qbits ? quant(T->box[node.children[i]], T->qref ? *T->qref : box, T->qbits) : T->box[node.children[i]];
                return !near(tb, ray, pad);
            };
            if (T && !T->after && tcull()) {
                ++c.culled;
                continue;
            }
            ++c.box_tests;
            double t;
            const bool bh = box_intersect(oc, ray, &t);
            if (bh && T && T->after && tcull()) {
                ++c.culled;
                continue;
            }
            if (bh) ++surv, ++c.survivors;
            if (!T) {
                ++c.f32_tests;
                const int cl = f32_class(oc, ray, 1e-5f);
                if (cl < 0) ++c.f32_amb;
                else if ((cl == 1) != bh) { std::fprintf(stderr, "f32 classification WRONG\n"); std::exit(2); }
            }
            if (bh) {
                if (!m.nodes[node.children[i]].leaf) ++c.descents;
                if (walk(m, node.children[i], oc, ray, h, tri, c, T, pad, rocts)) return true;
            }
        }
        if (!surv) ++c.dead_visits;
        return false;
    }
    ++c.leaves;
    bool any = false;
    for (int id : node.tris) {
        Hit hh;
        if (T && T->tri_cull) {
            const Tri t = m.tri(id);
            BBox tb{v3(std::fmin(std::fmin(t.a.x, t.b.x), t.c.x), std::fmin(std::fmin(t.a.y, t.b.y), t.c.y),
                       std::fmin(std::fmin(t.a.z, t.b.z), t.c.z)),
                    v3(std::fmax(std::fmax(t.a.x, t.b.x), t.c.x), std::fmax(std::fmax(t.a.y, t.b.y), t.c.y),
                       std::fmax(std::fmax(t.a.z, t.b.z), t.c.z))};
            if (T->qbits) tb = quant(tb, T->qref ? *T->qref : box, T->qbits);
            if (!near(tb, ray, pad)) {
                ++c.tri_culled;
                continue;
            }
        }
        ++c.tris;
        if (tri_intersect(m.tri(id), ray, &hh)) {
            if (!any || hh.t < h->t) { *h = hh; *tri = id; any = true; }
        }
    }
    return any;
}

}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 200000;
    double cp[3] = {50.0, 52.0, 295.6}, cd[3] = {0.0, -0.042612, -1.0};
    orc_scene_t* sc = orc_scene_new(cp, cd);
    double z3[3] = {0, 0, 0}, one3[3] = {0.75, 0.75, 0.75};
    auto plane = [&](double px, double py, double pz, double nx, double ny, double nz) {
        double g[6] = {px, py, pz, nx, ny, nz};
        orc_add_object(sc, z3, 0, one3, z3, z3, z3, 1, g, nullptr, 0, nullptr, nullptr);
    };
    plane(1, 0, 0, -1, 0, 0); plane(99, 0, 0, -1, 0, 0); plane(0, 0, 0, 0, 0, -1);
    plane(0, 0, 0, 0, 1, 0); plane(0, 81.6, 0, 0, -1, 0); plane(99, 0, 0, -1, 0, 0);
    {
        int kinds[4] = {1, 0, 4, 2};
        double vals[12] = {5.0, 0, 0, 35.0, 25.0, 65.0, -0.4, 0, 0, -1.5707963267948966, 0, 0};
        double g[6] = {0};
        if (orc_add_object(sc, z3, 0, one3, z3, z3, z3, 2, g, "scenes/assets/flying-unicorn.obj", 4, kinds, vals) < 0) {
            std::fprintf(stderr, "%s\n", orc_scene_error(sc));
            return 1;
        }
    }
    { double g[6] = {73.0, 16.5, 68.0, 16.5}; orc_add_object(sc, z3, 1, one3, z3, z3, z3, 0, g, nullptr, 0, nullptr, nullptr); }
    { double e[3] = {50, 50, 50}, g[6] = {50.0, 70.0, 100.0, 4.0}; orc_add_object(sc, e, 0, z3, z3, z3, z3, 0, g, nullptr, 0, nullptr, nullptr); }
    orc_scene_finalize(sc);
    const Scene& S = sc->s;
    const Mesh& M = S.meshes[0];
    Tight T;
    T.box.resize(M.nodes.size());
    tight_of(M, 0, T);
    double scale = 1;
    for (double v : {M.oct_bbox.min.x, M.oct_bbox.min.y, M.oct_bbox.min.z, M.oct_bbox.max.x, M.oct_bbox.max.y, M.oct_bbox.max.z})
        scale = std::fmax(scale, std::fabs(v));
    const double pad = 1e-7 * scale;
    BBox rocts[8];
    for (int i = 0; i < 8; ++i) rocts[i] = octant(M.oct_bbox, i);
    Rng rng(12345, 678, 9, 1);
    // queries: camera rays, their first-hit cosine bounces, shadow rays to the light
    std::vector<Ray> Q;
    const int W = 1920, H = 1080;
    V3 cx = v3(W * .5135 / H, 0, 0), cy = norm(cross(cx, S.camera.dir)) * .5135;
    const V3 L = S.objects[S.light].pos;
    while ((int)Q.size() < N) {
        double px = rng.uniform() * W, py = rng.uniform() * H;
        Ray r{S.camera.pos, norm(cx * (px / W - .5) + cy * (py / H - .5) + S.camera.dir)};
        Q.push_back(r);
        Hit h;
        if (!trace_ray(S, r, &h)) continue;
        V3 n = h.n;
        V3 u, v, w;
        create_local_coord(n, &u, &v, &w);
        double r1 = 2 * PI * rng.uniform(), r2 = rng.uniform(), r2s = std::sqrt(r2);
        V3 d = norm(u * (std::cos(r1) * r2s) + v * (std::sin(r1) * r2s) + w * std::sqrt(1 - r2));
        Q.push_back(Ray{h.pos, d});
        double zz = 2 * rng.uniform() - 1, ph = 2 * PI * rng.uniform();
        V3 y = L + norm(v3(std::sqrt(1 - zz * zz) * std::cos(ph), std::sqrt(1 - zz * zz) * std::sin(ph), zz)) * 4.0;
        Q.push_back(Ray{h.pos, norm(y - h.pos)});
    }
    Tight T2 = T, T3 = T, T4 = T, T5 = T;
    T5.after = true; T5.qbits = 16; T5.qref = &M.bbox; T5.tri_cull = true;
    T2.after = true;
    T3.after = true; T3.qbits = 8;
    T4.after = true; T4.qbits = 16; T4.qref = &M.bbox;
    Counts base, tight, after, q8, q16, q16t;
    long past = 0, root_dead = 0, miss_walks = 0;
    for (const Ray& r : Q) {
        if (!near(M.bbox, r, pad) && !near(M.oct_bbox, r, pad)) continue;
        ++past;
        Hit h1, h2;
        int t1 = -1, t2 = -1;
        const bool a = walk(M, 0, M.oct_bbox, r, &h1, &t1, base, nullptr, pad, rocts);
        const bool b = walk(M, 0, M.oct_bbox, r, &h2, &t2, tight, &T, pad, rocts);
        Hit h3; int t3 = -1;
        walk(M, 0, M.oct_bbox, r, &h3, &t3, after, &T2, pad, rocts);
        walk(M, 0, M.oct_bbox, r, &h3, &t3, q8, &T3, pad, rocts);
        walk(M, 0, M.oct_bbox, r, &h3, &t3, q16, &T4, pad, rocts);
        {
            Hit h5; int t5 = -1;
            const bool e = walk(M, 0, M.oct_bbox, r, &h5, &t5, q16t, &T5, pad, rocts);
            if (e != a || (a && (t5 != t1 || std::memcmp(&h1.t, &h5.t, 8) != 0))) {
                std::fprintf(stderr, "MISMATCH: triangle-bounds culling changed a result\n");
                return 2;
            }
        }
        {  // would a pre-test of the root children's subtree bounds have rejected this walk?
            bool any = false;
            for (int k = 0; k < 8; ++k) {
                const int ch = M.nodes[0].children[k];
                if (ch >= 0 && near(T.box[ch], r, pad)) any = true;
            }
            root_dead += !any;
            miss_walks += !a;
            if (!any && a) { std::fprintf(stderr, "root pre-test rejected a hit\n"); return 2; }
        }
        base.hits += a;
        tight.hits += b;
        if (a != b || (a && (t1 != t2 || std::memcmp(&h1.t, &h2.t, 8) != 0))) {
            std::fprintf(stderr, "MISMATCH: tight culling changed a result\n");
            return 2;
        }
    }
    auto pr = [&](const char* k, const Counts& c) {
        std::printf("%-6s per walk: parent visits %.2f (no survivor %.2f, survivors %.2f), octant box tests %.2f, descents %.2f, leaves %.2f, triangle tests %.2f, culled children %.2f; hit rate %.3f\n",
                    k, (double)c.visits / past, (double)c.dead_visits / past, (double)c.survivors / past, (double)c.box_tests / past,
                    (double)c.descents / past, (double)c.leaves / past, (double)c.tris / past, (double)c.culled / past, (double)c.hits / past);
    };
    std::printf("%zu queries, %ld walk the octree (nodes %zu)\n", Q.size(), past, M.nodes.size());
    pr("base", base);
    pr("tight", tight);
    std::printf("walks rejected by the 8 root children's subtree bounds: %.3f (misses %.3f)\n", (double)root_dead / past,
                (double)miss_walks / past);
    pr("after", after);
    pr("q8", q8);
    pr("q16 mesh", q16);
    pr("q16+tri", q16t);
    std::printf("q16+tri: triangle tests culled by the triangle's own bounds %.2f per walk (of %.2f)\n",
                (double)q16t.tri_culled / past, (double)(q16t.tri_culled + q16t.tris) / past);
    std::printf("f32 octant classification (margin 1e-5 of the box extent): %ld tests, %.4f ambiguous\n", base.f32_tests,
                (double)base.f32_amb / std::max(1L, base.f32_tests));
    return 0;
}
