// Host scene preparation (see scene_host.hpp for the reference map). Build with -ffp-contract=off.
#include "scene_host.hpp"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "toml_lite.hpp"

namespace rt::host {
namespace {

// ---- f64 vector helpers, same operation order as geometry.rs:28-134 ----
inline D3 add(D3 a, D3 b) { return D3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline D3 sub(D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline D3 scale(D3 a, double s) { return D3{a.x * s, a.y * s, a.z * s}; }
inline D3 divs(D3 a, double s) { return D3{a.x / s, a.y / s, a.z / s}; }
inline double dotp(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline D3 crossp(D3 a, D3 b) { return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double magn(D3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
inline D3 normd(D3 a) { return divs(a, magn(a)); }
inline D3 rotx(D3 a, double t) { return D3{a.x, a.y * std::cos(t) - a.z * std::sin(t), a.y * std::sin(t) + a.z * std::cos(t)}; }
inline D3 roty(D3 a, double t) { return D3{a.x * std::cos(t) + a.z * std::sin(t), a.y, a.z * std::cos(t) - a.x * std::sin(t)}; }
inline D3 rotz(D3 a, double t) { return D3{a.x * std::cos(t) - a.y * std::sin(t), a.x * std::sin(t) + a.y * std::cos(t), a.z}; }
inline D3 centre(const Box& b) { return divs(add(b.min, b.max), 2.0); }

Box enclose(const std::vector<D3>& pts) {  // geometry.rs:927
    Box b{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
    for (const D3& p : pts) {
        if (p.x < b.min.x) b.min.x = p.x;
        if (p.x > b.max.x) b.max.x = p.x;
        if (p.y < b.min.y) b.min.y = p.y;
        if (p.y > b.max.y) b.max.y = p.y;
        if (p.z < b.min.z) b.min.z = p.z;
        if (p.z > b.max.z) b.max.z = p.z;
    }
    return b;
}

Box octant_of(const Box& b, int i) {  // geometry.rs:1067-1099 (bit2 = x, bit1 = y, bit0 = z upper half)
    D3 c = centre(b);
    D3 lo{(i & 4) ? c.x : b.min.x, (i & 2) ? c.y : b.min.y, (i & 1) ? c.z : b.min.z};
    D3 hi{(i & 4) ? b.max.x : c.x, (i & 2) ? b.max.y : c.y, (i & 1) ? b.max.z : c.z};
    return Box{lo, hi};
}

// BoundingBox::intersect (geometry.rs:977-1036): the first face, in the order -x,+x,-y,+y,-z,+z,
// whose plane is crossed at t >= 1e-7 inside the face rectangle.
bool face_hit(const Box& b, D3 o, D3 d, double* tout) {
    const double EPS = 0.0000001;
    const double lo[3] = {b.min.x, b.min.y, b.min.z}, hi[3] = {b.max.x, b.max.y, b.max.z};
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    for (int axis = 0; axis < 3; ++axis) {
        for (int side = 0; side < 2; ++side) {
            double t = ((side ? hi[axis] : lo[axis]) - oo[axis]) / dd[axis];
            if (!(t >= EPS)) continue;
            // Ray::eval: pos + t * dir
            double p[3] = {oo[0] + t * dd[0], oo[1] + t * dd[1], oo[2] + t * dd[2]};
            int u = axis == 0 ? 1 : 0, v = axis == 2 ? 1 : 2;
            if (lo[u] <= p[u] && p[u] <= hi[u] && lo[v] <= p[v] && p[v] <= hi[v]) {
                *tout = t;
                return true;
            }
        }
    }
    return false;
}

inline bool inside(const Box& b, D3 p) {
    return b.min.x <= p.x && p.x <= b.max.x && b.min.y <= p.y && p.y <= b.max.y && b.min.z <= p.z && p.z <= b.max.z;
}

bool segment_hits(const Box& b, D3 a, D3 c) {  // intersect_line_segment (geometry.rs:1038)
    D3 dir = normd(sub(c, a));
    double t;
    if (face_hit(b, a, dir, &t)) return t <= magn(sub(c, a));
    return false;
}

struct TriV {
    D3 a, b, c;
};

bool overlaps(const Box& b, const TriV& t) {  // geometry.rs:1049
    if (inside(b, t.a) || inside(b, t.b) || inside(b, t.c)) return true;
    return segment_hits(b, t.a, t.b) || segment_hits(b, t.a, t.c) || segment_hits(b, t.b, t.c);
}

constexpr int kMaxDepth = 10;   // Octree::MAX_DEPTH
constexpr int kSmallNode = 9;   // Octree::SMALL_NODE

struct Builder {
    const std::vector<TriV>& tris;
    Octree& oc;

    int32_t new_node(int32_t kind, const Box& box, int32_t parent, int32_t slot) {
        oc.kind.push_back(kind);
        for (int k = 0; k < 8; ++k) oc.child.push_back(-1);
        oc.leaf_off.push_back(-1);
        oc.leaf_cnt.push_back(0);
        oc.parent.push_back(parent);
        oc.slot.push_back(slot);
        oc.box.push_back(box);
        return (int32_t)oc.kind.size() - 1;
    }

    // Octree::_build: empty -> no node; <= SMALL_NODE triangles or depth >= MAX_DEPTH -> leaf;
    // else a parent node is pushed BEFORE its children (pre-order), children built in octant order.
    int32_t build(const Box& box, std::vector<int32_t>&& ids, int depth, int32_t parent, int32_t slot) {
        if (ids.empty()) return -1;
        if ((int)ids.size() <= kSmallNode || depth >= kMaxDepth) {
            int32_t n = new_node(1, box, parent, slot);
            oc.leaf_off[n] = (int32_t)oc.refs.size();
            oc.leaf_cnt[n] = (int32_t)ids.size();
            oc.refs.insert(oc.refs.end(), ids.begin(), ids.end());
            oc.leaves++;
            if ((int64_t)ids.size() > oc.max_leaf) oc.max_leaf = (int64_t)ids.size();
            if (depth > oc.max_depth) oc.max_depth = depth;
            return n;
        }
        Box oct[8];
        for (int i = 0; i < 8; ++i) oct[i] = octant_of(box, i);
        std::vector<int32_t> part[8];
        for (int32_t id : ids) {
            const TriV& t = tris[id];
            for (int i = 0; i < 8; ++i)
                if (overlaps(oct[i], t)) part[i].push_back(id);
        }
        ids.clear();
        ids.shrink_to_fit();
        int32_t me = new_node(0, box, parent, slot);
        oc.parents++;
        for (int i = 0; i < 8; ++i) {
            int32_t c = build(oct[i], std::move(part[i]), depth + 1, me, i);
            oc.child[8 * (size_t)me + i] = c;
        }
        return me;
    }
};

// ---- TOML -> SceneSpec (serde semantics of scene.rs:292-348) ----
using toml::Value;

bool get_f64(const Value* v, double* out) {
    if (!v || !v->is_number()) return false;
    *out = v->as_f64();
    return true;
}
bool get_vec3(const Value& t, const char* key, D3* out, std::string* err, bool required = true) {
    const Value* v = t.get(key);
    if (!v) {
        if (required) *err = std::string("missing field `") + key + "`";
        return !required;
    }
    if (v->kind != Value::Kind::Array || v->array.size() != 3) {
        *err = std::string("field `") + key + "`: expected an array of 3 numbers";
        return false;
    }
    double x[3];
    for (int i = 0; i < 3; ++i)
        if (!get_f64(&v->array[i], &x[i])) {
            *err = std::string("field `") + key + "`: expected a number";
            return false;
        }
    *out = D3{x[0], x[1], x[2]};
    return true;
}
bool get_num(const Value& t, const char* key, double* out, std::string* err) {
    const Value* v = t.get(key);
    if (!v) { *err = std::string("missing field `") + key + "`"; return false; }
    if (!get_f64(v, out)) { *err = std::string("field `") + key + "`: expected a number"; return false; }
    return true;
}
bool get_str(const Value& t, const char* key, std::string* out, std::string* err) {
    const Value* v = t.get(key);
    if (!v) { *err = std::string("missing field `") + key + "`"; return false; }
    if (v->kind != Value::Kind::String) { *err = std::string("field `") + key + "`: expected a string"; return false; }
    *out = v->str;
    return true;
}

void apply_translate(Object& o, Mesh* m, D3 t) {  // geometry.rs:427
    if (o.geom == RT_GEOM_MESH) {
        for (D3& v : m->vertices) v = add(v, t);
        m->bbox.min = add(m->bbox.min, t);
        m->bbox.max = add(m->bbox.max, t);
    } else {
        o.pos = add(o.pos, t);
    }
}
void apply_scale(Object& o, Mesh* m, double s) {  // geometry.rs:493 (bbox growth quirk kept)
    if (o.geom == RT_GEOM_SPHERE) o.r *= s;
    else if (o.geom == RT_GEOM_MESH) {
        D3 c = centre(m->bbox);
        for (D3& v : m->vertices) v = add(c, scale(sub(v, c), s));
        m->bbox.min = add(m->bbox.min, scale(sub(m->bbox.min, c), s));
        m->bbox.max = add(m->bbox.max, scale(sub(m->bbox.max, c), s));
    }
}
void apply_rotate(Object& o, Mesh* m, int axis, double a) {  // geometry.rs:445-491
    auto rot = [&](D3 v) { return axis == 0 ? rotx(v, a) : axis == 1 ? roty(v, a) : rotz(v, a); };
    if (o.geom == RT_GEOM_PLANE) o.n = rot(o.n);
    else if (o.geom == RT_GEOM_MESH) {
        D3 c = centre(m->bbox);
        for (D3& v : m->vertices) v = add(c, rot(sub(v, c)));
        m->bbox = enclose(m->vertices);
    }
}

int parse_object(const Value& spec, const std::string& assets_dir, Scene* sc, std::string* err) {
    Object o;
    if (!get_vec3(spec, "emitted", &o.emitted, err, false)) return RT_E_PARSE;
    const Value* brdf = spec.get("brdf");
    if (!brdf || brdf->kind != Value::Kind::Table) { *err = "missing field `brdf`"; return RT_E_PARSE; }
    std::string bt;
    if (!get_str(*brdf, "type", &bt, err)) return RT_E_PARSE;
    if (bt == "diffuse") {
        o.brdf = RT_BRDF_DIFFUSE;
        if (!get_vec3(*brdf, "kd", &o.k, err)) return RT_E_PARSE;
    } else if (bt == "specular") {
        o.brdf = RT_BRDF_SPECULAR;
        if (!get_vec3(*brdf, "ks", &o.k, err)) return RT_E_PARSE;
    } else if (bt == "phong") {
        o.brdf = RT_BRDF_PHONG;
        if (!get_num(*brdf, "kd", &o.ph_kd, err) || !get_num(*brdf, "ks", &o.ph_ks, err) ||
            !get_vec3(*brdf, "color_d", &o.color_d, err) || !get_vec3(*brdf, "color_s", &o.color_s, err))
            return RT_E_PARSE;
        const Value* pw = brdf->get("power");
        if (!pw || pw->kind != Value::Kind::Int || pw->i < 0) { *err = "field `power`: expected a non-negative integer"; return RT_E_PARSE; }
        o.ph_power = (int32_t)pw->i;
    } else {
        *err = "unknown variant `" + bt + "`, expected one of `diffuse`, `specular`, `phong`";
        return RT_E_PARSE;
    }
    const Value* g = spec.get("geometry");
    if (!g || g->kind != Value::Kind::Table) { *err = "missing field `geometry`"; return RT_E_PARSE; }
    std::string gt;
    if (!get_str(*g, "type", &gt, err)) return RT_E_PARSE;
    Mesh mesh;
    if (gt == "sphere") {
        o.geom = RT_GEOM_SPHERE;
        if (!get_vec3(*g, "pos", &o.pos, err) || !get_num(*g, "r", &o.r, err)) return RT_E_PARSE;
    } else if (gt == "plane") {
        o.geom = RT_GEOM_PLANE;
        if (!get_vec3(*g, "pos", &o.pos, err) || !get_vec3(*g, "n", &o.n, err)) return RT_E_PARSE;
    } else if (gt == "cube") {
        D3 p;
        double s;
        if (!get_vec3(*g, "pos", &p, err) || !get_num(*g, "size", &s, err)) return RT_E_PARSE;
        o.geom = RT_GEOM_MESH;
        mesh = make_prism(p, s, s, s);
    } else if (gt == "prism") {
        D3 p, s;
        if (!get_vec3(*g, "pos", &p, err) || !get_vec3(*g, "size", &s, err)) return RT_E_PARSE;
        o.geom = RT_GEOM_MESH;
        mesh = make_prism(p, s.x, s.y, s.z);
    } else if (gt == "mesh") {
        std::string path;
        if (!get_str(*g, "path", &path, err)) return RT_E_PARSE;
        o.geom = RT_GEOM_MESH;
        int rc = load_obj(assets_dir + "/" + path, &mesh, err);
        if (rc != RT_OK) return rc;
    } else {
        *err = "unknown variant `" + gt + "`, expected one of `sphere`, `cube`, `prism`, `plane`, `mesh`";
        return RT_E_PARSE;
    }
    if (const Value* tfs = spec.get("transforms")) {  // scene.rs:411-429, applied in file order
        if (tfs->kind != Value::Kind::Array) { *err = "field `transforms`: expected an array"; return RT_E_PARSE; }
        for (const Value& t : tfs->array) {
            if (t.kind != Value::Kind::Table || t.table.size() != 1) {
                *err = "transform: expected a table with exactly one key";
                return RT_E_PARSE;
            }
            const std::string& name = t.table[0].first;
            const Value& val = t.table[0].second;
            Mesh* mp = o.geom == RT_GEOM_MESH ? &mesh : nullptr;
            if (name == "translate") {
                if (val.kind != Value::Kind::Array || val.array.size() != 3) { *err = "translate: expected [x, y, z]"; return RT_E_PARSE; }
                double x[3];
                for (int i = 0; i < 3; ++i)
                    if (!get_f64(&val.array[i], &x[i])) { *err = "translate: expected numbers"; return RT_E_PARSE; }
                apply_translate(o, mp, D3{x[0], x[1], x[2]});
            } else {
                double a;
                if (!get_f64(&val, &a)) { *err = name + ": expected a number"; return RT_E_PARSE; }
                if (name == "scale") apply_scale(o, mp, a);
                else if (name == "rotate_x") apply_rotate(o, mp, 0, a);
                else if (name == "rotate_y") apply_rotate(o, mp, 1, a);
                else if (name == "rotate_z") apply_rotate(o, mp, 2, a);
                else {
                    *err = "unknown variant `" + name + "`, expected one of `translate`, `scale`, `rotate_x`, `rotate_y`, `rotate_z`";
                    return RT_E_PARSE;
                }
            }
        }
    }
    if (o.geom == RT_GEOM_MESH) {
        build_octree(mesh);  // Mesh::accelerate (scene.rs:430-432)
        o.mesh = (int32_t)sc->meshes.size();
        sc->meshes.push_back(std::move(mesh));
    }
    sc->objects.push_back(o);
    return RT_OK;
}

// Rust `str::parse::<usize>`: optional '+', then at least one ASCII digit, nothing else; values
// above usize::MAX (64-bit) are an error.
bool parse_usize(const char* s, size_t n, uint64_t* out) {
    size_t i = 0;
    if (n && s[0] == '+') i = 1;
    if (i == n) return false;
    uint64_t v = 0;
    for (; i < n; ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        const uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = v;
    return true;
}

}  // namespace

Mesh make_mesh(std::vector<D3> vertices, std::vector<uint32_t> indices) {  // Mesh::new (geometry.rs:754)
    Mesh m;
    m.vertices = std::move(vertices);
    m.indices = std::move(indices);
    size_t nt = m.num_triangles();
    m.areas.resize(nt);
    double total = 0.0;
    for (size_t i = 0; i < nt; ++i) {
        D3 a = m.vertices[m.indices[3 * i]], b = m.vertices[m.indices[3 * i + 1]], c = m.vertices[m.indices[3 * i + 2]];
        double ab = magn(sub(a, b)), bc = magn(sub(b, c)), ca = magn(sub(c, a));  // Heron, geometry.rs:614
        double s = (ab + bc + ca) / 2.0;
        m.areas[i] = std::sqrt(s * (s - ab) * (s - bc) * (s - ca));
        total += m.areas[i];
    }
    m.surface_area = total;
    m.bbox = enclose(m.vertices);
    return m;
}

Mesh make_prism(D3 p, double w, double h, double d) {  // geometry.rs:839-866
    std::vector<D3> v = {{p.x, p.y, p.z},         {p.x, p.y, p.z + d},         {p.x, p.y + h, p.z},
                         {p.x, p.y + h, p.z + d}, {p.x + w, p.y, p.z},         {p.x + w, p.y, p.z + d},
                         {p.x + w, p.y + h, p.z}, {p.x + w, p.y + h, p.z + d}};
    std::vector<uint32_t> idx = {1, 3, 7, 1, 5, 7, 0, 2, 6, 0, 4, 6, 0, 1, 3, 0, 2, 3,
                                 4, 5, 7, 4, 6, 7, 2, 3, 7, 2, 6, 7, 0, 1, 5, 0, 4, 5};
    return make_mesh(std::move(v), std::move(idx));
}

int load_obj(const std::string& path, Mesh* out, std::string* err) {  // Mesh::load (geometry.rs:777-833)
    std::ifstream f(path, std::ios::binary);
    if (!f) { *err = "cannot open mesh file " + path + ": " + std::strerror(errno); return RT_E_IO; }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    std::vector<D3> verts;
    std::vector<uint32_t> idx;
    size_t pos = 0, lineno = 0;
    auto is_ws = [](char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; };
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size();
        ++lineno;
        // split_whitespace tokens of this line
        const char* tok[5];
        size_t len[5];
        int nt = 0;
        size_t i = pos;
        while (i < eol && nt < 5) {
            while (i < eol && is_ws(text[i])) ++i;
            if (i >= eol) break;
            size_t st = i;
            while (i < eol && !is_ws(text[i])) ++i;
            tok[nt] = text.data() + st;
            len[nt] = i - st;
            ++nt;
        }
        pos = eol + 1;
        if (nt == 0) continue;
        std::string cmd(tok[0], len[0]);
        if (cmd == "v" || cmd == "vn") {
            if (nt < 4) { *err = path + ":" + std::to_string(lineno) + ": unexpected end of file"; return RT_E_PARSE; }
            double x[3];
            for (int k = 0; k < 3; ++k) {
                std::string s(tok[k + 1], len[k + 1]);
                char* end = nullptr;
                x[k] = std::strtod(s.c_str(), &end);
                if (end == s.c_str() || *end) { *err = "Ill-formed float " + s; return RT_E_PARSE; }
            }
            if (cmd == "v") verts.push_back(D3{x[0], x[1], x[2]});
        } else if (cmd == "f") {
            if (nt < 4) { *err = path + ":" + std::to_string(lineno) + ": unexpected end of file"; return RT_E_PARSE; }
            for (int k = 0; k < 3; ++k) {
                // parse_face: up to three '/'-separated parts, each must be a usize
                const char* s = tok[k + 1];
                size_t n = len[k + 1], st = 0;
                uint64_t first = 0;
                for (int part = 0; part < 3; ++part) {
                    size_t sl = st;
                    while (sl < n && s[sl] != '/') ++sl;
                    uint64_t val;
                    if (!parse_usize(s + st, sl - st, &val)) {
                        *err = "Ill-formed integer " + std::string(s + st, sl - st);
                        return RT_E_PARSE;
                    }
                    if (part == 0) first = val;
                    if (sl >= n) break;
                    st = sl + 1;
                }
                if (first == 0) { *err = "face index 0 (usize underflow in the reference)"; return RT_E_PARSE; }
                idx.push_back((uint32_t)(first - 1));
            }
        }
    }
    for (uint32_t i : idx)
        if (i >= verts.size()) { *err = "face index out of range in " + path; return RT_E_PARSE; }
    *out = make_mesh(std::move(verts), std::move(idx));
    return RT_OK;
}

void build_octree(Mesh& m) {  // Octree::build (geometry.rs:1149)
    Octree oc;
    oc.root = m.bbox;
    std::vector<TriV> tris(m.num_triangles());
    for (size_t i = 0; i < tris.size(); ++i)
        tris[i] = TriV{m.vertices[m.indices[3 * i]], m.vertices[m.indices[3 * i + 1]], m.vertices[m.indices[3 * i + 2]]};
    std::vector<int32_t> all(tris.size());
    for (size_t i = 0; i < all.size(); ++i) all[i] = (int32_t)i;
    Builder b{tris, oc};
    b.build(m.bbox, std::move(all), 1, -1, 0);
    m.octree = std::move(oc);
}

int pick_light(Scene* s, std::string* err) {
    s->light = -1;
    for (size_t i = 0; i < s->objects.size(); ++i) {
        D3 e = s->objects[i].emitted;
        if (!(std::fabs(e.x) < 0.00001 && std::fabs(e.y) < 0.00001 && std::fabs(e.z) < 0.00001)) {
            s->light = (int32_t)i;
            break;
        }
    }
    if (s->light < 0) { *err = "scene has no emitting object (the reference hits unreachable!, scene.rs:136)"; return RT_E_INVAL; }
    if (s->objects[s->light].geom == RT_GEOM_PLANE) {
        *err = "light source is a plane: Geometry::sample is unimplemented! for planes (geometry.rs:593)";
        return RT_E_INVAL;
    }
    return RT_OK;
}

void camera_frame(const Scene& s, int width, int height, double cx[3], double cy[3]) {
    double w = (double)width, h = (double)height;
    D3 x{w * 0.5135 / h, 0., 0.};
    D3 y = scale(normd(crossp(x, s.cam_dir)), 0.5135);
    cx[0] = x.x; cx[1] = x.y; cx[2] = x.z;
    cy[0] = y.x; cy[1] = y.y; cy[2] = y.z;
}

int load_scene_toml(const std::string& toml_path, const std::string& assets_dir, Scene* out, std::string* err) {
    std::ifstream f(toml_path, std::ios::binary);
    if (!f) { *err = "cannot open scene " + toml_path + ": " + std::strerror(errno); return RT_E_IO; }
    std::stringstream ss;
    ss << f.rdbuf();
    Value root;
    std::string perr;
    if (!toml::parse(ss.str(), &root, &perr)) { *err = toml_path + ": " + perr; return RT_E_PARSE; }
    Scene sc;
    const Value* cam = root.get("camera");
    if (!cam || cam->kind != Value::Kind::Table) { *err = "missing field `camera`"; return RT_E_PARSE; }
    if (!get_vec3(*cam, "pos", &sc.cam_pos, err) || !get_vec3(*cam, "dir", &sc.cam_dir, err)) return RT_E_PARSE;
    const Value* objs = root.get("objects");
    if (!objs || objs->kind != Value::Kind::Array) { *err = "missing field `objects`"; return RT_E_PARSE; }
    for (size_t i = 0; i < objs->array.size(); ++i) {
        const Value& o = objs->array[i];
        if (o.kind != Value::Kind::Table) { *err = "objects: expected tables"; return RT_E_PARSE; }
        std::string e;
        int rc = parse_object(o, assets_dir, &sc, &e);
        if (rc != RT_OK) { *err = "objects[" + std::to_string(i) + "]: " + e; return rc; }
    }
    int rc = pick_light(&sc, err);
    if (rc != RT_OK) return rc;
    *out = std::move(sc);
    return RT_OK;
}

int scene_from_desc(const rt_scene_desc* d, Scene* out, std::string* err) {
    if (!d || (d->n_objects && !d->objects) || (d->n_meshes && !d->meshes)) { *err = "null scene descriptor"; return RT_E_INVAL; }
    Scene sc;
    sc.cam_pos = D3{d->cam_pos[0], d->cam_pos[1], d->cam_pos[2]};
    sc.cam_dir = D3{d->cam_dir[0], d->cam_dir[1], d->cam_dir[2]};
    for (uint32_t i = 0; i < d->n_meshes; ++i) {
        const rt_mesh_desc& md = d->meshes[i];
        if ((md.n_vertices && !md.vertices) || (md.n_triangles && !md.indices)) { *err = "null mesh arrays"; return RT_E_INVAL; }
        std::vector<D3> v(md.n_vertices);
        for (uint32_t k = 0; k < md.n_vertices; ++k) v[k] = D3{md.vertices[3 * k], md.vertices[3 * k + 1], md.vertices[3 * k + 2]};
        std::vector<uint32_t> idx(md.indices, md.indices + 3 * (size_t)md.n_triangles);
        for (uint32_t x : idx)
            if (x >= md.n_vertices) { *err = "mesh index out of range"; return RT_E_INVAL; }
        Mesh m = make_mesh(std::move(v), std::move(idx));
        m.bbox = Box{{md.bbox_min[0], md.bbox_min[1], md.bbox_min[2]}, {md.bbox_max[0], md.bbox_max[1], md.bbox_max[2]}};
        m.surface_area = md.surface_area;
        build_octree(m);
        sc.meshes.push_back(std::move(m));
    }
    for (uint32_t i = 0; i < d->n_objects; ++i) {
        const rt_object_desc& od = d->objects[i];
        Object o;
        o.emitted = D3{od.emitted[0], od.emitted[1], od.emitted[2]};
        o.brdf = od.brdf_kind;
        o.k = D3{od.k[0], od.k[1], od.k[2]};
        o.ph_kd = od.phong_kd;
        o.ph_ks = od.phong_ks;
        o.ph_power = od.phong_power;
        o.color_d = D3{od.color_d[0], od.color_d[1], od.color_d[2]};
        o.color_s = D3{od.color_s[0], od.color_s[1], od.color_s[2]};
        o.geom = od.geom_kind;
        o.pos = D3{od.pos[0], od.pos[1], od.pos[2]};
        o.r = od.r;
        o.n = D3{od.n[0], od.n[1], od.n[2]};
        o.mesh = od.mesh;
        if (o.brdf < 0 || o.brdf > 2 || o.geom < 0 || o.geom > 2) { *err = "bad brdf/geometry kind"; return RT_E_INVAL; }
        if (o.geom == RT_GEOM_MESH && (o.mesh < 0 || (uint32_t)o.mesh >= d->n_meshes)) { *err = "bad mesh index"; return RT_E_INVAL; }
        sc.objects.push_back(o);
    }
    int rc = pick_light(&sc, err);
    if (rc != RT_OK) return rc;
    *out = std::move(sc);
    return RT_OK;
}

}  // namespace rt::host
