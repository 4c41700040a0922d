// Host check (test infrastructure) of path_f64.h near_mesh32: every ray the f64 near_box passes also passes the padded
// single-precision test (random rays at the reference scenes' mesh boxes, half of them grazing a face within the f64
// pad, a fifth with an axis-parallel direction component; the device rcp modelled as 1 ulp off either way).
// g++ -O2 -std=c++17 -ffp-contract=off -o /tmp/near32_check tests/near32_check.cpp && /tmp/near32_check [rays per box]
#include <cmath>
#include <cstdio>
#include <random>
#include <algorithm>
#include <cstdlib>
static bool near_box(const double* bx, const double o[3], const double d[3], double pad, double tmax) {
    double t0 = 0.0, t1 = INFINITY;
    for (int k = 0; k < 3; ++k) {
        double lo = bx[k] - pad, hi = bx[3 + k] + pad;
        if (!(std::fabs(d[k]) >= 0x1p-900 && std::fabs(d[k]) <= 0x1p900)) {
            if (!(std::fabs(d[k]) < 0x1p-900)) return true;
            if (o[k] < lo || o[k] > hi) return false;
            continue;
        }
        double rc = 1.0 / d[k];
        double ta = (lo - o[k]) * rc, tb = (hi - o[k]) * rc;
        double tn = std::fmin(ta, tb), tf = std::fmax(ta, tb);
        t0 = std::fmax(t0, tn - 1e-9 * std::fabs(tn));
        t1 = std::fmin(t1, tf + 1e-9 * std::fabs(tf));
    }
    return t0 <= t1 && t0 <= tmax * (1.0 + 1e-9) + 1e-9;
}
static bool near32(const float* c32, float s32, const double od[3], const double dd[3], double tmax) {
    float o[3], d[3];
    for (int k = 0; k < 3; ++k) { o[k] = (float)od[k]; d[k] = (float)dd[k]; }
    const float pad = 0x1p-16f * (std::fmax(std::fabs(o[0]), std::fmax(std::fabs(o[1]), std::fabs(o[2]))) + s32);
    float t0 = 0.0f, t1 = INFINITY; bool keep = true;
    for (int k = 0; k < 3; ++k) {
        const float lo = c32[k] - pad, hi = c32[3 + k] + pad;
        const bool tiny = !(std::fabs(d[k]) >= 0x1p-60f);
        keep &= !tiny || !(o[k] < lo || o[k] > hi);
        float rc = 1.0f / d[k];
        rc = std::nextafter(rc, (rand() & 1) ? INFINITY : -INFINITY);  // the device's rcp is 1 ulp
        const float ta = (lo - o[k]) * rc, tb = (hi - o[k]) * rc;
        t0 = tiny ? t0 : std::fmax(t0, std::fmin(ta, tb));
        t1 = tiny ? t1 : std::fmin(t1, std::fmax(ta, tb));
    }
    const float tm = (float)tmax;
    return keep && !(t0 > t1 + 0x1p-16f * std::fabs(t1) + pad) && !(t0 > tm + 0x1p-16f * tm + pad);
}
int main(int argc, char** argv) {
    const int n_per_box = argc > 1 ? std::atoi(argv[1]) : 20000000;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(0, 1);
    const double boxes[3][6] = {{25.4, 15.3, 57.0, 44.7, 67.3, 82.2}, {-3.0, 0.0, 18.0, 34.0, 28.0, 49.0}, {48.0, 0.0, 15.0, 78.0, 24.0, 45.0}};
    long pass64 = 0, miss = 0, pass32 = 0, n = 0;
    for (const auto& bx : boxes) {
        double mx = 1.0;
        for (double v : bx) mx = std::fmax(mx, std::fabs(v));
        const double pad = 1e-7 * mx;
        float c32[6];
        for (int k = 0; k < 3; ++k) {
            float lo = (float)bx[k], hi = (float)bx[3 + k];
            if ((double)lo > bx[k]) lo = std::nextafter(lo, -INFINITY);
            if ((double)hi < bx[3 + k]) hi = std::nextafter(hi, INFINITY);
            c32[k] = lo; c32[3 + k] = hi;
        }
        const float s32 = (float)mx * (1.0f + 0x1p-20f);
        for (int i = 0; i < n_per_box; ++i) {
            double o[3], p[3], d[3];
            for (int k = 0; k < 3; ++k) o[k] = -20 + 140 * U(g);
            // aim at a point near the box surface (grazing cases) half the time
            for (int k = 0; k < 3; ++k) p[k] = bx[k] + (bx[3 + k] - bx[k]) * U(g);
            if (i & 1) { int k = i % 3; p[k] = (i & 2) ? bx[k] - pad * (U(g) * 2 - 0.5) : bx[3 + k] + pad * (U(g) * 2 - 0.5); }
            double L = 0; for (int k = 0; k < 3; ++k) { d[k] = p[k] - o[k]; L += d[k] * d[k]; }
            L = std::sqrt(L); for (int k = 0; k < 3; ++k) d[k] /= L;
            if (i % 5 == 0) d[i % 3] = 0.0;  // axis-parallel components
            const double tmax = (i % 7 == 0) ? INFINITY : L * (0.5 + U(g));
            const bool a = near_box(bx, o, d, pad, tmax), b = near32(c32, s32, o, d, tmax);
            pass64 += a; pass32 += b; ++n;
            if (a && !b) { ++miss; if (miss < 5) std::printf("MISS o=(%g %g %g) d=(%g %g %g) tmax=%g\n", o[0], o[1], o[2], d[0], d[1], d[2], tmax); }
        }
    }
    std::printf("%ld rays: f64 pass %ld, f32 pass %ld, f64-pass-but-f32-cull %ld\n", n, pass64, pass32, miss);
    return miss != 0;
}
