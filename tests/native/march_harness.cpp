// Test-only host build of the product's skipping march (pt_march.hpp) so the
// CPU suite can compare it, bit for bit, with the oracle's literal march.
#include <cstdint>

#include "../../rs-pathtracing_amd/csrc/pt_march.hpp"

extern "C" int march_heart(double step, int passes, const double *inv /*3x4 row-major*/, const double *o,
                           const double *d, double min_t, double max_t, double *t, uint32_t *steps,
                           uint32_t *blocks) {
    // inverse_transform_ray (transform.rs:32-37), as pt_device.hpp xf_point / xf_vector
    double ox = o[0] * inv[0] + o[1] * inv[1] + o[2] * inv[2] + inv[3];
    double oy = o[0] * inv[4] + o[1] * inv[5] + o[2] * inv[6] + inv[7];
    double oz = o[0] * inv[8] + o[1] * inv[9] + o[2] * inv[10] + inv[11];
    double dx = d[0] * inv[0] + d[1] * inv[1] + d[2] * inv[2];
    double dy = d[0] * inv[4] + d[1] * inv[5] + d[2] * inv[6];
    double dz = d[0] * inv[8] + d[1] * inv[9] + d[2] * inv[10];
    pt::march::MarchStats st{0, 0, 0};
    int hit = pt::march::heart_march<true>(step, passes, ox, oy, oz, dx, dy, dz, min_t, max_t, t, &st) ? 1 : 0;
    *steps = st.steps;
    *blocks = st.blocks;
    steps[1] = st.tries;
    return hit;
}

// lin_room (the straight-line form the kernels use) against lin_init (the
// branchy original) on n pseudo-random (x, c) pairs: the same room and the
// same (X, R, u) wherever lin_init's room is >= 2, a room < 2 elsewhere.
// Returns the number of disagreements.
extern "C" long lin_room_check(long n, uint64_t seed) {
    using namespace pt::march;
    uint64_t s = seed;
    auto next = [&s]() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto unit = [&]() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0; };
    long bad = 0;
    for (long i = 0; i < n; i++) {
        const int mode = (int)(i % 6);
        double x = unit() * ldexp(1.0, (int)(next() % 40) - 20);
        double c = unit() * ldexp(1.0, (int)(next() % 60) - 50);
        if (mode == 1) x = ldexp(1.0, (int)(next() % 20) - 10) * (1.0 + 1e-15 * (double)(next() % 8));  // binade edges
        if (mode == 2) c = ldexp((double)(next() % 8) + 0.5, (int)(next() % 10) - 57);                  // ties
        if (mode == 3) c = 0.0;
        if (mode == 4) x = -x;
        Lin A, B;
        const int64_t ra = lin_init(x, c, &A);
        const double rb = lin_room(x, c, &B);
        const double rad = ra >= BIG ? BIGD : (double)ra;
        const bool same = ra >= 2 ? rad == rb && (A.frozen ? B.frozen : (A.X == B.X && A.R == B.R && A.u == B.u))
                                  : rb < 2.0;
        bad += same ? 0 : 1;
    }
    return bad;
}

// advance(x, c, k) against k literal additions fl(x + c), on n pseudo-random
// walks of up to 3000 steps, a third of them across zero.  Returns the number
// of walks whose end point differs.
extern "C" long advance_check(long n, uint64_t seed) {
    using namespace pt::march;
    uint64_t s = seed;
    auto next = [&s]() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto unit = [&]() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0; };
    long bad = 0;
    for (long i = 0; i < n; i++) {
        const int64_t k = 1 + (int64_t)(next() % 3000);
        double c = unit() * ldexp(1.0, -(int)(next() % 20) - 4);
        double x = unit() * ldexp(1.0, (int)(next() % 8) - 4);
        if (i % 3 == 0) x = -c * (double)k * (0.2 + 0.6 * (unit() + 1.0) * 0.5);  // crosses zero within the walk
        double lit = x;
        for (int64_t j = 0; j < k; j++) lit = lit + c;
        bad += advance(x, c, k) == lit ? 0 : 1;
    }
    return bad;
}

