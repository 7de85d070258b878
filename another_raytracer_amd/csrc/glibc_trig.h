// glibc_trig.h — the C library's acos and atan2 as get_sphere_uv (sphere.h:24-37) calls them, restated operation by
// operation so that host and device return glibc's bits.
//
// glibc 2.35 (this image) selects, on x86-64 CPUs with FMA and AVX2, the FMA builds of sysdeps/ieee754/dbl-64/
// e_asin.c (__ieee754_acos) and e_atan2.c (__ieee754_atan2): IBM's table-driven algorithms with their multi-precision
// fallbacks removed.  Neither is correctly rounded (tools/acos_atan2_cr.c against MPFR: 0.07 % / 0.09 % of unit-vector
// arguments differ from the correct rounding), so no independent implementation reproduces their last bits; the
// sequences below are those builds' machine code read back instruction for instruction -- which products are fused
// (the compiler contracted a * b + c into FMAs), which are rounded separately, in its order -- with their data
// (glibc_trig_data.h, generated from libm.so.6 by tools/gen_glibc_trig.py).  tests/test_glibc_trig.py compares both
// with the C library on tens of millions of arguments (every branch, the unit-vector components get_sphere_uv passes,
// the special values); tools/uv_check.hip checks that the device computes the host's bits.
//
// The data sits in one table the caller passes (TrigTab): on the host the arrays below, on the device a copy uploaded
// with the scene (device.h uv_table), so that no constant becomes a literal the compiler would hoist into the path
// loop's registers.  atan2 runs in round-to-nearest, the only mode the renderer uses (glibc switches to it if needed).
#pragma once
#include <cstdint>
#include <cstring>

#include "glibc_trig_data.h"

#if defined(__HIPCC__)
#define ART_TRIG_HD __host__ __device__
#else
#define ART_TRIG_HD
#endif

namespace art {

namespace glibc_trig_data {
// the device copy's layout: [constants][asncs][rsqrt seeds by mantissa][rsqrt seeds by exponent][atan2 table]
constexpr int kOffConsts = 0;
constexpr int kOffAsncs = kNumConsts;
constexpr int kOffRsqM = kOffAsncs + kAsncsSize;
constexpr int kOffRsqE = kOffRsqM + kRsqMSize;
constexpr int kOffAtan = kOffRsqE + kRsqESize;
constexpr int kTrigDoubles = kOffAtan + kAtanSize;
static const double kTrigHost[kTrigDoubles] = {ART_TRIG_CONSTS, ART_TRIG_ASNCS, ART_TRIG_RSQ_M, ART_TRIG_RSQ_E, ART_TRIG_ATAN};
}  // namespace glibc_trig_data

// The data of one call site: constants (possibly an LDS copy) and the four tables (global memory on the device).
struct TrigTab {
    const double* c;  // kNumConsts constants
    const double* t;  // the whole kTrigHost layout (tables at their kOff* offsets)
    ART_TRIG_HD TrigTab(const double* consts, const double* all) : c(consts), t(all) {}
};

ART_TRIG_HD inline uint64_t trig_bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
ART_TRIG_HD inline double trig_from(uint64_t u) {
    double x;
    std::memcpy(&x, &u, 8);
    return x;
}
ART_TRIG_HD inline double trig_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
// (r & 0x7fff...) | (y & 0x8000...): the vandpd / vorpd pair that gives atan2's result the sign of y
ART_TRIG_HD inline double trig_copysign(double r, double y) {
    return trig_from((trig_bits(r) & 0x7FFFFFFFFFFFFFFFull) | (trig_bits(y) & 0x8000000000000000ull));
}

// acos's table intervals: xx = |x| - T[n]; p = T[n+m] .. T[n+2] by Horner in xx, then x^2 * p + T[n+m+1];
// t = xx * T[n+1] + p; y = T[n+m+2]; x > 0: (hp1 - t) + (hp0 - y), x < 0: (t + hp1) + (y + hp0)
ART_TRIG_HD inline double glibc_acos_interval(const TrigTab& g, double x, int32_t hx, int n, int m) {
    using namespace glibc_trig_data;
    const double* T = g.t + kOffAsncs;
    const double ax = hx > 0 ? x : -x;
    const double xx = ax - T[n];
    double p = T[n + m];
    for (int j = m - 1; j >= 2; --j) p = trig_fma(xx, p, T[n + j]);
    const double x2 = xx * xx;
    p = trig_fma(x2, p, T[n + m + 1]);
    const double t = trig_fma(xx, T[n + 1], p);
    const double y = T[n + m + 2];
    if (hx > 0) return (g.c[kHp1] - t) + (g.c[kHp0] - y);
    return (t + g.c[kHp1]) + (y + g.c[kHp0]);
}

ART_TRIG_HD inline double glibc_acos(double x, const TrigTab& g) {
    using namespace glibc_trig_data;
    const double* c = g.c;
    const uint64_t b = trig_bits(x);
    const int32_t hx = static_cast<int32_t>(b >> 32);
    const uint32_t lx = static_cast<uint32_t>(b);
    const int32_t k = hx & 0x7fffffff;
    if (k <= 0x3c87ffff) return c[kHp0];
    if (k <= 0x3fbfffff) {  // |x| < 0.125: an odd polynomial about 0
        const double x2 = x * x;
        double p = c[kA0];
        p = trig_fma(x2, p, c[kA1]);
        p = trig_fma(x2, p, c[kA2]);
        const double r = c[kHp0] - x;
        p = trig_fma(x2, p, c[kA3]);
        p = trig_fma(x2, p, c[kA4]);
        p = trig_fma(x2, p, c[kA5]);
        double s = c[kHp0] - r;
        const double x3 = x * x2;
        s = s - x;
        s = s + c[kHp1];
        p = trig_fma(-p, x3, s);
        return r + p;
    }
    if (k <= 0x3fdfffff) {  // [0.125, 0.5)
        const int n = k <= 0x3fcfffff ? 11 * ((k >> 15) & 0x1f) : 11 * ((k >> 14) & 0x3f) + 0x160;
        return glibc_acos_interval(g, x, hx, n, 6);
    }
    if (k <= 0x3fe7ffff) return glibc_acos_interval(g, x, hx, 12 * ((k >> 13) & 0x7f) + 0x420, 7);  // [0.5, 0.75)
    if (k <= 0x3fed7fff) return glibc_acos_interval(g, x, hx, 13 * ((k >> 13) & 0x7f) + 0x3e0, 8);  // [0.75, 0.921875)
    if (k <= 0x3fee7fff) return glibc_acos_interval(g, x, hx, 14 * ((k >> 13) & 0x7f) + 0x374, 9);  // [0.921875, 0.953125)
    if (k <= 0x3feeffff) return glibc_acos_interval(g, x, hx, 15 * ((k >> 13) & 0x7f) + 0x300, 10);  // [0.953125, 0.96875)
    if (k <= 0x3fefffff) {  // [0.96875, 1): acos = 2 asin(sqrt((1 - |x|) / 2)), the square root by a seeded Newton step
        const double one = c[kOne];
        double z = hx > 0 ? one - x : x + one;
        z = z * c[kHalf];
        const uint64_t zb = trig_bits(z);
        const int32_t e = static_cast<int32_t>(static_cast<int64_t>(zb) >> 53);
        const int32_t mi = static_cast<int32_t>(static_cast<int64_t>(zb) >> 46) & 0x7f;
        const double y0 = g.t[kOffRsqM + mi] * g.t[kOffRsqE + (0x1ff - e)];
        double t = y0 * y0;
        t = trig_fma(-t, z, one);
        double q = c[kS0];
        q = trig_fma(t, q, c[kS1]);
        q = trig_fma(t, q, c[kS2]);
        q = trig_fma(t, q, c[kS3]);
        const double c27 = c[kTwo27];
        q = q * y0;
        const double s = z * q;
        double h = q * c[kHalf];
        h = trig_fma(-s, h, c[kThreeHalves]);
        const double a = trig_fma(s, c27, s);
        const double hi = trig_fma(-c27, s, a);
        h = trig_fma(h, s, hi);
        double r = trig_fma(-hi, hi, z);
        r = r / h;
        double pz = c[kA0];
        pz = trig_fma(z, pz, c[kA1]);
        pz = trig_fma(z, pz, c[kA2]);
        pz = trig_fma(z, pz, c[kA3]);
        pz = trig_fma(z, pz, c[kA4]);
        pz = trig_fma(z, pz, c[kA5]);
        double w = pz * z;
        const double sq = hi + r;
        w = w * sq;
        if (hx < 0) {
            double a2 = c[kHp1] - r;
            const double b2 = c[kHp0] - hi;
            a2 = a2 - w;
            const double res = a2 + b2;
            return res + res;
        }
        double res = r + w;
        res = res + hi;
        return res + res;
    }
    if (k == 0x3ff00000 && lx == 0) return hx > 0 ? 0.0 : c[kPi];  // acos(1) = +0, acos(-1) = pi
    if (k > 0x7ff00000 || (k == 0x7ff00000 && lx != 0)) return x + x;  // NaN
    // |x| > 1 (infinities included): the compat wrapper's __kernel_standard value, NAN -- the positive quiet NaN (the
    // x86 0/0 default NaN would carry the sign bit)
    return trig_from(0x7ff8000000000000ull);
}

// atan2's table evaluation about its entry i (u in [1/16, 1]): returns the table's polynomial in z = (u - T[7i]) + uu
ART_TRIG_HD inline int glibc_atan_entry(const TrigTab& g, double u) {
    using namespace glibc_trig_data;
    double r = trig_fma(u, g.c[kTwo8], g.c[kTwo52]);  // round(256 u) by the 2^52 shifter
    r = r - g.c[kTwo52];
    return static_cast<int>(r) - 16;
}
ART_TRIG_HD inline double glibc_atan_poly(const double* E, double z) {
    double p = E[6];
    p = trig_fma(z, p, E[5]);
    p = trig_fma(z, p, E[4]);
    p = trig_fma(z, p, E[3]);
    p = trig_fma(z, p, E[2]);
    return p;
}
// the small-argument polynomial (u < 1/16): coefficients d0..d5 in v = u^2
ART_TRIG_HD inline double glibc_atan_small(const double* c, double v) {
    using namespace glibc_trig_data;
    double p = c[kD0];
    p = trig_fma(v, p, c[kD1]);
    p = trig_fma(v, p, c[kD2]);
    p = trig_fma(v, p, c[kD3]);
    p = trig_fma(v, p, c[kD4]);
    p = trig_fma(v, p, c[kD5]);
    return p;
}

ART_TRIG_HD inline double glibc_atan2(double y, double x, const TrigTab& g) {
    using namespace glibc_trig_data;
    const double* c = g.c;
    const uint64_t bx = trig_bits(x), by = trig_bits(y);
    const int32_t hx = static_cast<int32_t>(bx >> 32), hy = static_cast<int32_t>(by >> 32);
    const uint32_t lx = static_cast<uint32_t>(bx), ly = static_cast<uint32_t>(by);
    const int32_t ex = hx & 0x7ff00000, ey = hy & 0x7ff00000;
    // special operands (e_atan2.c's prologue)
    if (ex == 0x7ff00000 && ((hx & 0xfffff) | lx) != 0) return x + y;  // x NaN
    bool general = false;
    if (ey == 0x7ff00000) {
        if (((hy & 0xfffff) | ly) != 0) return y + y;  // y NaN
    } else if (hy == 0) {
        if (ly == 0) return hx < 0 ? c[kPi] : 0.0;  // y = +0
        if (x != x || x != 0.0) general = true;    // y positive subnormal
        else return c[kHp0];
    }
    if (!general) {
        if (ly == 0 && hy == static_cast<int32_t>(0x80000000u)) return hx < 0 ? c[kMPi] : -0.0;  // y = -0
        if (x == 0.0) return hy < 0 ? c[kMHp0] : c[kHp0];  // x = +-0, y != 0
    }
    // x or y infinite
    if (hx == 0x7ff00000 && lx == 0) {  // x = +inf
        if (hy == 0x7ff00000) return c[kPi4];
        if (hy == static_cast<int32_t>(0xfff00000u)) return c[kMPi4];
        return hy < 0 ? -0.0 : 0.0;
    }
    if (lx == 0 && hx == static_cast<int32_t>(0xfff00000u)) {  // x = -inf
        if (hy == 0x7ff00000) return c[kPi34];
        if (hy == static_cast<int32_t>(0xfff00000u)) return c[kMPi34];
        return hy < 0 ? c[kMPi] : c[kPi];
    }
    if (hy == 0x7ff00000) return c[kHp0];                                           // y = +inf
    if (hy == static_cast<int32_t>(0xfff00000u) && ly == 0) return c[kMHp0];       // y = -inf
    // finite, non-zero x (and y)
    double ax = x < 0.0 ? -x : x;
    double ay = y < 0.0 ? -y : y;
    const int32_t d = ey - ex;
    if (d > 0x38fffff) return !(0.0 < y) ? c[kMHp0] : c[kHp0];  // |y / x| > 2^57
    if (d < static_cast<int32_t>(0xfc700001u)) {                    // |y / x| < 2^-57
        if (!(x > 0.0)) return !(0.0 < y) ? c[kMPi] : c[kPi];
        return trig_copysign(ay / ax, y);
    }
    if (c[kTwoM500] > ax || c[kTwoM500] > ay) {
        ax = ax * c[kTwo500];
        ay = ay * c[kTwo500];
    }
    if (ax > c[kTwo500] || ay > c[kTwo500]) {
        ax = ax * c[kTwoM500];
        ay = ay * c[kTwoM500];
    }
    // u = min / max and its correction uu (the quotient's remainder, exact by an FMA)
    double u, uu;
    if (ax > ay) {
        u = ay / ax;
        const double p = ax * u;
        const double e = trig_fma(ax, u, -p);
        uu = ay - p;
        uu = uu - e;
        uu = uu / ax;
    } else {
        u = ax / ay;
        const double p = ay * u;
        const double e = trig_fma(ay, u, -p);
        uu = ax - p;
        uu = uu - e;
        uu = uu / ay;
    }
    const double* T = g.t + kOffAtan;
    if (x > 0.0) {
        if (ax > ay) {  // |y| < x: atan(u)
            if (c[kSixteenth] > u) {
                const double v = u * u;
                const double p = glibc_atan_small(c, v);
                double w = u * v;
                w = trig_fma(w, p, uu);
                w = u + w;
                return trig_copysign(w, y);
            }
            const int i = glibc_atan_entry(g, u);
            const double* E = T + 7 * i;
            double z6 = u - E[0];
            double s = uu + z6;  // the argument about the entry, with its rounding error in uu'
            double uu2;
            if (__builtin_fabs(z6) > __builtin_fabs(uu)) {
                z6 = z6 - s;
                uu2 = z6 + uu;
            } else {
                uu2 = uu - s;
                uu2 = uu2 + z6;
            }
            const double z2 = s * s;
            double p = E[6];
            p = trig_fma(s, p, E[5]);
            p = trig_fma(s, p, E[4]);
            const double e2 = E[2];
            p = trig_fma(s, p, E[3]);
            p = z2 * p;
            p = trig_fma(uu2, e2, p);
            double r = trig_fma(s, e2, p);
            r = r + E[1];
            return trig_copysign(r, y);
        }
        // |y| >= x: pi/2 - atan(u)
        if (c[kSixteenth] > u) {
            const double v = u * u;
            const double p = glibc_atan_small(c, v);
            double w = u * v;
            const double h = c[kHp0] - u;
            w = w * p;
            double s;
            if (c[kHp0] > __builtin_fabs(u)) {
                s = c[kHp0] - h;
                s = s - u;
            } else {
                const double t6 = u + h;
                s = c[kHp0] - t6;
            }
            s = s + c[kHp1];
            s = s - uu;
            s = s - w;
            s = s + h;
            return trig_copysign(s, y);
        }
        const int i = glibc_atan_entry(g, u);
        const double* E = T + 7 * i;
        double z = u - E[0];
        z = z + uu;
        double p = glibc_atan_poly(E, z);
        p = trig_fma(-z, p, c[kHp1]);
        double r = c[kHp0] - E[1];
        r = r + p;
        return trig_copysign(r, y);
    }
    // x < 0
    if (!(ay <= ax)) {  // |y| > |x|: pi/2 + atan(u)
        if (c[kSixteenth] > u) {
            const double v = u * u;
            const double p = glibc_atan_small(c, v);
            const double t7 = u + c[kHp0];
            double w = v * u;
            w = w * p;
            double s1;
            if (c[kHp0] > __builtin_fabs(u)) {
                double s = c[kHp0] - t7;
                s1 = s + u;
            } else {
                s1 = u - t7;
                s1 = s1 + c[kHp0];
            }
            s1 = s1 + c[kHp1];
            s1 = s1 + uu;
            s1 = s1 + w;
            s1 = s1 + t7;
            return trig_copysign(s1, y);
        }
        const int i = glibc_atan_entry(g, u);
        const double* E = T + 7 * i;
        double z = u - E[0];
        z = z + uu;
        double p = glibc_atan_poly(E, z);
        p = trig_fma(z, p, c[kHp1]);
        double r = c[kHp0] + E[1];
        r = r + p;
        return trig_copysign(r, y);
    }
    // |y| <= |x|: pi - atan(u)
    if (c[kSixteenth] > u) {
        const double v = u * u;
        const double p = glibc_atan_small(c, v);
        double w = v * u;
        const double h = c[kPi] - u;
        w = w * p;
        double s;
        if (c[kPi] > __builtin_fabs(u)) {
            s = c[kPi] - h;
            s = s - u;
        } else {
            const double t6 = h + u;
            s = c[kPi] - t6;
        }
        s = s + c[kPiLo];
        s = s - uu;
        s = s - w;
        s = s + h;
        return trig_copysign(s, y);
    }
    const int i = glibc_atan_entry(g, u);
    const double* E = T + 7 * i;
    double z = u - E[0];
    z = z + uu;
    double p = glibc_atan_poly(E, z);
    p = trig_fma(-z, p, c[kPiLo]);
    double r = c[kPi] - E[1];
    r = r + p;
    return trig_copysign(r, y);
}

// host callers (tests, tools): the host tables
inline double glibc_acos(double x) { return glibc_acos(x, TrigTab(glibc_trig_data::kTrigHost, glibc_trig_data::kTrigHost)); }
inline double glibc_atan2(double y, double x) { return glibc_atan2(y, x, TrigTab(glibc_trig_data::kTrigHost, glibc_trig_data::kTrigHost)); }

}  // namespace art
