// Host check of csrc/glibc_trig.h against the C library's acos and atan2 (tests/test_glibc_trig.py builds and runs
// it): N uniform unit vectors (the acos(-y), atan2(-z, x) arguments get_sphere_uv passes), N arguments per acos
// interval and per atan2 octant / ratio band, the special values, and N random doubles of every exponent, compared
// bit for bit (NaN sign and payload included).  Prints one line per set and "mismatches <m> of <n>"; exit status 1
// if any.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "glibc_trig.h"

static uint64_t sm(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(uint64_t& s) { return static_cast<double>(sm(s) >> 11) * 0x1p-53; }
static bool same(double a, double b) {
    uint64_t x, y;
    std::memcpy(&x, &a, 8);
    std::memcpy(&y, &b, 8);
    return x == y;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
    uint64_t s = 2024, bad = 0, total = 0;
    auto acos_chk = [&](double x, uint64_t& b) {
        const double a = art::glibc_acos(x), r = std::acos(x);
        if (!same(a, r)) {
            if (bad + b < 8) std::printf("acos %a: restated %a, libm %a\n", x, a, r);
            ++b;
        }
    };
    auto atan2_chk = [&](double y, double x, uint64_t& b) {
        const double a = art::glibc_atan2(y, x), r = std::atan2(y, x);
        if (!same(a, r)) {
            if (bad + b < 8) std::printf("atan2 %a %a: restated %a, libm %a\n", y, x, a, r);
            ++b;
        }
    };
    {  // unit vectors
        uint64_t b = 0;
        for (uint64_t k = 0; k < n; ++k) {
            const double zc = 2.0 * u01(s) - 1.0, ph = 6.283185307179586 * u01(s), r = std::sqrt(std::fmax(0.0, 1.0 - zc * zc));
            const double x = r * std::cos(ph), y = zc, z = r * std::sin(ph);
            acos_chk(-y, b);
            atan2_chk(-z, x, b);
        }
        std::printf("unit_vectors n=%" PRIu64 " differs %" PRIu64 "\n", 2 * n, b);
        bad += b;
        total += 2 * n;
    }
    {  // acos: every interval, both signs, and the ends near +-1
        uint64_t b = 0, c = 0;
        const double edges[] = {0.0, 0x1p-54, 0.125, 0.25, 0.5, 0.75, 0.921875, 0.953125, 0.96875, 1.0};
        for (int i = 0; i + 1 < 10; ++i)
            for (uint64_t k = 0; k < n / 4; ++k, ++c) {
                const double x = edges[i] + (edges[i + 1] - edges[i]) * u01(s);
                acos_chk((sm(s) & 1) ? -x : x, b);
            }
        for (uint64_t k = 0; k < n / 4; ++k, ++c) {  // 1 - 2^-e..: the seeded square-root path's smallest arguments
            const double x = 1.0 - std::ldexp(1.0 + u01(s), -static_cast<int>(6 + sm(s) % 48));
            acos_chk((sm(s) & 1) ? -x : x, b);
        }
        std::printf("acos_intervals n=%" PRIu64 " differs %" PRIu64 "\n", c, b);
        bad += b;
        total += c;
    }
    {  // atan2: ratios across every band (|y/x| from 2^-70 to 2^70), every sign, magnitudes across the scaling limits
        uint64_t b = 0, c = 0;
        for (uint64_t k = 0; k < 2 * n; ++k, ++c) {
            const double ratio = std::ldexp(1.0 + u01(s), static_cast<int>(sm(s) % 141) - 70);
            const double mag = std::ldexp(1.0 + u01(s), static_cast<int>(sm(s) % 1200) - 600);
            double x = mag, y = mag * ratio;
            if (sm(s) & 1) std::swap(x, y);
            if (sm(s) & 1) x = -x;
            if (sm(s) & 1) y = -y;
            atan2_chk(y, x, b);
        }
        for (uint64_t k = 0; k < n; ++k, ++c) {  // |y/x| in [1/16, 1] and its inverse: the table path, densely
            const double u = 0.0625 + 0.9375 * u01(s), x = 1.0 + u01(s);
            double yy = u * x, xx = x;
            if (sm(s) & 1) std::swap(xx, yy);
            if (sm(s) & 1) xx = -xx;
            if (sm(s) & 1) yy = -yy;
            atan2_chk(yy, xx, b);
        }
        std::printf("atan2_bands n=%" PRIu64 " differs %" PRIu64 "\n", c, b);
        bad += b;
        total += c;
    }
    {  // special values
        uint64_t b = 0, c = 0;
        const double sp[] = {0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1e-310, -1e-310, 1e300, -1e300, INFINITY, -INFINITY, NAN, 1.0000000000000002,
                             -1.0000000000000002, 0x1p-1074, 0x1p-1022, 0.9999999999999999, -0.9999999999999999, 2.0, -2.0};
        for (double a : sp) {
            acos_chk(a, b);
            ++c;
            for (double d : sp) {
                atan2_chk(a, d, b);
                ++c;
            }
        }
        std::printf("special n=%" PRIu64 " differs %" PRIu64 "\n", c, b);
        bad += b;
        total += c;
    }
    {  // random doubles of every exponent
        uint64_t b = 0;
        for (uint64_t k = 0; k < n; ++k) {
            uint64_t bx = sm(s), by = sm(s);
            double x, y;
            std::memcpy(&x, &bx, 8);
            std::memcpy(&y, &by, 8);
            acos_chk(x, b);
            atan2_chk(y, x, b);
        }
        std::printf("random_doubles n=%" PRIu64 " differs %" PRIu64 "\n", 2 * n, b);
        bad += b;
        total += 2 * n;
    }
    std::printf("mismatches %" PRIu64 " of %" PRIu64 "\n", bad, total);
    return bad ? 1 : 0;
}
