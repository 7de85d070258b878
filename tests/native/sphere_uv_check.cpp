// csrc/sphere_uv.h (the device's get_sphere_uv: glibc_trig.h's restated acos / atan2) on the host against glibc's
// acos / atan2 (the reference's libm): ulp difference of each function, and u / v bits and texel choices (1024 x 512 earth texture,
// texture.h:90-117) over two sets of unit normals -- uniform directions, and directions placed on texel edges nudged
// by -4..+4 ulps per component (tools/uv_check.hip's sets).  Prints one line per set and a summary line.
#include <cinttypes>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "sphere_uv.h"

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(uint64_t& s) { return static_cast<double>(splitmix(s) >> 11) * 0x1p-53; }
static int64_t ord(double x) {
    int64_t i;
    std::memcpy(&i, &x, 8);
    return i < 0 ? INT64_MIN - i : i;
}
static void texel(double u, double v, int W, int H, int& i, int& j) {
    u = std::fmin(std::fmax(u, 0.0), 1.0);
    v = 1.0 - std::fmin(std::fmax(v, 0.0), 1.0);
    i = static_cast<int>(u * W);
    j = static_cast<int>(v * H);
    if (i >= W) i = W - 1;
    if (j >= H) j = H - 1;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? static_cast<uint32_t>(std::atol(argv[1])) : (1u << 22);
    const int W = 1024, H = 512;
    const double pi = 3.1415926535897932385;
    uint64_t s = 12345;
    int64_t max_acos = 0, max_atan2 = 0;
    for (int set = 0; set < 2; ++set) {
        uint64_t ubad = 0, vbad = 0, tbad = 0, acos_bad = 0, atan2_bad = 0;
        for (uint32_t k = 0; k < n; ++k) {
            double x, y, z;
            if (set == 0) {
                const double zc = 2.0 * u01(s) - 1.0, a = 2.0 * pi * u01(s), r = std::sqrt(std::fmax(0.0, 1.0 - zc * zc));
                x = r * std::cos(a);
                y = zc;
                z = r * std::sin(a);
            } else {
                if (k & 1) {
                    const double phi = 2.0 * pi * static_cast<double>(splitmix(s) % W) / W - pi, yy = 2.0 * u01(s) - 1.0,
                                 r = std::sqrt(1.0 - yy * yy);
                    x = r * std::cos(phi);
                    z = -r * std::sin(phi);
                    y = yy;
                } else {
                    const double theta = pi * static_cast<double>(splitmix(s) % (H + 1)) / H, a = 2.0 * pi * u01(s);
                    y = -std::cos(theta);
                    const double r = std::sin(theta);
                    x = r * std::cos(a);
                    z = r * std::sin(a);
                }
                auto nudge = [&](double v) {
                    int d = static_cast<int>(splitmix(s) % 9) - 4;
                    for (; d > 0; --d) v = std::nextafter(v, INFINITY);
                    for (; d < 0; ++d) v = std::nextafter(v, -INFINITY);
                    return v;
                };
                x = nudge(x);
                y = nudge(y);
                z = nudge(z);
            }
            const double ga = std::acos(-y), gt = std::atan2(-z, x);
            const double ma = art::glibc_acos(-y), mt = art::glibc_atan2(-z, x);
            // bit for bit, NaN (a nudged component just past +-1) included
            const int64_t ea = std::memcmp(&ga, &ma, 8) == 0 ? 0 : std::isnan(ga) || std::isnan(ma) ? INT64_MAX : std::llabs(ord(ga) - ord(ma));
            const int64_t et = std::memcmp(&gt, &mt, 8) == 0 ? 0 : std::isnan(gt) || std::isnan(mt) ? INT64_MAX : std::llabs(ord(gt) - ord(mt));
            max_acos = ea > max_acos ? ea : max_acos;
            max_atan2 = et > max_atan2 ? et : max_atan2;
            acos_bad += ea != 0;
            atan2_bad += et != 0;
            const double u0 = (gt + pi) / (2.0 * pi), v0 = ga / pi;
            double u1, v1;
            const art::UvPair w1 = art::sphere_uv(x, y, z);
            u1 = w1.u;
            v1 = w1.v;
            ubad += std::memcmp(&u0, &u1, 8) != 0;
            vbad += std::memcmp(&v0, &v1, 8) != 0;
            int i0, j0, i1, j1;
            texel(u0, v0, W, H, i0, j0);
            texel(u1, v1, W, H, i1, j1);
            tbad += (i0 != i1 || j0 != j1);
        }
        std::printf("%s n=%u acos_differs %" PRIu64 " atan2_differs %" PRIu64 " u_bits_differ %" PRIu64 " v_bits_differ %" PRIu64
                    " texel_differs %" PRIu64 "\n",
                    set == 0 ? "random" : "adversarial", n, acos_bad, atan2_bad, ubad, vbad, tbad);
    }
    // the exact cases (each pair's result is correctly rounded by both): poles, quadrant boundaries, signed zeros,
    // infinities, |y / x| beyond 2^60 either way
    const double sp[] = {0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1e-300, -1e-300, 1e300, -1e300, INFINITY, -INFINITY};
    uint64_t special_bad = 0, special_n = 0;
    for (double a : sp) {
        ++special_n;
        if (std::fabs(a) <= 1.0) {
            const double g = std::acos(a), m = art::glibc_acos(a);
            special_bad += std::memcmp(&g, &m, 8) != 0;
        }
        for (double b : sp) {
            const double g = std::atan2(a, b), m = art::glibc_atan2(a, b);
            special_bad += std::memcmp(&g, &m, 8) != 0;
            ++special_n;
        }
    }
    std::printf("special n=%" PRIu64 " differs %" PRIu64 "\n", special_n, special_bad);
    std::printf("max_ulp acos %" PRId64 " atan2 %" PRId64 "\n", max_acos, max_atan2);
    return 0;
}
