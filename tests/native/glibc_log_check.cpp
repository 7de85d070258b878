// Host check of csrc/glibc_log.h against the C library's log (tests/test_glibc_log.py builds and runs it):
// every uniform a draw can give (k * 2^-24, k < 2^24), then N random positive normal doubles (all exponents).
// Prints "mismatches <m> of <n>" and the first few differing inputs; exit status 1 if any.
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "glibc_log.h"

int main(int argc, char** argv) {
    const uint64_t extra = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
    uint64_t bad = 0, n = 0;
    auto check = [&](double x) {
        const double a = art::glibc_log(x), b = std::log(x);
        ++n;
        if (art::f64_bits(a) != art::f64_bits(b)) {
            if (bad < 5) std::printf("x %a: restated %a, libm %a\n", x, a, b);
            ++bad;
        }
    };
    for (uint32_t k = 0; k < (1u << 24); ++k) check(static_cast<double>(k) * 0x1p-24);
    uint64_t s = 0x9e3779b97f4a7c15ull;
    for (uint64_t j = 0; j < extra; ++j) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        const uint64_t e = 1 + (s >> 33) % 2046;  // normal exponents
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        check(art::f64_from((e << 52) | (s >> 12)));
    }
    std::printf("mismatches %" PRIu64 " of %" PRIu64 "\n", bad, n);
    return bad ? 1 : 0;
}
