// glibc_log.h — the C library's log as the reference calls it, restated operation by operation so that the device
// returns the same bits.
//
// constant_medium.h:61 takes log(random_double()) from glibc (2.35 in this image).  On x86-64 CPUs with FMA and AVX2
// glibc's ifunc selects the FMA build of sysdeps/ieee754/dbl-64/e_log.c (the table + polynomial algorithm of ARM's
// optimized-routines): the sequence below is that build's machine code read back instruction for instruction —
// which products are fused and which are rounded separately, in its order — with its data (glibc_log_data.h,
// generated from libm.so.6 by tools/gen_glibc_log.py).  The device's own log (OCML) differs from it in the last bit
// for 445 762 of the 2^24 values a uniform draw takes; this function equals glibc's for all of them
// (tests/test_glibc_log.py compares every one on the host; tools/log_check on the GPU).
//
// Domain: +0 and positive normal doubles (a uniform draw is k * 2^-24, k < 2^24).  Host and device.
#pragma once
#include <cstdint>
#include <cstring>

#include "glibc_log_data.h"

#if defined(__HIPCC__)
#define ART_LOG_HD __host__ __device__
#else
#define ART_LOG_HD
#endif

namespace art {

ART_LOG_HD inline uint64_t f64_bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, sizeof u);
    return u;
}
ART_LOG_HD inline double f64_from(uint64_t u) {
    double x;
    std::memcpy(&x, &u, sizeof x);
    return x;
}

ART_LOG_HD inline double glibc_log(double x) {
    using namespace glibc_log_data;
    const uint64_t ix = f64_bits(x);
    if (ix - 0x3fee000000000000ull < 0x3090000000000ull) {  // 1 - 2^-4 <= x < 1 + 0x1.09p-4: the near-1 polynomial
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double r = x - 1.0;
        const double r2 = r * r;
        const double r3 = r * r2;
        const double p0 = __builtin_fma(r2, kB[3], __builtin_fma(r, kB[2], kB[1]));
        const double p1 = __builtin_fma(r2, kB[6], __builtin_fma(r, kB[5], kB[4]));
        double p2 = __builtin_fma(r2, kB[9], __builtin_fma(r, kB[8], kB[7]));
        p2 = __builtin_fma(r3, kB[10], p2);
        const double p = __builtin_fma(__builtin_fma(p2, r3, p1), r3, p0);
        // r split into rhi (top 26 bits) + rlo for the exact B0 * r^2 term
        const double rw = __builtin_fma(r, 0x1p27, r);
        const double rhi = __builtin_fma(-0x1p27, r, rw);
        const double rlo = r - rhi;
        const double rhi2 = rhi * rhi;
        const double hi = __builtin_fma(rhi2, kB[0], r);
        const double lo = __builtin_fma(kB[0] * rlo, r + rhi, __builtin_fma(rhi2, kB[0], r - hi));
        return hi + __builtin_fma(p, r3, lo);
    }
    if ((ix >> 48) - 0x10u >= 0x7ff0u - 0x10u) return ix == 0 ? -__builtin_inf() : __builtin_nan("");  // outside the domain
    // x = 2^k z, z in [0x1.6p-1, 0x1.6p0); c ~ z from the 128-entry table, log x = k ln2 + log c + log(z / c)
    const uint64_t tmp = ix - 0x3fe6000000000000ull;
    const uint32_t i = static_cast<uint32_t>(tmp >> 45) & 127u;
    const double kd = static_cast<double>(static_cast<int32_t>(static_cast<int64_t>(tmp) >> 52));
    const double z = f64_from(ix - (tmp & 0xfff0000000000000ull));
    const double invc = kTab[2 * i], logc = kTab[2 * i + 1];
    const double r = __builtin_fma(z, invc, -1.0);
    const double w = __builtin_fma(kd, kLn2hi, logc);
    const double a12 = __builtin_fma(r, kA[2], kA[1]);
    const double hi = r + w;
    const double r2 = r * r;
    const double lo = __builtin_fma(kd, kLn2lo, (w - hi) + r);
    const double a34 = __builtin_fma(r, kA[4], kA[3]);
    const double y = __builtin_fma(r * r2, __builtin_fma(a34, r2, a12), __builtin_fma(r2, kA[0], lo));
    return y + hi;
}

}  // namespace art
