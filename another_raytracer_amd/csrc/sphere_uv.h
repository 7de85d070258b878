// sphere_uv.h -- get_sphere_uv (sphere.h:24-37) for the device: acos and atan2 written out here, host and device the
// same code, instead of the device library's.
//
// The reference calls glibc's acos / atan2 (IBM Accurate Mathematical Library, glibc 2.35).  Those are not correctly
// rounded (tools/acos_atan2_cr.c against MPFR: 0.07 % / 0.09 % of unit-vector arguments differ from correct rounding),
// so no independent implementation reproduces their last bit, and restating IBM's table-driven code (asincos.tbl,
// uatan2.tbl, multi-precision fallbacks) from libm's machine code is out of proportion to what it buys: u, v only choose
// an image texel, int(u * W) / int((1 - v) * H) (texture.h:90-117), which a last-bit difference changes only for a
// normal within a few ulps of a texel edge (probability ~1e-12 per earth / capsule hit).
//
// What this header buys is control of the code.  The device library's acos / atan2 materialise ~30 f64 polynomial
// constants that the compiler hoists out of k_paths_g's path loop and spills to scratch at kernel start (the Next-Week
// final's kernel: 50+ spilled VGPRs).  Here the coefficients are read from a table the caller passes (device.h
// uv_table: a device copy of kUvCoefHost, or k_paths_g's LDS copy of it), so every use is a load inside the (rarely executed)
// u, v code: nothing is hoisted into the path loop's registers.  (A __constant__ table read through an opaque zero
// offset was r4's first form: its scalar loads were merged into 16-dword batches whose SGPRs spilled into VGPR lanes,
// ~300 v_readlane per evaluation.)  The algorithms are
// fdlibm 5.3's (Sun Microsystems; e_acos.c rational approximation, s_atan.c four-interval reduction, e_atan2.c
// quadrants), accurate to < 1 ulp, with one change: atan2 returns +-pio2_hi once |y / x| > 2^60 in every quadrant (the
// correct rounding, as glibc gives it; fdlibm is 1 ulp high for x < 0) -- tests/test_sphere_uv.py measures them against glibc and the texel choices they
// imply, and tools/uv_check.hip checks on the GPU that the device computes the host's bits.
#pragma once
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#define ART_UV_HD __host__ __device__
#else
#define ART_UV_HD
#endif

namespace art {

// fdlibm 5.3 constants (the decimal strings of e_acos.c / s_atan.c / e_atan2.c; each is the double the comment hex
// there names)
enum UvCoef : int {
    kPS0, kPS1, kPS2, kPS3, kPS4, kPS5, kQS1, kQS2, kQS3, kQS4,   // acos: R(x^2) = x^2 * P / Q
    kAT0, kAT1, kAT2, kAT3, kAT4, kAT5, kAT6, kAT7, kAT8, kAT9, kAT10,  // atan polynomial
    kAtanHi0, kAtanHi1, kAtanHi2, kAtanHi3, kAtanLo0, kAtanLo1, kAtanLo2, kAtanLo3,
    kPi, kPio2Hi, kPio2Lo, kPiLo, kOneHalf3, kTiny, kTwoPi, kUvCoefs
};
// (the last: sphere.h:36's 2 * pi; the reference's pi constant, tracer_utils.h, is kPi's double)
#define ART_UV_COEFS \
    1.66666666666666657415e-01, -3.25565818622400915405e-01, 2.01212532134862925881e-01, -4.00555345006794114027e-02, \
    7.91534994289814532176e-04, 3.47933107596021167570e-05, -2.40339491173441421878e+00, 2.02094576023350569471e+00, \
    -6.88283971605453293030e-01, 7.70381505559019352791e-02, \
    3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01, -1.11111104054623557880e-01, \
    9.09088713343650656196e-02, -7.69187620504482999495e-02, 6.66107313738753120669e-02, -5.83357013379057348645e-02, \
    4.97687799461593236017e-02, -3.65315727442169155270e-02, 1.62858201153657823623e-02, \
    4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01, 1.57079632679489655800e+00, \
    2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17, 6.12323399573676603587e-17, \
    3.14159265358979311600e+00, 1.57079632679489655800e+00, 6.12323399573676603587e-17, 1.2246467991473531772e-16, \
    1.5, 1.0e-300, \
    2.0 * 3.1415926535897932385
// The host's table; the device reads a copy of it (uploaded with the scene: device.h uv_table).
static const double kUvCoefHost[kUvCoefs] = {ART_UV_COEFS};
constexpr size_t kUvTableBytes = (sizeof(double) * kUvCoefs + 15u) & ~size_t(15);  // the copy's size, 16-B aligned
#undef ART_UV_COEFS

struct UvTab {
    const double* t;
    ART_UV_HD explicit UvTab(const double* p) : t(p) {}
    ART_UV_HD double operator[](int k) const { return t[k]; }
};

ART_UV_HD inline uint64_t uv_bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
ART_UV_HD inline double uv_from(uint64_t u) {
    double x;
    std::memcpy(&x, &u, 8);
    return x;
}
ART_UV_HD inline double uv_fabs(double x) { return uv_from(uv_bits(x) & 0x7FFFFFFFFFFFFFFFull); }  // -0 -> +0
// sqrt, correctly rounded on both sides (the device's sqrt_rn / sqrt give the same bits as the host's)
ART_UV_HD inline double uv_sqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_sqrt(x);
#else
    return __builtin_sqrt(x);
#endif
}

// fdlibm e_acos.c
ART_UV_HD inline double uv_acos(double x, const UvTab& c) {
    const uint64_t b = uv_bits(x);
    const int32_t hx = static_cast<int32_t>(b >> 32);
    const int32_t ix = hx & 0x7fffffff;
    const uint32_t lx = static_cast<uint32_t>(b);
    if (ix >= 0x3ff00000) {  // |x| >= 1
        if (((ix - 0x3ff00000) | lx) == 0) return hx > 0 ? 0.0 : c[kPi] + 2.0 * c[kPio2Lo];  // acos(1) = 0, acos(-1) = pi
        return (x - x) / (x - x);  // |x| > 1: NaN
    }
    if (ix < 0x3fe00000) {  // |x| < 0.5
        if (ix <= 0x3c600000) return c[kPio2Hi] + c[kPio2Lo];  // |x| < 2^-57
        const double z = x * x;
        const double p = z * (c[kPS0] + z * (c[kPS1] + z * (c[kPS2] + z * (c[kPS3] + z * (c[kPS4] + z * c[kPS5])))));
        const double q = 1.0 + z * (c[kQS1] + z * (c[kQS2] + z * (c[kQS3] + z * c[kQS4])));
        const double r = p / q;
        return c[kPio2Hi] - (x - (c[kPio2Lo] - x * r));
    }
    if (hx < 0) {  // x < -0.5
        const double z = (1.0 + x) * 0.5;
        const double p = z * (c[kPS0] + z * (c[kPS1] + z * (c[kPS2] + z * (c[kPS3] + z * (c[kPS4] + z * c[kPS5])))));
        const double q = 1.0 + z * (c[kQS1] + z * (c[kQS2] + z * (c[kQS3] + z * c[kQS4])));
        const double s = uv_sqrt(z);
        const double r = p / q;
        const double w = r * s - c[kPio2Lo];
        return c[kPi] - 2.0 * (s + w);
    }
    // x > 0.5
    const double z = (1.0 - x) * 0.5;
    const double s = uv_sqrt(z);
    const double df = uv_from(uv_bits(s) & 0xFFFFFFFF00000000ull);
    const double cc = (z - df * df) / (s + df);
    const double p = z * (c[kPS0] + z * (c[kPS1] + z * (c[kPS2] + z * (c[kPS3] + z * (c[kPS4] + z * c[kPS5])))));
    const double q = 1.0 + z * (c[kQS1] + z * (c[kQS2] + z * (c[kQS3] + z * c[kQS4])));
    const double r = p / q;
    const double w = r * s + cc;
    return 2.0 * (df + w);
}

// fdlibm s_atan.c for 0 <= x (atan2's |y / x|)
ART_UV_HD inline double uv_atan_pos(double x, const UvTab& c) {
    const int32_t ix = static_cast<int32_t>(uv_bits(x) >> 32) & 0x7fffffff;
    if (ix >= 0x44100000) {  // x >= 2^66
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && static_cast<uint32_t>(uv_bits(x)) != 0)) return x + x;  // NaN
        return c[kAtanHi3] + c[kAtanLo3];
    }
    int id;
    if (ix < 0x3fdc0000) {  // x < 0.4375
        if (ix < 0x3e200000) return x;  // x < 2^-29 (fdlibm: huge + x > one, raising inexact)
        id = -1;
    } else if (ix < 0x3ff30000) {  // x < 1.1875
        if (ix < 0x3fe60000) {  // 7/16 <= x < 11/16
            id = 0;
            x = (2.0 * x - 1.0) / (2.0 + x);
        } else {  // 11/16 <= x < 19/16
            id = 1;
            x = (x - 1.0) / (x + 1.0);
        }
    } else if (ix < 0x40038000) {  // x < 2.4375
        id = 2;
        x = (x - c[kOneHalf3]) / (1.0 + c[kOneHalf3] * x);
    } else {  // 2.4375 <= x < 2^66
        id = 3;
        x = -1.0 / x;
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (c[kAT0] + w * (c[kAT2] + w * (c[kAT4] + w * (c[kAT6] + w * (c[kAT8] + w * c[kAT10])))));
    const double s2 = w * (c[kAT1] + w * (c[kAT3] + w * (c[kAT5] + w * (c[kAT7] + w * c[kAT9]))));
    if (id < 0) return x - x * (s1 + s2);
    return c[kAtanHi0 + id] - ((x * (s1 + s2) - c[kAtanLo0 + id]) - x);
}

// fdlibm e_atan2.c (finite arguments: the components of a unit normal; inf / NaN handled as fdlibm does)
ART_UV_HD inline double uv_atan2(double y, double x, const UvTab& c) {
    const uint64_t bx = uv_bits(x), by = uv_bits(y);
    const int32_t hx = static_cast<int32_t>(bx >> 32), hy = static_cast<int32_t>(by >> 32);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const uint32_t lx = static_cast<uint32_t>(bx), ly = static_cast<uint32_t>(by);
    const double tiny = c[kTiny];
    if ((static_cast<uint32_t>(ix) | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || (static_cast<uint32_t>(iy) | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;  // NaN
    if (((hx - 0x3ff00000) | static_cast<int32_t>(lx)) == 0) {  // x = 1.0: atan(y)
        const double z = uv_atan_pos(uv_fabs(y), c);
        return hy < 0 ? -z : z;
    }
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  // 2 * sign(x) + sign(y)
    if ((static_cast<uint32_t>(iy) | ly) == 0) {  // y = 0
        switch (m) {
            case 0:
            case 1: return y;                   // atan(+-0, +anything) = +-0
            case 2: return c[kPi] + tiny;       // atan(+0, -anything) = pi
            default: return -c[kPi] - tiny;     // atan(-0, -anything) = -pi
        }
    }
    if ((static_cast<uint32_t>(ix) | lx) == 0) return hy < 0 ? -c[kPio2Hi] - tiny : c[kPio2Hi] + tiny;  // x = 0
    if (ix == 0x7ff00000) {  // x = +-inf
        if (iy == 0x7ff00000) {
            switch (m) {
                case 0: return c[kAtanHi1] + tiny;           // atan(+inf, +inf)
                case 1: return -c[kAtanHi1] - tiny;          // atan(-inf, +inf)
                case 2: return 3.0 * c[kAtanHi1] + tiny;     // atan(+inf, -inf)
                default: return -3.0 * c[kAtanHi1] - tiny;   // atan(-inf, -inf)
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return c[kPi] + tiny;
            default: return -c[kPi] - tiny;
        }
    }
    if (iy == 0x7ff00000) return hy < 0 ? -c[kPio2Hi] - tiny : c[kPio2Hi] + tiny;  // y = +-inf
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) {
        // |y / x| > 2^60: atan2 = +-pi/2 -+ x/y, within 0.004 ulp of pi/2, whose correct rounding is pio2_hi in every
        // quadrant (fdlibm's pi - (z - pi_lo) for x < 0 is 1 ulp above it; glibc rounds correctly)
        return hy < 0 ? -c[kPio2Hi] : c[kPio2Hi];
    } else if (hx < 0 && k < -60) {
        z = 0.0;  // |y| / x < -2^60
    } else {
        z = uv_atan_pos(uv_fabs(y / x), c);
    }
    switch (m) {
        case 0: return z;                                  // atan(+, +)
        case 1: return -z;                                 // atan(-, +) (fdlibm flips the sign bit)
        case 2: return c[kPi] - (z - c[kPiLo]);            // atan(+, -)
        default: return (z - c[kPiLo]) - c[kPi];           // atan(-, -)
    }
}

// get_sphere_uv (sphere.h:24-37) of an outward unit normal (ox, oy, oz): theta = acos(-y), phi = atan2(-z, x) + pi,
// u = phi / (2 pi), v = theta / pi -- the reference's operation order, pi = 3.1415926535897932385 (tracer_utils.h)
struct UvPair {
    double u, v;
};
// coef: the kUvCoefHost table or a copy of it
ART_UV_HD inline UvPair sphere_uv(double ox, double oy, double oz, const double* coef) {
    const UvTab c(coef);
    const double pi = c[kPi];  // 3.1415926535897932385 (tracer_utils.h) is this double
    const double theta = uv_acos(-oy, c);
    const double phi = uv_atan2(-oz, ox, c) + pi;
    return UvPair{phi / c[kTwoPi], theta / pi};
}
// host callers (tests, tools): the host table
inline double uv_acos(double x) { return uv_acos(x, UvTab(kUvCoefHost)); }
inline double uv_atan2(double y, double x) { return uv_atan2(y, x, UvTab(kUvCoefHost)); }
inline UvPair sphere_uv(double ox, double oy, double oz) { return sphere_uv(ox, oy, oz, kUvCoefHost); }

}  // namespace art
