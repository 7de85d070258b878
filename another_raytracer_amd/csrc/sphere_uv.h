// sphere_uv.h -- get_sphere_uv (sphere.h:24-37) for host and device: theta = acos(-y), phi = atan2(-z, x) + pi,
// u = phi / (2 pi), v = theta / pi, with glibc 2.35's acos and atan2 restated operation by operation (glibc_trig.h),
// so the u, v bits -- and the image texel int(u * W), int((1 - v) * H) they choose (texture.h:90-117) -- are the
// reference's.
//
// The data (constants and tables) is read through a TrigTab the caller passes: on the device the copy uploaded with
// the scene in front of the image records (device.h uv_table), its constants possibly from k_paths_g's LDS copy.  A
// table read at each use keeps the constants out of the path loop's registers: the device library's acos / atan2
// materialise ~30 f64 literals that the compiler hoisted out of k_paths_g's loop and spilled (the Next-Week final's
// kernel: 54 spilled VGPRs), and a __constant__ table's scalar loads were merged into 16-dword batches that spilled
// SGPRs (~300 v_readlane).  r4's interim fdlibm version differed from glibc in the last bit for ~8 % of normals and
// chose another texel for 2.5 % of normals placed on texel edges; this one equals glibc on every argument tested
// (tests/test_glibc_trig.py, tests/test_sphere_uv.py on the host; tools/uv_check.hip on the GPU).
#pragma once
#include <cstddef>
#include <cstdint>

#include "glibc_trig.h"

namespace art {

// the device copy of glibc_trig_data::kTrigHost (device.h uv_table): its size in bytes, 16-B aligned
constexpr size_t kUvTableBytes = (sizeof(double) * glibc_trig_data::kTrigDoubles + 15u) & ~size_t(15);
// the leading constants alone (k_paths_g's LDS copy), 16-B aligned
constexpr int kUvConsts = glibc_trig_data::kNumConsts;
constexpr size_t kUvConstBytes = (sizeof(double) * kUvConsts + 15u) & ~size_t(15);

struct UvPair {
    double u, v;
};
ART_TRIG_HD inline UvPair sphere_uv(double ox, double oy, double oz, const TrigTab& g) {
    const double pi = g.c[glibc_trig_data::kPi];  // 3.1415926535897932385 (tracer_utils.h) is this double
    const double theta = glibc_acos(-oy, g);
    const double phi = glibc_atan2(-oz, ox, g) + pi;
    return UvPair{phi / (pi + pi), theta / pi};  // pi + pi: sphere.h:36's 2 * pi, exactly
}
// host callers (tests, tools): the host tables
inline UvPair sphere_uv(double ox, double oy, double oz) {
    return sphere_uv(ox, oy, oz, TrigTab(glibc_trig_data::kTrigHost, glibc_trig_data::kTrigHost));
}

}  // namespace art
