// tools/uv_check.hip — the device's get_sphere_uv (sphere.h:24-37; csrc/sphere_uv.h, glibc's acos / atan2 restated in
// glibc_trig.h, the code k_paths / k_paths_g run): does the device compute the host build's bits, and are they glibc's
// (the reference's libm)?  Both must hold exactly.  The image texture reads texel (int(clamp(u) * W),
// int((1 - clamp(v)) * H)) (texture.h:67-118), so a last-bit difference in u or v would move a lookup when u * W or
// (1 - v) * H lies within a few ulps of an integer; the second set is built to sit there.  Two sets, 2^24 unit vectors each:
//   random       uniform directions (a splitmix64 stream), as hit normals (p - c) / r spread over a sphere;
//   adversarial  directions placed on the texel boundaries of the earth texture (1024 x 512, scene_manager.cpp:117,
//                the final scene's earth): u = k / 1024 and v = 1 - j / 512, each nudged by -4..+4 ulps per component.
// Prints one JSON line: per set, normals whose u or v bits differ from glibc's, normals whose texel differs, and
// normals whose device bits differ from the host's sphere_uv (all expected 0).
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -Ianother_raytracer_amd/csrc tools/uv_check.hip -o tools/uv_check
#include <hip/hip_runtime.h>

#include "sphere_uv.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_uv(const double* n, double* uv, uint32_t count, const double* tab) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    double u, v;
    const art::UvPair w = art::sphere_uv(n[3 * k], n[3 * k + 1], n[3 * k + 2], art::TrigTab(tab, tab));  // device.h prim_surface's call
    u = w.u;
    v = w.v;
    uv[2 * k] = u;
    uv[2 * k + 1] = v;
}

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(uint64_t& s) { return static_cast<double>(splitmix(s) >> 11) * 0x1p-53; }
static uint64_t bits(double d) {
    uint64_t b;
    std::memcpy(&b, &d, 8);
    return b;
}
static void texel(double u, double v, int W, int H, int& i, int& j) {  // texture.h:67-118
    u = std::fmin(std::fmax(u, 0.0), 1.0);
    v = 1.0 - std::fmin(std::fmax(v, 0.0), 1.0);
    i = static_cast<int>(u * W);
    j = static_cast<int>(v * H);
    if (i >= W) i = W - 1;
    if (j >= H) j = H - 1;
}

int main() {
    const uint32_t n = 1u << 24;
    const int W = 1024, H = 512;
    const double pi = 3.1415926535897932385;
    std::vector<double> sets[2];
    uint64_t s = 12345;
    for (auto& v : sets) v.resize(3 * size_t(n));
    for (uint32_t k = 0; k < n; ++k) {  // uniform directions
        const double zc = 2.0 * u01(s) - 1.0, a = 2.0 * pi * u01(s), r = std::sqrt(std::fmax(0.0, 1.0 - zc * zc));
        sets[0][3 * k] = r * std::cos(a);
        sets[0][3 * k + 1] = zc;
        sets[0][3 * k + 2] = r * std::sin(a);
    }
    for (uint32_t k = 0; k < n; ++k) {  // texel boundaries, nudged
        double x, y, z;
        if (k & 1) {  // a u boundary: phi = 2 pi i / W, i.e. atan2(-z, x) = phi - pi
            const double phi = 2.0 * pi * static_cast<double>(splitmix(s) % W) / W - pi, yy = 2.0 * u01(s) - 1.0,
                         r = std::sqrt(1.0 - yy * yy);
            x = r * std::cos(phi);
            z = -r * std::sin(phi);
            y = yy;
        } else {  // a v boundary: theta = pi j / H, i.e. -y = cos(theta)
            const double theta = pi * static_cast<double>(splitmix(s) % (H + 1)) / H, a = 2.0 * pi * u01(s);
            y = -std::cos(theta);
            const double r = std::sin(theta);
            x = r * std::cos(a);
            z = r * std::sin(a);
        }
        const int dx = static_cast<int>(splitmix(s) % 9) - 4, dy = static_cast<int>(splitmix(s) % 9) - 4, dz = static_cast<int>(splitmix(s) % 9) - 4;
        auto nudge = [](double v, int d) {
            for (; d > 0; --d) v = std::nextafter(v, INFINITY);
            for (; d < 0; ++d) v = std::nextafter(v, -INFINITY);
            return v;
        };
        sets[1][3 * k] = nudge(x, dx);
        sets[1][3 * k + 1] = nudge(y, dy);
        sets[1][3 * k + 2] = nudge(z, dz);
    }
    double *dn = nullptr, *duv = nullptr;
    double* dtab = nullptr;
    if (hipMalloc(&dn, sizeof(double) * 3 * n) != hipSuccess || hipMalloc(&duv, sizeof(double) * 2 * n) != hipSuccess ||
        hipMalloc(&dtab, sizeof(art::glibc_trig_data::kTrigHost)) != hipSuccess)
        return 2;
    if (hipMemcpy(dtab, art::glibc_trig_data::kTrigHost, sizeof(art::glibc_trig_data::kTrigHost), hipMemcpyHostToDevice) != hipSuccess) return 2;
    std::vector<double> uv(2 * size_t(n));
    const char* names[2] = {"random", "adversarial"};
    std::printf("{\"normals_per_set\": %u, \"texture\": [%d, %d]", n, W, H);
    for (int t = 0; t < 2; ++t) {
        if (hipMemcpy(dn, sets[t].data(), sizeof(double) * 3 * n, hipMemcpyHostToDevice) != hipSuccess) return 2;
        hipLaunchKernelGGL(k_uv, dim3(n / 256), dim3(256), 0, 0, dn, duv, n, dtab);
        if (hipMemcpy(uv.data(), duv, sizeof(double) * 2 * n, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        uint64_t ubad = 0, vbad = 0, tbad = 0, hbad = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const double x = sets[t][3 * k], y = sets[t][3 * k + 1], z = sets[t][3 * k + 2];
            const double theta = std::acos(-y), phi = std::atan2(-z, x) + pi;  // glibc: the reference's libm
            const double u = phi / (2.0 * pi), v = theta / pi;
            ubad += bits(u) != bits(uv[2 * k]);
            vbad += bits(v) != bits(uv[2 * k + 1]);
            int i0, j0, i1, j1;
            texel(u, v, W, H, i0, j0);
            texel(uv[2 * k], uv[2 * k + 1], W, H, i1, j1);
            tbad += (i0 != i1 || j0 != j1);
            double hu, hv;
            const art::UvPair hw = art::sphere_uv(x, y, z);
            hu = hw.u;
            hv = hw.v;
            hbad += bits(hu) != bits(uv[2 * k]) || bits(hv) != bits(uv[2 * k + 1]);
        }
        std::printf(", \"%s\": {\"u_bits_differ\": %llu, \"v_bits_differ\": %llu, \"texel_differs\": %llu, \"device_vs_host\": %llu}", names[t],
                    static_cast<unsigned long long>(ubad), static_cast<unsigned long long>(vbad), static_cast<unsigned long long>(tbad),
                    static_cast<unsigned long long>(hbad));
    }
    std::printf("}\n");
    return 0;
}
