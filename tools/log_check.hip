// tools/log_check.hip — does a device log agree with the host's (glibc) on every argument the renderer can pass it?
// constant_medium::hit (constant_medium.h:61) takes log(random_double()); under the product's RNG contract a uniform
// is k * 2^-24 with k < 2^24, so its 2^24 possible arguments can be checked exhaustively.  Two device functions:
// the device library's log (OCML: expected to differ for some k) and art::glibc_log (csrc/glibc_log.h, the one
// hit_medium uses: must differ for none).  Prints one JSON line; writes the OCML exceptions (k, device bits, glibc
// bits) to the file named by argv[1].  Exit status 1 if glibc_log differs anywhere.
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -Ianother_raytracer_amd/csrc tools/log_check.hip -o tools/log_check
//   ./tools/log_check gpurun_out/log_exceptions.txt
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "glibc_log.h"

__global__ void k_log(double* ocml, double* restated, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double x = static_cast<double>(k) * 0x1p-24;  // the uniform<double> value of the kernels (device.h)
    ocml[k] = log(x);
    restated[k] = art::glibc_log(x);
}

int main(int argc, char** argv) {
    const uint32_t n = 1u << 24;
    double* d = nullptr;
    if (hipMalloc(&d, 2 * sizeof(double) * n) != hipSuccess) return 2;
    hipLaunchKernelGGL(k_log, dim3(n / 256), dim3(256), 0, 0, d, d + n, n);
    std::vector<double> h(2 * size_t(n));
    if (hipMemcpy(h.data(), d, 2 * sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    FILE* f = argc > 1 ? std::fopen(argv[1], "w") : nullptr;
    uint64_t bad_ocml = 0, bad_restated = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const double ref = std::log(static_cast<double>(k) * 0x1p-24);
        const uint64_t a = art::f64_bits(h[k]), b = art::f64_bits(ref), c = art::f64_bits(h[n + k]);
        if (a != b) {
            ++bad_ocml;
            if (f) std::fprintf(f, "%u %016llx %016llx\n", k, static_cast<unsigned long long>(a), static_cast<unsigned long long>(b));
        }
        bad_restated += c != b;
    }
    if (f) std::fclose(f);
    std::printf("{\"arguments\": %u, \"ocml_log_mismatches\": %llu, \"glibc_log_restated_mismatches\": %llu}\n", n,
                static_cast<unsigned long long>(bad_ocml), static_cast<unsigned long long>(bad_restated));
    return bad_restated ? 1 : 0;
}
