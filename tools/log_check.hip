// tools/log_check.hip — does the device's f64 log agree with the host's (glibc) on every argument the renderer can
// pass it?  constant_medium::hit (constant_medium.h:61) takes log(random_double()); under the product's RNG contract
// a uniform is k * 2^-24 with k < 2^24, so its 2^24 possible arguments can be checked exhaustively.  Prints the number
// of k where the bits differ and writes them (k, device bits, glibc bits) to the file named by argv[1].
//   hipcc -O3 --offload-arch=gfx950 tools/log_check.hip -o tools/log_check && ./tools/log_check gpurun_out/log_exceptions.txt
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void k_log(double* out, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    out[k] = log(static_cast<double>(k) * (1.0 / 16777216.0));  // the uniform<double> value of kernels (device.h)
}

int main(int argc, char** argv) {
    const uint32_t n = 1u << 24;
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * n) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_log, dim3(n / 256), dim3(256), 0, 0, d, n);
    std::vector<double> h(n);
    if (hipMemcpy(h.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    FILE* f = argc > 1 ? std::fopen(argv[1], "w") : nullptr;
    uint64_t bad = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const double ref = std::log(static_cast<double>(k) * (1.0 / 16777216.0));
        uint64_t a, b;
        std::memcpy(&a, &h[k], 8);
        std::memcpy(&b, &ref, 8);
        if (a != b) {
            ++bad;
            if (f) std::fprintf(f, "%u %016llx %016llx\n", k, static_cast<unsigned long long>(a), static_cast<unsigned long long>(b));
        }
    }
    if (f) std::fclose(f);
    std::printf("{\"arguments\": %u, \"log_mismatches\": %llu}\n", n, static_cast<unsigned long long>(bad));
    return 0;
}
