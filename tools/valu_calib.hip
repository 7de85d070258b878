// tools/valu_calib.hip — issue-cost calibration of the VALU instruction classes k_paths uses, on gfx950.
//
// Why: the PMC summary of k_paths has to turn per-type instruction counts (SQ_INSTS_VALU_*) into SIMD issue cycles,
// and the SQ counters' units (instructions vs quad-cycles) must be pinned on a kernel whose instruction stream is
// known.  Each op kernel runs, per lane, kIters iterations of kChains independent dependency chains of ONE
// instruction (inline asm, so the compiler cannot change it), at 1, 4 and 8 waves per SIMD (256- and 1024-lane
// blocks, one or two blocks per CU; k_paths runs 4).  Lane 0 of every wave stamps s_memtime (shader clock) and s_memrealtime
// (100 MHz) around the loop; the host reports
//   cycles per wave-instruction per SIMD = median(dclk) / (instructions per wave x waves per SIMD)
// and the in-kernel clock.  Run under `rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU ...` to read what each
// counter reports for a known stream (every kernel name carries its op).
//   hipcc -O3 --offload-arch=gfx950 tools/valu_calib.hip -o tools/valu_calib && ./tools/valu_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

constexpr int kChains = 8;
constexpr int kIters = 4096;

enum Op { FMA_F32, PK_FMA_F32, FMA_F64, ADD_F64, MUL_F64, MAX_U32, MAD_U64_U32, MUL_LO_U32, CNDMASK, RCP_F32, RSQ_F64,
          SQRT_F32, CVT_F32_F64, MIXED_F32_F64, kNumOps };
static const char* kNames[kNumOps] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_max_u32",
                                      "v_mad_u64_u32", "v_mul_lo_u32", "v_cndmask_b32", "v_rcp_f32", "v_rsq_f64",
                                      "v_sqrt_f32", "v_cvt_f32_f64", "f32+f64 fma (1:1)"};

template <int OP>
__global__ void k_calib(float* sink, unsigned long long* stamps, float seed) {
    float a[kChains];
    double d[kChains];
    unsigned u[kChains];
    unsigned long long w[kChains];
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p[kChains];
    for (int c = 0; c < kChains; ++c) {
        a[c] = seed + threadIdx.x * 1e-7f + c;
        d[c] = a[c];
        u[c] = threadIdx.x + c;
        w[c] = u[c];
        p[c] = f2{a[c], a[c] + 1.0f};
    }
    const float m = 0.999f, b = 1e-7f;
    const double dm = 0.999, db = 1e-7;
    const f2 pm = {m, m}, pb = {b, b};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            if constexpr (OP == FMA_F32) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[c]) : "v"(m), "v"(b));
            if constexpr (OP == PK_FMA_F32) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[c]) : "v"(pm), "v"(pb));
            if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[c]) : "v"(dm), "v"(db));
            if constexpr (OP == ADD_F64) asm volatile("v_add_f64 %0, %1, %0" : "+v"(d[c]) : "v"(db));
            if constexpr (OP == MUL_F64) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(d[c]) : "v"(dm));
            if constexpr (OP == MAX_U32) asm volatile("v_max_u32 %0, %1, %0" : "+v"(u[c]) : "v"(u[(c + 1) % kChains]));
            if constexpr (OP == MAD_U64_U32) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(w[c]) : "v"(u[c]) : "s0", "s1");
            if constexpr (OP == MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[c]) : "v"(u[(c + 3) % kChains]));
            if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(u[(c + 1) % kChains]) : "vcc");
            if constexpr (OP == RCP_F32) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[c]));
            if constexpr (OP == RSQ_F64) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[c]));
            if constexpr (OP == SQRT_F32) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[c]));
            if constexpr (OP == CVT_F32_F64) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a[c]) : "v"(d[c]));
            if constexpr (OP == MIXED_F32_F64) {
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[c]) : "v"(m), "v"(b));
                asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[c]) : "v"(dm), "v"(db));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0;
    for (int c = 0; c < kChains; ++c) s += a[c] + static_cast<float>(d[c]) + static_cast<float>(u[c]) + static_cast<float>(w[c]) + p[c].x + p[c].y;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        stamps[2 * wave] = t1 - t0;
        stamps[2 * wave + 1] = r1 - r0;
    }
}

// blocks_per_cu = 2 with 1024-lane blocks: 8 waves per SIMD (the kernel's few registers let two blocks share a CU)
template <int OP>
static void run(int cus, int block, float* sink, unsigned long long* stamps, int blocks_per_cu = 1) {
    const int waves = cus * blocks_per_cu * block / 64;
    hipLaunchKernelGGL(k_calib<OP>, dim3(cus * blocks_per_cu), dim3(block), 0, 0, sink, stamps, 1.0f);  // warm
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_calib<OP>, dim3(cus * blocks_per_cu), dim3(block), 0, 0, sink, stamps, 1.0f);
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    std::vector<unsigned long long> h(2 * waves);
    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> clk(waves), ghz(waves);
    for (int i = 0; i < waves; ++i) {
        clk[i] = static_cast<double>(h[2 * i]);
        ghz[i] = h[2 * i] / (h[2 * i + 1] * 10.0);  // memrealtime ticks at 100 MHz
    }
    std::sort(clk.begin(), clk.end());
    std::sort(ghz.begin(), ghz.end());
    const int per_op = (OP == MIXED_F32_F64) ? 2 : 1;
    const double insts = static_cast<double>(kIters) * kChains * per_op;  // wave-instructions per wave
    const double wps = blocks_per_cu * block / 256.0;                      // waves per SIMD
    // wall-clock cross-check: launch time x in-kernel clock over the SIMD's whole stream (catches blocks that were
    // not co-resident, which the per-wave stamps cannot see)
    const double wall_cyc = ms * 1e-3 * ghz[waves / 2] * 1e9 / (insts * wps);
    std::printf("{\"op\": \"%s\", \"waves_per_simd\": %g, \"cycles_per_inst_per_simd\": %.3f, \"clock_ghz\": %.3f, \"wall_cycles_per_inst_per_simd\": %.3f}\n",
                kNames[OP], wps, clk[waves / 2] / (insts * wps), ghz[waves / 2], wall_cyc);
}

template <int OP>
static void run_all(int cus, float* sink, unsigned long long* stamps) {
    run<OP>(cus, 256, sink, stamps);
    run<OP>(cus, 1024, sink, stamps);
    run<OP>(cus, 1024, sink, stamps, 2);
    if constexpr (OP + 1 < kNumOps) run_all<OP + 1>(cus, sink, stamps);
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float* sink;
    unsigned long long* stamps;
    CK(hipMalloc(&sink, sizeof(float) * cus * 2048));
    CK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * cus * 32));
    std::printf("{\"cus\": %d, \"chains\": %d, \"iters\": %d}\n", cus, kChains, kIters);
    run_all<0>(cus, sink, stamps);
    CK(hipFree(sink));
    CK(hipFree(stamps));
    return 0;
}
