// pass_plan.h's path_chunk (the slots a persistent kernel's wave claims per atomic): the values at the BASELINE
// configs' pass sizes, and its invariants over a sweep of pass sizes and CU counts.  Prints "ok" or the first failure.
#include <cstdint>
#include <cstdio>
#include <initializer_list>

#include "pass_plan.h"

static int fail(const char* what, uint64_t P, int cu, uint32_t c) {
    std::printf("FAIL %s P=%llu cu=%d chunk=%u\n", what, static_cast<unsigned long long>(P), cu, c);
    return 1;
}

int main() {
    // configs at 256 CUs: C2 1920x1080 (2 073 600 padded pixels) x 1024 spp in one pass, C3 x 512, C4/C5 passes of
    // ~1-2 G slots, and the 0.54 G pass of a 256-spp frame (1024: smaller chunks won at that size)
    struct Case { uint64_t P; uint32_t want; } cases[] = {
        {2073600ull * 1024, 2048}, {2073600ull * 512, 2048}, {2073600ull * 256, 1024}, {16777216ull * 128, 2048},
        {320ull * 192 * 4, 64}, {0, 64}, {1, 64}};
    for (const Case& k : cases) {
        const uint32_t c = art::path_chunk(static_cast<uint32_t>(k.P), 256);
        if (c != k.want) return fail("config value", k.P, 256, c);
    }
    for (int cu : {1, 8, 64, 256, 304}) {
        uint32_t prev = 0;
        for (uint64_t P = 1; P < (1ull << 31); P = P * 3 / 2 + 1) {
            const uint32_t c = art::path_chunk(static_cast<uint32_t>(P), cu);
            if (c < 64 || c > 2048 || (c & (c - 1)) != 0) return fail("power of two in [64, 2048]", P, cu, c);
            if (c < prev) return fail("monotone in P", P, cu, c);
            if (c > 64 && static_cast<uint64_t>(c) * cu * 16u * 64u > P) return fail("at least 64 claims per wave", P, cu, c);
            prev = c;
        }
    }
    std::printf("ok\n");
    return 0;
}
