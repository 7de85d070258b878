// pass_plan.h -- how a pass's path slots are handed out to the persistent kernels' waves (host side; g++ and hipcc).
#pragma once
#include <cstdint>

namespace art {

// The chunk (PassGeom::chunk, path_chunk on the host) is a power of two in [64, 2048], at most the pass's slots / 64
// claims per wave of a full CU.  The counter is one word every wave of the chip claims from: at 256 slots per claim
// k_paths took ~67 M claims/s, and each claim stalls its wave for the device-scope atomic's round trip.  Against 256
// (r4r_ab_path_chunk.txt): C2 +2.9 %, cow +3.2 %, the final +1.2 %, dino +1.2 %.  Larger chunks leave longer tails at
// the end of a pass: at 0.27-0.54 G slots per pass k_paths_g was fastest at 1024 (2048: -1 to -2.6 %, 4096: -3 to
// -8 %), at the configs' 1.1-1.7 G at 2048 (cow +0.9 % over 1024, the final +-0); k_paths (C2, 2.1 G) +-0 from 2048
// to 4096.  Claiming the next chunk one chunk ahead lost 1.5-2 % (its return is waited for at the loop's next vmcnt
// wait).  Small passes (pixel lists, small frames) keep at least 64 claims per wave.
constexpr uint32_t path_chunk(uint32_t P, int num_cu) {
    const uint64_t per = static_cast<uint64_t>(P) / (static_cast<uint64_t>(num_cu > 0 ? num_cu : 1) * 16u * 64u);
    uint32_t c = 64;
    while (c < 2048u && 2ull * c <= per) c *= 2;
    return c;
}

}  // namespace art
