// layout.h's 16-bit child codes (BvhNode::pad, the packed-key traversal of k_paths_g F_CODE16 kernels): every leaf
// (first < 8192, count 1..4) that leaf16_ok accepts round-trips through make_leaf16 / leaf16_first / leaf16_count, is a
// negative int16 below kNodeEmpty (so `code < kNodeEmpty` marks a leaf and inner indices 0..32767 stay apart), and
// kNodeEmpty decodes as an empty range.  Prints "ok <n>" or the first failure.
#include <cstdint>
#include <cstdio>

#include "layout.h"

using namespace art;

int main() {
    long n = 0;
    for (uint32_t count = 0; count <= 8; ++count)
        for (uint32_t first = 0; first < 9000; ++first) {
            const bool ok = leaf16_ok(first, count);
            const bool expect = count >= 1 && count <= 4 && first < 8192 && !(count == 4 && first == 8191);
            if (ok != expect) {
                std::printf("leaf16_ok(%u, %u) = %d\n", first, count, ok);
                return 1;
            }
            if (!ok) continue;
            const int32_t c = make_leaf16(first, count);
            if (c >= kNodeEmpty || c < -32768 || static_cast<int16_t>(c) != c || leaf16_first(c) != first || leaf16_count(c) != count) {
                std::printf("leaf (%u, %u) -> %d -> (%u, %u)\n", first, count, c, leaf16_first(c), leaf16_count(c));
                return 1;
            }
            ++n;
        }
    if (leaf16_count(kNodeEmpty) != 0) {
        std::printf("kNodeEmpty decodes with count %u\n", leaf16_count(kNodeEmpty));
        return 1;
    }
    std::printf("ok %ld\n", n);
    return 0;
}
