// Host-side check of the launch grid cap (mpich_amd/csrc/redop_dispatch.h):
// grid_for never asks HIP for more than UINT32_MAX work-items in one
// dispatch, whatever the block size, and below the cap it still covers the
// work (one block per `work` units).  Built with g++ by tests/test_grid_cap.py.
#include "redop_dispatch.h"

#include <stdint.h>
#include <stdio.h>

using mpix::grid_for;
using mpix::max_blocks;

static int fails = 0;

static void check(uint64_t work, uint64_t n, int max_grid, uint64_t block)
{
    const uint64_t g = grid_for(work, n, max_grid, block);
    const uint64_t want = n ? (n + work - 1) / work : 1;
    uint64_t expect = want;
    if (max_grid > 0 && expect > (uint64_t) max_grid)
        expect = (uint64_t) max_grid;
    if (expect > 0xffffffffull / block)
        expect = 0xffffffffull / block;
    if (g * block > 0xffffffffull || g != expect || g == 0) {
        printf("FAIL work=%llu n=%llu max_grid=%d block=%llu -> grid %llu (expect %llu)\n",
               (unsigned long long) work, (unsigned long long) n, max_grid,
               (unsigned long long) block, (unsigned long long) g, (unsigned long long) expect);
        ++fails;
    }
}

int main()
{
    const uint64_t blocks[] = {64, 128, 256, 1024};
    const uint64_t sizes[] = {0, 1, 63, 64, 65, 1ull << 26, (1ull << 32) - 1, 1ull << 32,
                              (1ull << 32) + 17, 1ull << 36, 1ull << 40, 1ull << 48};
    for (uint64_t b : blocks) {
        if (max_blocks(b) * b > 0xffffffffull || (max_blocks(b) + 1) * b <= 0xffffffffull) {
            printf("FAIL max_blocks(%llu) = %llu\n", (unsigned long long) b,
                   (unsigned long long) max_blocks(b));
            ++fails;
        }
        for (uint64_t n : sizes)
            for (uint64_t per : {b, 2 * b, 4 * b})
                for (int mg : {0, 256, 1 << 30})
                    check(per, n, mg, b);
    }
    // the ADVICE r05 case: one 16-byte packet per one-wave lane, 2^32 packets
    // (64 GiB per operand) -- the old 2^31-block cap gave 2^26 x 64 ... x 2^5
    if ((uint64_t) grid_for(64, 1ull << 32, 0, 64) * 64 > 0xffffffffull)
        ++fails;
    printf("%s\n", fails ? "grid cap: FAIL" : "grid cap: ok");
    return fails ? 1 : 0;
}
