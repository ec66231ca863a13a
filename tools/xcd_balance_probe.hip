// xcd_balance_probe.hip -- with the store policy (blocks on XCDs 3 and 7
// store write-through, the rest non-temporally) do the eight XCDs finish their
// share of the 1 GiB fp32 SUM stream together, or does one group wait for the
// other (which a dynamic tile assignment could rebalance)?  Every block
// records its XCD and its start / end on the 100 MHz wall clock; per XCD the
// last end and the blocks' mean duration are reported, for the policy off and on.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xcd_balance_probe.hip -o tools/bin/xcd_balance_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t _e = (x);                                                         \
        if (_e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(_e)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;

__device__ __forceinline__ unsigned xcc()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7;
}

constexpr int U = 4, NT = 256;

// ROT: block b takes tile 8*(b/8) + (b % 8 + b/8) % 8 -- a rotation inside
// every group of eight tiles, so the blocks of one XCD (b % 8 fixed under
// round-robin dispatch) visit every address residue mod 8 tiles instead of one
template <bool ROT = false>
__global__ void __launch_bounds__(256) k_rec(const v4u *__restrict__ in, v4u *__restrict__ io,
                                             uint64_t npk, unsigned mask, uint64_t *rec)
{
    const uint64_t t0 = wall_clock64();
    const unsigned x = xcc();
    const bool wt = (mask >> x) & 1;
    uint64_t tileno = blockIdx.x;
    if (ROT)
        tileno = (tileno & ~7ull) | (((tileno & 7) + (tileno >> 3)) & 7);
    const uint64_t i = tileno * NT * U + threadIdx.x;
    if (i + (U - 1) * NT < npk) {
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = __builtin_nontemporal_load(io + i + u * NT);
#pragma unroll
        for (int u = 0; u < U; ++u)
            b[u] = __builtin_nontemporal_load(in + i + u * NT);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4 p = __builtin_bit_cast(float4, a[u]), q = __builtin_bit_cast(float4, b[u]);
            p.x += q.x; p.y += q.y; p.z += q.z; p.w += q.w;
            if (wt)
                *(volatile gv4u *) (gv4u *) (io + i + u * NT) = __builtin_bit_cast(v4u, p);
            else
                __builtin_nontemporal_store(__builtin_bit_cast(v4u, p), io + i + u * NT);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);      // this lane's stores acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
        rec[3 * blockIdx.x] = x;
        rec[3 * blockIdx.x + 1] = t0;
        rec[3 * blockIdx.x + 2] = wall_clock64();
    }
}

// Persistent form: G blocks take 16 KiB tiles by ticket (the next ticket is
// fetched while the current tile is in flight), so an XCD that runs faster
// takes more tiles; tiles per XCD are counted in cnt[8].
// LIGHT: the loop's barrier waits for LDS only (s_waitcnt lgkmcnt(0);
// s_barrier), not for the tile's stores as __syncthreads()'s workgroup fence
// does (s_waitcnt vmcnt(0)), so stores drain while the next tile loads
__device__ __forceinline__ void bar_lds()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool LIGHT>
__global__ void __launch_bounds__(256) k_pers(const v4u *__restrict__ in, v4u *__restrict__ io,
                                              uint64_t ntiles, unsigned mask, unsigned *ctr,
                                              unsigned *cnt)
{
    __shared__ unsigned s_t[2];
    const unsigned x = xcc();
    const bool wt = (mask >> x) & 1;
    if (threadIdx.x == 0)
        s_t[0] = atomicAdd(ctr, 1u);
    __syncthreads();
    unsigned t = s_t[0], mine = 0;
    int cur = 0;
    while (t < ntiles) {
        if (threadIdx.x == 0)
            s_t[cur ^ 1] = atomicAdd(ctr, 1u);
        const uint64_t i = (uint64_t) t * NT * U + threadIdx.x;
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = __builtin_nontemporal_load(io + i + u * NT);
#pragma unroll
        for (int u = 0; u < U; ++u)
            b[u] = __builtin_nontemporal_load(in + i + u * NT);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4 p = __builtin_bit_cast(float4, a[u]), q = __builtin_bit_cast(float4, b[u]);
            p.x += q.x; p.y += q.y; p.z += q.z; p.w += q.w;
            if (wt)
                *(volatile gv4u *) (gv4u *) (io + i + u * NT) = __builtin_bit_cast(v4u, p);
            else
                __builtin_nontemporal_store(__builtin_bit_cast(v4u, p), io + i + u * NT);
        }
        ++mine;
        if (LIGHT)
            bar_lds();
        else
            __syncthreads();
        cur ^= 1;
        t = s_t[cur];
    }
    if (threadIdx.x == 0)
        atomicAdd(&cnt[x], mine);
}

// Tile stealing: a grid of (ntiles - K) blocks, each takes tiles by ticket
// until they run out -- most blocks do one tile, and the blocks that finish
// while tickets remain (those on the fast XCDs) take the rest.
__global__ void __launch_bounds__(256) k_steal(const v4u *__restrict__ in, v4u *__restrict__ io,
                                               uint64_t ntiles, unsigned mask, unsigned *ctr,
                                               unsigned *cnt)
{
    __shared__ unsigned s_t;
    const unsigned x = xcc();
    const bool wt = (mask >> x) & 1;
    unsigned mine = 0;
    for (;;) {
        if (threadIdx.x == 0)
            s_t = atomicAdd(ctr, 1u);
        __syncthreads();
        const unsigned t = s_t;
        if (t >= ntiles)
            break;
        const uint64_t i = (uint64_t) t * NT * U + threadIdx.x;
        v4u a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = __builtin_nontemporal_load(io + i + u * NT);
#pragma unroll
        for (int u = 0; u < U; ++u)
            b[u] = __builtin_nontemporal_load(in + i + u * NT);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4 p = __builtin_bit_cast(float4, a[u]), q = __builtin_bit_cast(float4, b[u]);
            p.x += q.x; p.y += q.y; p.z += q.z; p.w += q.w;
            if (wt)
                *(volatile gv4u *) (gv4u *) (io + i + u * NT) = __builtin_bit_cast(v4u, p);
            else
                __builtin_nontemporal_store(__builtin_bit_cast(v4u, p), io + i + u * NT);
        }
        ++mine;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (threadIdx.x == 0 && mine > 1)
        atomicAdd(&cnt[x], mine - 1);       // extra tiles taken on this XCD
}

int main()
{
    const size_t bytes = (size_t) 1 << 30;
    const uint64_t npk = bytes / 16;
    const unsigned grid = (unsigned) (npk / (NT * U));
    v4u *in, *io;
    uint64_t *rec;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&io, bytes));
    CK(hipMalloc(&rec, (size_t) grid * 3 * 8));
    CK(hipMemset(in, 0, bytes));
    CK(hipMemset(io, 0, bytes));
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> h((size_t) grid * 3);
    printf("{\"probe\": \"xcd_balance_probe\", \"grid\": %u, \"runs\": [", grid);
    const unsigned masks[] = {0x00, 0x88, 0x00, 0x88, 0x00, 0x88, 0x00, 0x88};
    for (int r = 0; r < 8; ++r) {
        const bool rot = r >= 4;
        auto go = [&]() {
            if (rot)
                hipLaunchKernelGGL(k_rec<true>, dim3(grid), dim3(NT), 0, 0, in, io, npk, masks[r], rec);
            else
                hipLaunchKernelGGL(k_rec<false>, dim3(grid), dim3(NT), 0, 0, in, io, npk, masks[r], rec);
        };
        for (int w = 0; w < 3; ++w)     // warm-up launches, then the recorded one
            go();
        go();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t_start = ~0ull, t_end = 0;
        uint64_t last[8] = {0}, nblk[8] = {0}, dur[8] = {0};
        for (unsigned b = 0; b < grid; ++b) {
            const unsigned x = (unsigned) h[3 * b] & 7;
            t_start = std::min(t_start, h[3 * b + 1]);
            t_end = std::max(t_end, h[3 * b + 2]);
            last[x] = std::max(last[x], h[3 * b + 2]);
            ++nblk[x];
            dur[x] += h[3 * b + 2] - h[3 * b + 1];
        }
        printf("%s{\"mask\": %u, \"rotated\": %s, \"span_us\": %.2f, \"xcd\": [", r ? ", " : "",
               masks[r], rot ? "true" : "false", (t_end - t_start) / 100.0);
        for (int x = 0; x < 8; ++x)
            printf("%s{\"blocks\": %llu, \"last_end_us\": %.2f, \"mean_block_us\": %.3f}", x ? ", " : "",
                   (unsigned long long) nblk[x], (last[x] - t_start) / 100.0,
                   nblk[x] ? dur[x] / 100.0 / nblk[x] : 0.0);
        printf("]}");
    }
    printf("], \"persistent\": [");
    unsigned *ctr;
    CK(hipMalloc(&ctr, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // grid 0: the one-tile-per-block kernel; > 0: persistent with __syncthreads;
    // < 0 (as int): persistent with the LDS-only barrier
    const int grids[] = {0, 2048, -1024, -2048, -4096, 0, 2048, -1024, -2048, -4096};
    for (int r = 0; r < 10; ++r) {
        const bool light = grids[r] < 0;
        const unsigned G = (unsigned) (grids[r] < 0 ? -grids[r] : grids[r]);
        float tot = 0;
        unsigned cnt[8] = {0};
        for (int rep = 0; rep < 11; ++rep) {
            CK(hipMemsetAsync(ctr, 0, 64, 0));
            CK(hipEventRecord(e0, 0));
            if (G && light)
                hipLaunchKernelGGL(k_pers<true>, dim3(G), dim3(NT), 0, 0, in, io, (uint64_t) grid,
                                   0x88u, ctr, ctr + 4);
            else if (G)
                hipLaunchKernelGGL(k_pers<false>, dim3(G), dim3(NT), 0, 0, in, io, (uint64_t) grid,
                                   0x88u, ctr, ctr + 4);
            else
                hipLaunchKernelGGL(k_rec<false>, dim3(grid), dim3(NT), 0, 0, in, io, npk, 0x88u, rec);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep)
                tot += ms;
            if (G && rep == 10) {
                unsigned h2[12];
                CK(hipMemcpy(h2, ctr, 48, hipMemcpyDeviceToHost));
                for (int k = 0; k < 8; ++k)
                    cnt[k] = h2[4 + k];
            }
        }
        printf("%s{\"grid\": %u, \"lds_only_barrier\": %s, \"ms\": %.4f, \"tiles_per_xcd\": [",
               r ? ", " : "", G, light ? "true" : "false", tot / 10);
        for (int k = 0; k < 8; ++k)
            printf("%s%u", k ? ", " : "", cnt[k]);
        printf("]}");
    }
    printf("], \"timed\": [");
    for (int r = 0; r < 6; ++r) {
        const bool rot = r % 2;
        float tot = 0;
        for (int rep = 0; rep < 11; ++rep) {
            CK(hipEventRecord(e0, 0));
            if (rot)
                hipLaunchKernelGGL(k_rec<true>, dim3(grid), dim3(NT), 0, 0, in, io, npk, 0x88u, rec);
            else
                hipLaunchKernelGGL(k_rec<false>, dim3(grid), dim3(NT), 0, 0, in, io, npk, 0x88u, rec);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep)
                tot += ms;
        }
        printf("%s{\"rotated\": %s, \"ms\": %.4f}", r ? ", " : "", rot ? "true" : "false", tot / 10);
    }
    printf("], \"steal\": [");
    const double fr[] = {0.0, 0.0, 0.01, 0.03, 0.06, 0.0, 0.01, 0.03, 0.06};
    for (int r = 0; r < 9; ++r) {
        const bool plain = r == 0;
        const unsigned G = grid - (unsigned) (fr[r] * grid);
        float tot = 0;
        unsigned cnt[8] = {0};
        for (int rep = 0; rep < 11; ++rep) {
            CK(hipMemsetAsync(ctr, 0, 64, 0));
            CK(hipEventRecord(e0, 0));
            if (plain)
                hipLaunchKernelGGL(k_rec<false>, dim3(grid), dim3(NT), 0, 0, in, io, npk, 0x88u, rec);
            else
                hipLaunchKernelGGL(k_steal, dim3(G), dim3(NT), 0, 0, in, io, (uint64_t) grid, 0x88u,
                                   ctr, ctr + 4);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep)
                tot += ms;
            if (!plain && rep == 10) {
                unsigned h2[12];
                CK(hipMemcpy(h2, ctr, 48, hipMemcpyDeviceToHost));
                for (int k = 0; k < 8; ++k)
                    cnt[k] = h2[4 + k];
            }
        }
        printf("%s{\"one_tile_per_block\": %s, \"blocks\": %u, \"ms\": %.4f, \"extra_tiles_per_xcd\": [",
               r ? ", " : "", plain ? "true" : "false", plain ? grid : G, tot / 10);
        for (int k = 0; k < 8; ++k)
            printf("%s%u", k ? ", " : "", cnt[k]);
        printf("]}");
    }
    printf("]}\n");
    return 0;
}
