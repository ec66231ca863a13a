// tools/tune_sum.hip -- launch-geometry / cache-policy sweep of the product
// packet kernel (mpich_amd/csrc/redop_kernels.h) on fp32 SUM, 1 GiB per
// operand.  All variants run interleaved in one process (guide §5.4 rule 24);
// prints median GB/s (algorithmic 3 x 1 GiB per launch) per variant.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 \
//        -I mpich_amd/csrc -I include tools/tune_sum.hip -o /tmp/tune_sum
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <string>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
using C = FSum<float>;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

struct Var {
    std::string name;
    void (*launch)(const float *, float *, uint64_t, int, int, hipStream_t);
    int block, maxgrid;
    std::vector<float> ms;
};

template <int U, bool NTL, bool NTS>
void launch_v(const float *in, float *io, uint64_t n, int block, int maxgrid, hipStream_t s)
{
    uint64_t npk = n / 4;
    unsigned grid = grid_for((uint64_t) block * U, npk, maxgrid);
    hipLaunchKernelGGL((k_contig<C, U, NTL, NTS>), dim3(grid), dim3(block), 0, s, in, io,
                       (uint64_t) 0, npk, npk * 4, (uint32_t) 0, Params{1, 0});
}

template <int U, bool NTL, bool NTS>
void add(std::vector<Var> &v, int block, int maxgrid)
{
    char nm[128];
    snprintf(nm, sizeof nm, "U=%d ntl=%d nts=%d block=%d maxgrid=%d", U, NTL, NTS, block, maxgrid);
    v.push_back(Var{nm, &launch_v<U, NTL, NTS>, block, maxgrid, {}});
}

template <int U>
void add_all(std::vector<Var> &v, int block, int maxgrid)
{
    add<U, false, false>(v, block, maxgrid);
    add<U, true, false>(v, block, maxgrid);
    add<U, false, true>(v, block, maxgrid);
    add<U, true, true>(v, block, maxgrid);
}

// XCD-aware variant: with round-robin placement, block b runs on XCD b % 8;
// remap so each XCD walks one contiguous eighth of the buffer.
template <int U>
__global__ void __launch_bounds__(1024) k_xcd(const float *__restrict__ in, float *__restrict__ io,
                                              uint64_t npk)
{
    const v4u *vin = reinterpret_cast<const v4u *>(in);
    v4u *vio = reinterpret_cast<v4u *>(io);
    const uint64_t nt = blockDim.x, G = gridDim.x;
    const uint64_t b = blockIdx.x;
    const uint64_t per = G / 8;
    const uint64_t lb = (b < per * 8) ? (b % 8) * per + b / 8 : b;
    uint64_t i = lb * nt * U + threadIdx.x;
    v4u a[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * nt < npk) {
            a[u] = __builtin_nontemporal_load(vio + i + u * nt);
            c[u] = __builtin_nontemporal_load(vin + i + u * nt);
        }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * nt < npk)
            __builtin_nontemporal_store(combine16<C>(a[u], c[u], Params{1, 0}), vio + i + u * nt);
}

template <int U>
void launch_x(const float *in, float *io, uint64_t n, int block, int, hipStream_t s)
{
    uint64_t npk = n / 4;
    unsigned grid = grid_for((uint64_t) block * U, npk, 0);
    hipLaunchKernelGGL((k_xcd<U>), dim3(grid), dim3(block), 0, s, in, io, npk);
}

__global__ void fill(float *p, uint64_t n, uint32_t seed)
{
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t) i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (float) (x & 0xffffff) / 8388608.0f - 1.0f;
    }
}

int main(int argc, char **argv)
{
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 28);
    int rounds = argc > 2 ? atoi(argv[2]) : 3;
    int reps = argc > 3 ? atoi(argv[3]) : 10;
    float *a, *b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a, n, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, b, n, 2u);
    CK(hipDeviceSynchronize());
    bool focus = argc > 4 && std::string(argv[4]) == "focus";
    std::vector<Var> v;
    if (argc > 4 && std::string(argv[4]) == "xcd") {   // shipped geometry vs XCD remap
        for (int block : {256, 512}) {
            add<4, true, true>(v, block, 0);
            add<1, true, true>(v, block, 0);
            char nm[64];
            snprintf(nm, sizeof nm, "XCD-remap U=4 block=%d", block);
            v.push_back(Var{nm, &launch_x<4>, block, 0, {}});
            snprintf(nm, sizeof nm, "XCD-remap U=1 block=%d", block);
            v.push_back(Var{nm, &launch_x<1>, block, 0, {}});
        }
    } else if (focus) { // NT/NT, one tile per block: the winners of the full sweep
        for (int block : {256, 512, 1024}) {
            add<1, true, true>(v, block, 0);
            add<2, true, true>(v, block, 0);
            add<4, true, true>(v, block, 0);
            add<8, true, true>(v, block, 0);
            add<16, true, true>(v, block, 0);
        }
    } else {
        for (int block : {256, 512, 1024}) {
            for (int mg : {0, 2048, 4096}) {
                add_all<1>(v, block, mg);
                add_all<2>(v, block, mg);
                add_all<4>(v, block, mg);
                add_all<8>(v, block, mg);
            }
        }
    }
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto &x : v) {
            for (int w = 0; w < 2; ++w)
                x.launch(b, a, n, x.block, x.maxgrid, s);
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0, s));
                x.launch(b, a, n, x.block, x.maxgrid, s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                x.ms.push_back(ms);
            }
        }
    }
    std::vector<std::pair<double, std::string>> res;
    for (auto &x : v) {
        std::sort(x.ms.begin(), x.ms.end());
        double med = x.ms[x.ms.size() / 2];
        res.push_back({3.0 * n * 4 / (med * 1e-3) / 1e9, x.name});
    }
    std::sort(res.begin(), res.end());
    for (auto &r : res)
        printf("%8.1f GB/s  %s\n", r.first, r.second.c_str());
    for (auto &x : v) {     // spread per variant (min / median / max of all launches)
        printf("# %-40s min %.4f med %.4f max %.4f ms (n=%zu)\n", x.name.c_str(), x.ms.front(),
               x.ms[x.ms.size() / 2], x.ms.back(), x.ms.size());
    }
    return 0;
}
