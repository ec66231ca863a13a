// tools/tune_lds.hip -- LDS-DMA (global_load_lds_dwordx4) variants of the
// fp32 SUM packet kernel, interleaved in one process against the shipped
// k_contig<U=4, NT, NT> geometry.  The guide measures an nt LDS-DMA read
// stream at 6.5-6.8 TB/s chip-wide; this checks whether staging the two
// operand streams through LDS (each lane reads back its own 16-B slot, so
// only the issuing wave's vmcnt orders it: no barrier) lifts the combined
// read+write stream.  glds<U, AUX, T, IO>: T threads per block, U packets
// per lane per operand, AUX cache bits on the LDS-DMA loads, IO = inout also
// via LDS-DMA (else an nt register load).
// Usage: tune_lds [count=2^28] [rounds=4] [reps=10]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <string>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
using C = FSum<float>;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef void (*LaunchFn)(const float *, float *, uint64_t, hipStream_t);
struct Var {
    std::string name;
    LaunchFn launch;
    std::vector<float> ms;
};

typedef __attribute__((address_space(3))) void lds_void;

template <int U, int AUX, int T, bool IO>
__global__ void __launch_bounds__(T) k_glds(const float *in, float *io, uint64_t npk)
{
    __shared__ v4u sm[2][U][T];
    const v4u *vin = reinterpret_cast<const v4u *>(in);
    v4u *vio = reinterpret_cast<v4u *>(io);
    const int w = threadIdx.x / 64;
    const uint64_t i = (uint64_t) blockIdx.x * T * U + threadIdx.x;
    if (i + (U - 1) * T >= npk)
        return;                 // whole tiles only (count is a multiple of T*U*4)
    v4u a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if constexpr (IO)
            __builtin_amdgcn_global_load_lds((const void *) (vio + i + u * T),
                                             (lds_void *) &sm[0][u][w * 64], 16, 0, AUX);
        else
            a[u] = __builtin_nontemporal_load(vio + i + u * T);
        __builtin_amdgcn_global_load_lds((const void *) (vin + i + u * T),
                                         (lds_void *) &sm[1][u][w * 64], 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
        v4u x = IO ? sm[0][u][threadIdx.x] : a[u];
        __builtin_nontemporal_store(combine16<C>(x, sm[1][u][threadIdx.x], Params{1, 0}),
                                    vio + i + u * T);
    }
}

template <int U, int AUX, int T, bool IO>
void launch_glds(const float *in, float *io, uint64_t n, hipStream_t s)
{
    uint64_t npk = n / 4;
    hipLaunchKernelGGL((k_glds<U, AUX, T, IO>), dim3((unsigned) (npk / (T * U))), dim3(T), 0, s,
                       in, io, npk);
}

void launch_shipped(const float *in, float *io, uint64_t n, hipStream_t s)
{
    uint64_t npk = n / 4;
    unsigned grid = grid_for(256ull * 4, npk, 0);
    hipLaunchKernelGGL((k_contig<C, 4, true, true>), dim3(grid), dim3(256), 0, s, in, io,
                       (uint64_t) 0, npk, npk * 4, (uint32_t) 0, Params{1, 0});
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

__global__ void snap(const float *p, float *q, uint64_t n)
{
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x)
        q[i] = p[i];
}

int main(int argc, char **argv)
{
    uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 28);
    int rounds = argc > 2 ? atoi(argv[2]) : 4;
    int reps = argc > 3 ? atoi(argv[3]) : 10;
    if (n % (4 * 512 * 8)) {
        fprintf(stderr, "count must be a multiple of 16384\n");
        return 2;
    }
    float *a, *b, *ref, *chk;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&ref, n * 4));
    CK(hipMalloc(&chk, n * 4));
    std::vector<Var> v;
    v.push_back({"shipped k_contig U=4 nt/nt", launch_shipped, {}});
    v.push_back({"glds U=2 nt T=256 io+in", launch_glds<2, 2, 256, true>, {}});
    v.push_back({"glds U=4 nt T=256 io+in", launch_glds<4, 2, 256, true>, {}});
    v.push_back({"glds U=8 nt T=256 io+in", launch_glds<8, 2, 256, true>, {}});
    v.push_back({"glds U=4 def T=256 io+in", launch_glds<4, 0, 256, true>, {}});
    v.push_back({"glds U=4 nt T=512 io+in", launch_glds<4, 2, 512, true>, {}});
    v.push_back({"glds U=2 nt T=512 io+in", launch_glds<2, 2, 512, true>, {}});
    v.push_back({"glds U=4 nt T=256 in only", launch_glds<4, 2, 256, false>, {}});
    v.push_back({"glds U=2 nt T=256 in only", launch_glds<2, 2, 256, false>, {}});

    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, b, n, 2u);
    int bad = 0;
    for (size_t k = 0; k < v.size(); ++k) {
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, a, n, 1u);
        v[k].launch(b, a, n, s);
        hipLaunchKernelGGL(snap, dim3(4096), dim3(256), 0, s, a, k == 0 ? ref : chk, n);
        CK(hipStreamSynchronize(s));
        CK(hipGetLastError());
        if (k) {
            std::vector<float> x(1 << 16), y(1 << 16);
            for (uint64_t off : {(uint64_t) 0, n / 2, n - (1 << 16)}) {
                CK(hipMemcpy(x.data(), ref + off, 4 << 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(y.data(), chk + off, 4 << 16, hipMemcpyDeviceToHost));
                if (memcmp(x.data(), y.data(), 4 << 16)) {
                    printf("MISMATCH %s at window %llu\n", v[k].name.c_str(),
                           (unsigned long long) off);
                    bad = 1;
                }
            }
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto &x : v) {
            for (int w = 0; w < 2; ++w)
                x.launch(b, a, n, s);
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0, s));
                x.launch(b, a, n, s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                x.ms.push_back(ms);
            }
        }
    }
    printf("# count %llu fp32 per operand (%llu MiB), %d rounds x %d reps, interleaved\n",
           (unsigned long long) n, (unsigned long long) (n * 4 >> 20), rounds, reps);
    std::vector<std::pair<double, std::string>> res;
    for (auto &x : v) {
        std::sort(x.ms.begin(), x.ms.end());
        double med = x.ms[x.ms.size() / 2];
        res.push_back({3.0 * n * 4 / (med * 1e-3) / 1e9, x.name});
    }
    std::sort(res.begin(), res.end());
    for (auto &r : res)
        printf("%8.1f GB/s  %s\n", r.first, r.second.c_str());
    for (auto &x : v)
        printf("# %-32s min %.4f med %.4f max %.4f ms (n=%zu)\n", x.name.c_str(), x.ms.front(),
               x.ms[x.ms.size() / 2], x.ms.back(), x.ms.size());
    return bad;
}
