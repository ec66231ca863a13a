// tools/tune_vector.hip -- variants of the vector-target kernel for BASELINE
// config 5: vector(67108864, 1, 2, MPI_DOUBLE) SUM, packed source.
// V0 = product k_vector1 (8-B target loads at 16-B stride);
// V1<U,NT> = 16-B target packets (payload + gap) loaded whole, U per lane,
//            8-B payload stores (gaps never written);
// V2<NTS>  = two adjacent pairs per lane: 32 B of target (2 x 16-B loads),
//            one 16-B source packet (non-temporal if NTS), two 8-B stores;
// V3<B>    = V1 U=1 with the source read non-temporally, block size B;
// Interleaved rounds in one process; median GB/s (algorithmic 3 x 512 MiB).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <string>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
using C = FSum<double>;
typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int U, bool NT>
__global__ void __launch_bounds__(256) k_v1(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    const uint64_t nt = blockDim.x;
    uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x;
    d2 t[U];
    double s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint64_t k = i + u * nt;
        if (k < n) {
            if constexpr (NT) {
                t[u] = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(io) + k);
                s[u] = __builtin_nontemporal_load(in + k);
            } else {
                t[u] = reinterpret_cast<const d2 *>(io)[k];
                s[u] = in[k];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint64_t k = i + u * nt;
        if (k < n) {
            double r = t[u].x + s[u];
            if constexpr (NT)
                __builtin_nontemporal_store(r, io + 2 * k);
            else
                io[2 * k] = r;
        }
    }
}

template <bool NTS>
__global__ void __launch_bounds__(256) k_v2(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n2)
{
    uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;     // pair-of-pairs index
    if (i >= n2)
        return;
    const d2 *t = reinterpret_cast<const d2 *>(io) + 2 * i;
    d2 a = t[0], b = t[1];
    d2 x = NTS ? __builtin_nontemporal_load(reinterpret_cast<const d2 *>(in) + i)
               : reinterpret_cast<const d2 *>(in)[i];
    io[4 * i] = a.x + x.x;
    io[4 * i + 2] = b.x + x.y;
}

template <int B>
__global__ void __launch_bounds__(1024) k_v3(const double *__restrict__ in, double *__restrict__ io,
                                             uint64_t n)
{
    uint64_t k = (uint64_t) blockIdx.x * B + threadIdx.x;
    if (k >= n)
        return;
    d2 t = reinterpret_cast<const d2 *>(io)[k];
    double x = __builtin_nontemporal_load(in + k);
    io[2 * k] = t.x + x;
}

struct Var {
    std::string name;
    void (*launch)(const double *, double *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

void v0(const double *in, double *io, uint64_t n, hipStream_t s)
{
    LaunchCfg cfg{256, 0};
    launch_vector<C>(in, io, n, 1, 2, Params{1, 0}, cfg, s);
}

template <int U, bool NT>
void v1(const double *in, double *io, uint64_t n, hipStream_t s)
{
    unsigned grid = (unsigned) ((n + 256ull * U - 1) / (256ull * U));
    hipLaunchKernelGGL((k_v1<U, NT>), dim3(grid), dim3(256), 0, s, in, io, n);
}

template <bool NTS>
void v2(const double *in, double *io, uint64_t n, hipStream_t s)
{
    uint64_t n2 = n / 2;
    hipLaunchKernelGGL((k_v2<NTS>), dim3((unsigned) ((n2 + 255) / 256)), dim3(256), 0, s, in, io,
                       n2);
}

template <int B>
void v3(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL((k_v3<B>), dim3((unsigned) ((n + B - 1) / B)), dim3(B), 0, s, in, io, n);
}

int main()
{
    uint64_t n = 67108864;
    double *src, *dst;
    CK(hipMalloc(&src, n * 8));
    CK(hipMalloc(&dst, 2 * n * 8));
    CK(hipMemset(src, 0, n * 8));
    CK(hipMemset(dst, 0, 2 * n * 8));
    std::vector<Var> v = {{"V0 product k_vector1", v0, {}},
                          {"V1 U=1 nt=0", v1<1, false>, {}}, {"V1 U=1 nt=1", v1<1, true>, {}},
                          {"V1 U=2 nt=0", v1<2, false>, {}}, {"V1 U=2 nt=1", v1<2, true>, {}},
                          {"V1 U=4 nt=0", v1<4, false>, {}}, {"V1 U=4 nt=1", v1<4, true>, {}},
                          {"V1 U=8 nt=1", v1<8, true>, {}},
                          {"V2 nts=0", v2<false>, {}}, {"V2 nts=1", v2<true>, {}},
                          {"V3 block=256", v3<256>, {}}, {"V3 block=512", v3<512>, {}},
                          {"V3 block=1024", v3<1024>, {}}};
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 5; ++r)
        for (auto &x : v) {
            x.launch(src, dst, n, s);
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < 10; ++k)
                x.launch(src, dst, n, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            x.ms.push_back(ms / 10);
        }
    for (auto &x : v) {
        std::sort(x.ms.begin(), x.ms.end());
        double med = x.ms[x.ms.size() / 2];
        printf("%8.1f GB/s alg  %.4f ms  %s\n", 3.0 * n * 8 / (med * 1e-3) / 1e9, med, x.name.c_str());
    }
    return 0;
}
