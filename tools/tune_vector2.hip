// tools/tune_vector2.hip -- round-2 variants of the stride-2 vector-target
// kernel (BASELINE config 5: vector(67108864, 1, 2, MPI_DOUBLE) SUM, packed
// source), next to the shipped k_vector_s2.  The traffic floor of the layout
// is 2.5 GiB per launch (whole 1 GiB target span read, 512 MiB source read,
// 1 GiB of half-dirty lines written back: profiles/r01_pmc_vector.json); these
// variants probe what sets the rate at that floor:
//   S0  shipped (launch_vector<FSum<double>>: one {payload, gap} 16-B load per lane)
//   S1  S0 with the payload store write-through (relaxed system-scope atomic
//       store: global_store sc0 sc1, the line leaves L2 at once)
//   S2  S0 as a persistent grid (2048 blocks, grid-stride, one pair per lane
//       per iteration)
//   S3  S0 with the source load non-temporal and 2 pairs per lane at
//       block stride (both target loads issued before either source load)
//   S4  LDS-staged: a block loads a 16 KiB target tile + its 4 KiB source
//       with 16-B loads, adds in LDS, then the payload is stored by lanes
//       walking the tile in order (same bytes, different store order)
// Interleaved rounds in one process; median GB/s algorithmic (3 x 512 MiB) and
// physical (2.5 GiB).  Every variant's result is checked against S0's.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
using C = FSum<double>;
typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_s1(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    d2 t = reinterpret_cast<const d2 *>(io)[k];
    double r = t.x + in[k];
    __hip_atomic_store(io + 2 * k, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(256) k_s2(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        d2 t = reinterpret_cast<const d2 *>(io)[k];
        io[2 * k] = t.x + in[k];
    }
}

__global__ void __launch_bounds__(256) k_s3(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    const uint64_t k0 = (uint64_t) blockIdx.x * 512 + threadIdx.x, k1 = k0 + 256;
    d2 t0 = {0, 0}, t1 = {0, 0};
    if (k0 < n)
        t0 = reinterpret_cast<const d2 *>(io)[k0];
    if (k1 < n)
        t1 = reinterpret_cast<const d2 *>(io)[k1];
    if (k0 < n)
        io[2 * k0] = t0.x + __builtin_nontemporal_load(in + k0);
    if (k1 < n)
        io[2 * k1] = t1.x + __builtin_nontemporal_load(in + k1);
}

// tile = 1024 pairs (16 KiB of target), 256 lanes x 4
__global__ void __launch_bounds__(256) k_s4(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    __shared__ double pay[1024];
    const uint64_t base = (uint64_t) blockIdx.x * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t k = base + u * 256 + threadIdx.x;
        if (k < n) {
            d2 t = reinterpret_cast<const d2 *>(io)[k];
            pay[u * 256 + threadIdx.x] = t.x;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t k = base + u * 256 + threadIdx.x;
        if (k < n)
            io[2 * k] = pay[u * 256 + threadIdx.x] + in[k];
    }
}

// S5 = S1's write-through store + S3's shape (2 pairs per lane at block stride, nt source)
__global__ void __launch_bounds__(256) k_s5(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    const uint64_t k0 = (uint64_t) blockIdx.x * 512 + threadIdx.x, k1 = k0 + 256;
    d2 t0 = {0, 0}, t1 = {0, 0};
    if (k0 < n)
        t0 = reinterpret_cast<const d2 *>(io)[k0];
    if (k1 < n)
        t1 = reinterpret_cast<const d2 *>(io)[k1];
    if (k0 < n)
        __hip_atomic_store(io + 2 * k0, t0.x + __builtin_nontemporal_load(in + k0),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (k1 < n)
        __hip_atomic_store(io + 2 * k1, t1.x + __builtin_nontemporal_load(in + k1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// S6 = S1 with the source read non-temporally
__global__ void __launch_bounds__(256) k_s6(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    d2 t = reinterpret_cast<const d2 *>(io)[k];
    __hip_atomic_store(io + 2 * k, t.x + __builtin_nontemporal_load(in + k), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// S7 = S6 with the target pair loaded non-temporally too
__global__ void __launch_bounds__(256) k_s7(const double *__restrict__ in, double *__restrict__ io,
                                            uint64_t n)
{
    uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    d2 t = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(io) + k);
    __hip_atomic_store(io + 2 * k, t.x + __builtin_nontemporal_load(in + k), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// S8 = S6 with 512-thread blocks; S9 = S6 with 1024-thread blocks (same kernel body)
template <int B>
__global__ void __launch_bounds__(1024) k_s8(const double *__restrict__ in, double *__restrict__ io,
                                             uint64_t n)
{
    uint64_t k = (uint64_t) blockIdx.x * B + threadIdx.x;
    if (k >= n)
        return;
    d2 t = reinterpret_cast<const d2 *>(io)[k];
    __hip_atomic_store(io + 2 * k, t.x + __builtin_nontemporal_load(in + k), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// S10 = S6 with the target loaded as relaxed system-scope atomics (sc0 sc1 loads)
__global__ void __launch_bounds__(256) k_s10(const double *__restrict__ in, double *__restrict__ io,
                                             uint64_t n)
{
    uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n)
        return;
    double t = __hip_atomic_load(io + 2 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(io + 2 * k, t + __builtin_nontemporal_load(in + k), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Var {
    std::string name;
    void (*launch)(const double *, double *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

void s0(const double *in, double *io, uint64_t n, hipStream_t s)
{
    launch_vector<C>(in, io, n, 1, 2, Params{1, 0}, LaunchCfg{256, 0}, s);
}
void s1(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s1, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, in, io, n);
}
void s2(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s2, dim3(2048), dim3(256), 0, s, in, io, n);
}
void s3(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s3, dim3((unsigned) ((n + 511) / 512)), dim3(256), 0, s, in, io, n);
}
void s4(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s4, dim3((unsigned) ((n + 1023) / 1024)), dim3(256), 0, s, in, io, n);
}

void s5(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s5, dim3((unsigned) ((n + 511) / 512)), dim3(256), 0, s, in, io, n);
}
void s6(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s6, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, in, io, n);
}

void s7(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s7, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, in, io, n);
}
template <int B>
void s8(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL((k_s8<B>), dim3((unsigned) ((n + B - 1) / B)), dim3(B), 0, s, in, io, n);
}
void s10(const double *in, double *io, uint64_t n, hipStream_t s)
{
    hipLaunchKernelGGL(k_s10, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, in, io, n);
}

int main()
{
    const uint64_t n = 67108864;
    double *src, *dst, *ref;
    CK(hipMalloc(&src, n * 8));
    CK(hipMalloc(&dst, 2 * n * 8));
    CK(hipMalloc(&ref, 2 * n * 8));
    std::vector<Var> v = {{"S0 shipped k_vector_s2", s0, {}}, {"S1 write-through store", s1, {}},
                          {"S2 persistent grid 2048", s2, {}},
                          {"S3 2 pairs/lane, nt source", s3, {}},
                          {"S4 LDS-staged 16 KiB tile", s4, {}},
                          {"S5 write-through + 2 pairs/lane + nt source", s5, {}},
                          {"S6 write-through + nt source", s6, {}},
                          {"S7 S6 + nt target load", s7, {}},
                          {"S8 S6 with 512-thread blocks", s8<512>, {}},
                          {"S9 S6 with 1024-thread blocks", s8<1024>, {}},
                          {"S10 S6 with sc0 sc1 payload-only target load", s10, {}}};
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // correctness first: every variant from the same start equals S0
    std::vector<double> h(2 * n);
    for (uint64_t i = 0; i < 2 * n; ++i)
        h[i] = (double) ((i * 2654435761u) % 1000) * 0.25;
    CK(hipMemcpy(src, h.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(ref, h.data(), 2 * n * 8, hipMemcpyHostToDevice));
    s0(src, ref, n, s);
    std::vector<double> want(2 * n), got(2 * n);
    CK(hipMemcpy(want.data(), ref, 2 * n * 8, hipMemcpyDeviceToHost));
    for (auto &x : v) {
        CK(hipMemcpy(dst, h.data(), 2 * n * 8, hipMemcpyHostToDevice));
        x.launch(src, dst, n, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(got.data(), dst, 2 * n * 8, hipMemcpyDeviceToHost));
        if (memcmp(got.data(), want.data(), 2 * n * 8) != 0) {
            printf("MISMATCH %s\n", x.name.c_str());
            return 1;
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 7; ++r)
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
        printf("%8.1f GB/s alg  %8.1f GB/s phys  %.4f ms  %s\n", 3.0 * n * 8 / (med * 1e-3) / 1e9,
               2.5 * (1 << 30) / (med * 1e-3) / 1e9, med, x.name.c_str());
    }
    return 0;
}
