// tools/tune_policy.hip -- cache-policy and pipelining variants of the fp32
// SUM packet kernel, interleaved in one process against the shipped
// k_contig<U=4, NT, NT> geometry (256 threads, one tile per block).
//   buf<L,S>  : buffer_load/store_dwordx4 with cache-policy aux bits
//               (gfx950: sc0 = 1, nt = 2, sc1 = 16) on loads (L) / stores (S)
//   pipe<U,G> : persistent grid of G blocks per CU-equivalent (G*256 blocks),
//               the next tile's loads issued before the current tile's stores
//   ioFirst   : all inout packets loaded before any in packet
// Usage: tune_policy [count=2^28] [rounds=4] [reps=10]
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

__device__ __forceinline__ v4u add4(v4u a, v4u b) { return combine16<C>(a, b, Params{1, 0}); }

template <int LAUX, int SAUX, int U>
__global__ void __launch_bounds__(256) k_buf(const float *in, float *io, uint64_t npk)
{
    const uint64_t tile = 256ull * U;
    const uint64_t p0 = (uint64_t) blockIdx.x * tile;
    const uint64_t left = npk - p0;
    const int bytes = (int) ((left < tile ? left : tile) * 16);
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(
        (void *) (in + 4 * p0), (short) 0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void *) (io + 4 * p0), (short) 0, bytes, 0x00020000);
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int off = (threadIdx.x + u * 256) * 16;
        a[u] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, LAUX));
        b[u] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, LAUX));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int off = (threadIdx.x + u * 256) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(add4(a[u], b[u]), ro, off, 0, SAUX);
    }
}

template <int LAUX, int SAUX, int U>
void launch_buf(const float *in, float *io, uint64_t n, hipStream_t s)
{
    uint64_t npk = n / 4;
    unsigned grid = (unsigned) ((npk + 256 * U - 1) / (256 * U));
    hipLaunchKernelGGL((k_buf<LAUX, SAUX, U>), dim3(grid), dim3(256), 0, s, in, io, npk);
}

template <int U>
__global__ void __launch_bounds__(256) k_iofirst(const float *in, float *io, uint64_t npk)
{
    const v4u *vin = reinterpret_cast<const v4u *>(in);
    v4u *vio = reinterpret_cast<v4u *>(io);
    uint64_t i = (uint64_t) blockIdx.x * 256 * U + threadIdx.x;
    if (i + (U - 1) * 256 >= npk)
        return;
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        a[u] = __builtin_nontemporal_load(vio + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u)
        b[u] = __builtin_nontemporal_load(vin + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(add4(a[u], b[u]), vio + i + u * 256);
}

template <int U>
void launch_iofirst(const float *in, float *io, uint64_t n, hipStream_t s)
{
    uint64_t npk = n / 4;
    hipLaunchKernelGGL((k_iofirst<U>), dim3((unsigned) (npk / (256 * U))), dim3(256), 0, s, in, io,
                       npk);
}

// software-pipelined persistent loop: tile t+G's loads are in flight while
// tile t is combined and stored
template <int U>
__global__ void __launch_bounds__(256) k_pipe(const float *in, float *io, uint64_t ntiles)
{
    const v4u *vin = reinterpret_cast<const v4u *>(in);
    v4u *vio = reinterpret_cast<v4u *>(io);
    const uint64_t tile = 256ull * U;
    uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        a[u] = __builtin_nontemporal_load(vio + t * tile + threadIdx.x + u * 256);
        b[u] = __builtin_nontemporal_load(vin + t * tile + threadIdx.x + u * 256);
    }
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t tn = t + gridDim.x;
        v4u a2[U], b2[U];
        if (tn < ntiles) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a2[u] = __builtin_nontemporal_load(vio + tn * tile + threadIdx.x + u * 256);
                b2[u] = __builtin_nontemporal_load(vin + tn * tile + threadIdx.x + u * 256);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_nontemporal_store(add4(a[u], b[u]), vio + t * tile + threadIdx.x + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = a2[u];
            b[u] = b2[u];
        }
    }
}

template <int U, int G>
void launch_pipe(const float *in, float *io, uint64_t n, hipStream_t s)
{
    uint64_t ntiles = n / 4 / (256 * U);
    hipLaunchKernelGGL((k_pipe<U>), dim3(256 * G), dim3(256), 0, s, in, io, ntiles);
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
    if (n % (4 * 256 * 8)) {
        fprintf(stderr, "count must be a multiple of 8192\n");
        return 2;
    }
    float *a, *b, *ref, *chk;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&ref, n * 4));
    CK(hipMalloc(&chk, n * 4));
    std::vector<Var> v;
    v.push_back({"shipped k_contig U=4 nt/nt", launch_shipped, {}});
    v.push_back({"buf L=nt S=nt", launch_buf<2, 2, 4>, {}});
    v.push_back({"buf L=0 S=nt", launch_buf<0, 2, 4>, {}});
    v.push_back({"buf L=sc0|nt S=nt", launch_buf<3, 2, 4>, {}});
    v.push_back({"buf L=sc1|nt S=nt", launch_buf<18, 2, 4>, {}});
    v.push_back({"buf L=sc0|sc1|nt S=nt", launch_buf<19, 2, 4>, {}});
    v.push_back({"buf L=nt S=0", launch_buf<2, 0, 4>, {}});
    v.push_back({"buf L=nt S=sc1", launch_buf<2, 16, 4>, {}});
    v.push_back({"buf L=nt S=sc0|sc1", launch_buf<2, 17, 4>, {}});
    v.push_back({"buf L=nt S=sc1|nt", launch_buf<2, 18, 4>, {}});
    v.push_back({"buf L=nt S=sc0|sc1|nt", launch_buf<2, 19, 4>, {}});
    v.push_back({"buf L=nt S=sc0|nt", launch_buf<2, 3, 4>, {}});
    v.push_back({"buf L=nt S=nt U=2", launch_buf<2, 2, 2>, {}});
    v.push_back({"buf L=nt S=nt U=8", launch_buf<2, 2, 8>, {}});
    v.push_back({"iofirst U=4", launch_iofirst<4>, {}});
    v.push_back({"iofirst U=8", launch_iofirst<8>, {}});
    v.push_back({"pipe U=2 G=4", launch_pipe<2, 4>, {}});
    v.push_back({"pipe U=2 G=8", launch_pipe<2, 8>, {}});
    v.push_back({"pipe U=4 G=2", launch_pipe<4, 2>, {}});
    v.push_back({"pipe U=4 G=4", launch_pipe<4, 4>, {}});
    v.push_back({"pipe U=4 G=8", launch_pipe<4, 8>, {}});

    hipStream_t s;
    CK(hipStreamCreate(&s));
    // correctness: every variant's one launch equals the shipped kernel's bits
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
