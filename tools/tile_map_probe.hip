// tile_map_probe.hip -- does the order in which blocks walk the tiles decide
// the per-placement split of the 1 GiB fp32 SUM (DESIGN "per-process split")?
// The shipped kernel maps block b to tile b, so every in-flight block sits in
// one ~16 MiB window of each operand and the two read streams meet the HBM
// channels in lock-step.  Variants keep the shipped tile body (U = 4 grouped
// nt loads, nt stores, 256 threads) and only permute block -> tile:
//   0 linear       t = b (shipped)
//   1 xcd8         t = (b % 8) * T/8 + b / 8   (8 windows, one per XCD group)
//   2 halves       t = (b % 2) * T/2 + b / 2
//   3 scatter      t = b * S mod T, S odd ~ 0.618 T (in-flight tiles spread over the buffer)
//   4 split64      t = (b % 64) * T/64 + b / 64
//   5 ends         even b from the front, odd b from the back
// Placements: two separate 1 GiB allocations, and one slab with `in` at
// +0 / +4 KiB / +64 KiB / +2 MiB behind `inout` (the slow ones in
// profiles/r02_split_offsets.jsonl).  Launches interleaved, 6 rounds x 10.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Impich_amd/csrc -Iinclude \
//        -o tools/bin/tile_map_probe tools/tile_map_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "redop_kernels.h"

using namespace mpix;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int NV = 6;
constexpr int U = 4;
constexpr int NT = 256;

template <int M> __device__ __forceinline__ uint64_t tile_of(uint64_t b, uint64_t T)
{
    if constexpr (M == 0)
        return b;
    else if constexpr (M == 1)
        return (b & 7) * (T >> 3) + (b >> 3);
    else if constexpr (M == 2)
        return (b & 1) * (T >> 1) + (b >> 1);
    else if constexpr (M == 3)
        return (b * ((T * 618 / 1000) | 1)) & (T - 1);
    else if constexpr (M == 4)
        return (b & 63) * (T >> 6) + (b >> 6);
    else
        return (b & 1) ? T - 1 - (b >> 1) : (b >> 1);
}

// T = gridDim.x tiles of NT * U packets, T a power of two (checked on the host)
template <int M>
__global__ void __launch_bounds__(NT) k_map(const float *__restrict__ in, float *__restrict__ io)
{
    const v4u *__restrict__ vin = reinterpret_cast<const v4u *>(in);
    v4u *__restrict__ vio = reinterpret_cast<v4u *>(io);
    const uint64_t t = tile_of<M>(blockIdx.x, gridDim.x);
    const uint64_t i = t * (NT * U) + threadIdx.x;
    v4u a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        a[u] = ld16<true>(vio + i + u * NT);
#pragma unroll
    for (int u = 0; u < U; ++u)
        b[u] = ld16<true>(vin + i + u * NT);
    const Params prm{};
#pragma unroll
    for (int u = 0; u < U; ++u)
        st16<true>(vio + i + u * NT, combine16<FSum<float>>(a[u], b[u], prm));
}

static void launch(int v, const float *in, float *io, uint64_t n, hipStream_t s)
{
    const unsigned T = (unsigned) (n / 4 / (NT * U));
    switch (v) {
        case 0: hipLaunchKernelGGL(k_map<0>, dim3(T), dim3(NT), 0, s, in, io); break;
        case 1: hipLaunchKernelGGL(k_map<1>, dim3(T), dim3(NT), 0, s, in, io); break;
        case 2: hipLaunchKernelGGL(k_map<2>, dim3(T), dim3(NT), 0, s, in, io); break;
        case 3: hipLaunchKernelGGL(k_map<3>, dim3(T), dim3(NT), 0, s, in, io); break;
        case 4: hipLaunchKernelGGL(k_map<4>, dim3(T), dim3(NT), 0, s, in, io); break;
        default: hipLaunchKernelGGL(k_map<5>, dim3(T), dim3(NT), 0, s, in, io); break;
    }
}

static double timeit(int v, const float *in, float *io, uint64_t n, hipStream_t s)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch(v, in, io, n, s);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 10; ++r)
        launch(v, in, io, n, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / 10;
}

__global__ void fill(float *p, uint64_t n, uint32_t seed)
{
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t) i * 2654435761u ^ seed;
        x ^= x >> 13;
        p[i] = (float) (x & 0xffff) / 65536.0f - 0.5f;
    }
}

int main()
{
    const uint64_t N = 1ull << 28;
    const uint64_t T = N / 4 / (NT * U);
    if (T & (T - 1)) {
        fprintf(stderr, "tile count %llu is not a power of two\n", (unsigned long long) T);
        return 1;
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x, *y, *ref, *slab;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y, N * 4));
    CK(hipMalloc(&ref, N * 4));
    CK(hipMalloc(&slab, 2 * N * 4 + (4 << 20)));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, x, N, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, ref, N, 2u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, slab, 2 * N + (1 << 20), 3u);
    CK(hipStreamSynchronize(s));
    // every mapping is a permutation of the tiles: one launch of each from the
    // same state must give the same bits as the linear one
    bool ok = true;
    {
        std::vector<float> h0(N), h1(N);
        CK(hipMemcpyAsync(y, ref, N * 4, hipMemcpyDeviceToDevice, s));
        launch(0, x, y, N, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h0.data(), y, N * 4, hipMemcpyDeviceToHost));
        for (int v = 1; v < NV; ++v) {
            CK(hipMemcpyAsync(y, ref, N * 4, hipMemcpyDeviceToDevice, s));
            launch(v, x, y, N, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h1.data(), y, N * 4, hipMemcpyDeviceToHost));
            ok = ok && memcmp(h0.data(), h1.data(), N * 4) == 0;
        }
    }
    struct P { const char *name; const float *in; float *io; };
    std::vector<P> ps = {{"separate", x, y},
                         {"slab+0", slab + N, slab},
                         {"slab+4KiB", slab + N + 1024, slab},
                         {"slab+64KiB", slab + N + 16384, slab},
                         {"slab+2MiB", slab + N + (1 << 19), slab}};
    const char *names[NV] = {"linear", "xcd8", "halves", "scatter", "split64", "ends"};
    printf("{\"ok\": %s", ok ? "true" : "false");
    for (auto &p : ps) {
        double t[NV] = {};
        for (int r = 0; r < 6; ++r)
            for (int v = 0; v < NV; ++v)
                t[v] += timeit(v, p.in, p.io, N, s);
        printf(", \"%s\": {", p.name);
        for (int v = 0; v < NV; ++v)
            printf("%s\"%s_ms\": %.4f", v ? ", " : "", names[v], t[v] / 6);
        printf("}");
        fflush(stdout);
    }
    printf("}\n");
    return ok ? 0 : 1;
}
