// skew_probe.hip -- can a time skew between the two read streams move the
// contiguous combine out of the slow placement mode?
//
// DESIGN.md ("The per-process 0.50 / 0.52 ms split") traced the slow mode to
// HBM credit stalls that depend on where the inout and in streams sit
// physically relative to each other while both are read in lock step.  The
// shipped kernel (k_contig<FSum<float>, 4, NT, NT>, one 16 KiB tile per
// workgroup) keeps the two streams at the same offset.  The variants here keep
// the same tile body and packet loads but run a persistent grid whose lanes
// load the `in` packets of their NEXT tile while combining the current one, so
// the `in` stream leads the `inout` stream by one grid of tiles (G x 16 KiB):
//   0  shipped kernel (grid = tiles)
//   1  persistent grid G = 2048, no lead (grid-stride baseline)
//   2  G = 2048, `in` leads by one grid (32 MiB)
//   3  G = 1024, `in` leads by one grid (16 MiB)
//   4  G = 2048, `inout` leads by one grid
// Every variant is checked bit-identical to the shipped one first.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Impich_amd/csrc -Iinclude \
//        -o tools/bin/skew_probe tools/skew_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "redop_kernels.h"

using namespace mpix;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

using C = FSum<float>;
constexpr int U = 4;
constexpr int NT = 256;

// persistent tile loop; LEAD 0: none, 1: `in` of the next tile preloaded,
// 2: `inout` of the next tile preloaded.  npk is a multiple of the tile.
template <int LEAD>
__global__ void __launch_bounds__(NT) k_skew(const v4u *__restrict__ in, v4u *__restrict__ io,
                                             uint64_t ntiles, Params prm)
{
    const uint64_t G = gridDim.x;
    uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;
    v4u nx[U];
    if constexpr (LEAD != 0) {
        const v4u *src = LEAD == 1 ? in : io;
#pragma unroll
        for (int u = 0; u < U; ++u)
            nx[u] = ld16<true>(src + t * (NT * U) + threadIdx.x + u * NT);
    }
    for (; t < ntiles; t += G) {
        const uint64_t i = t * (NT * U) + threadIdx.x;
        v4u a[U], b[U];
        if constexpr (LEAD == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                a[u] = ld16<true>(io + i + u * NT);
#pragma unroll
            for (int u = 0; u < U; ++u)
                b[u] = ld16<true>(in + i + u * NT);
        } else {
            const bool more = t + G < ntiles;
            const uint64_t j = (t + G) * (NT * U) + threadIdx.x;
            const v4u *other = LEAD == 1 ? io : in;
            const v4u *lead = LEAD == 1 ? in : io;
            v4u cur[U], oth[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cur[u] = nx[u];
                oth[u] = ld16<true>(other + i + u * NT);
            }
            if (more) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    nx[u] = ld16<true>(lead + j + u * NT);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a[u] = LEAD == 1 ? oth[u] : cur[u];
                b[u] = LEAD == 1 ? cur[u] : oth[u];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            st16<true>(io + i + u * NT, combine16<C>(a[u], b[u], prm));
    }
}

static void launch(int v, const float *in, float *io, uint64_t n, hipStream_t s)
{
    const uint64_t npk = n / 4;
    const uint64_t ntiles = npk / (NT * U);
    Params prm{};
    const v4u *vin = reinterpret_cast<const v4u *>(in);
    v4u *vio = reinterpret_cast<v4u *>(io);
    switch (v) {
        case 0:
            hipLaunchKernelGGL((k_contig<C, 4, true, true, true, true>), dim3((unsigned) ntiles),
                               dim3(NT), 0, s, in, io, 0, npk, npk * 4, 0u, prm);
            break;
        case 1:
            hipLaunchKernelGGL(k_skew<0>, dim3(2048), dim3(NT), 0, s, vin, vio, ntiles, prm);
            break;
        case 2:
            hipLaunchKernelGGL(k_skew<1>, dim3(2048), dim3(NT), 0, s, vin, vio, ntiles, prm);
            break;
        case 3:
            hipLaunchKernelGGL(k_skew<1>, dim3(1024), dim3(NT), 0, s, vin, vio, ntiles, prm);
            break;
        default:
            hipLaunchKernelGGL(k_skew<2>, dim3(2048), dim3(NT), 0, s, vin, vio, ntiles, prm);
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

constexpr int NV = 5;

int main()
{
    const uint64_t N = 1ull << 28;     // 1 GiB per operand, 16384 tiles
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x, *y, *y2, *slab;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y, N * 4));
    CK(hipMalloc(&y2, N * 4));
    CK(hipMalloc(&slab, 2 * N * 4 + (4 << 20)));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, x, N, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, y, N, 2u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, slab, 2 * N + (1 << 20), 3u);
    CK(hipStreamSynchronize(s));
    bool ok = true;
    std::vector<float> h1(1 << 20), h2(1 << 20);
    for (int v = 1; v < NV; ++v) {      // same bits as the shipped kernel
        CK(hipMemcpyAsync(y2, y, N * 4, hipMemcpyDeviceToDevice, s));
        CK(hipMemcpyAsync(slab, y, N * 4, hipMemcpyDeviceToDevice, s));
        launch(0, x, y2, N, s);
        launch(v, x, slab, N, s);
        CK(hipStreamSynchronize(s));
        for (uint64_t off : {(uint64_t) 0, N / 2 + 12345 * 4, N - (1 << 20)}) {
            CK(hipMemcpy(h1.data(), y2 + off, 4 << 20, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), slab + off, 4 << 20, hipMemcpyDeviceToHost));
            ok = ok && memcmp(h1.data(), h2.data(), 4 << 20) == 0;
        }
    }
    struct P { const char *name; const float *in; float *io; };
    std::vector<P> ps = {{"separate", x, y},
                         {"slab+0", slab + N, slab},
                         {"slab+4KiB", slab + N + 1024, slab},
                         {"slab+64KiB", slab + N + 16384, slab},
                         {"slab+2MiB", slab + N + (1 << 19), slab}};
    printf("{\"ok\": %s", ok ? "true" : "false");
    const char *names[NV] = {"shipped", "persist2048", "in_lead2048", "in_lead1024",
                             "inout_lead2048"};
    for (auto &p : ps) {
        double t[NV] = {0};
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
