// contig_order_probe.hip -- in-process A/B of the shipped contiguous kernel
// (k_contig<FSum<float>, 4, NT, NT>, redop_kernels.h) with its loads
// alternating inout/in per packet (the round-1 order) against the same
// kernel issuing all inout loads, then all in loads (GRP).  fp32 SUM, 1 GiB,
// separate allocations and slab placements; launches interleaved A, B, A, B.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Impich_amd/csrc -Iinclude \
//        -o tools/bin/contig_order_probe tools/contig_order_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

using C = FSum<float>;

// variant 0: alternating U=4 (round 1), 1: grouped U=4 (shipped), 2: grouped U=8,
// 3: grouped U=2, 4: grouped U=4 with 512-thread blocks
static void launch(int v, const float *in, float *io, uint64_t n, hipStream_t s)
{
    const uint64_t npk = n / 4;
    Params prm{};
    switch (v) {
        case 0:
            hipLaunchKernelGGL((k_contig<C, 4, true, true, true, false>), dim3((unsigned) (npk / 1024)),
                               dim3(256), 0, s, in, io, 0, npk, npk * 4, 0u, prm,
                               (uint32_t) (npk / 1024), 256u);
            break;
        case 2:
            hipLaunchKernelGGL((k_contig<C, 8, true, true, true, true>), dim3((unsigned) (npk / 2048)),
                               dim3(256), 0, s, in, io, 0, npk, npk * 4, 0u, prm,
                               (uint32_t) (npk / 2048), 256u);
            break;
        case 3:
            hipLaunchKernelGGL((k_contig<C, 2, true, true, true, true>), dim3((unsigned) (npk / 512)),
                               dim3(256), 0, s, in, io, 0, npk, npk * 4, 0u, prm,
                               (uint32_t) (npk / 512), 256u);
            break;
        case 4:
            hipLaunchKernelGGL((k_contig<C, 4, true, true, true, true>), dim3((unsigned) (npk / 2048)),
                               dim3(512), 0, s, in, io, 0, npk, npk * 4, 0u, prm,
                               (uint32_t) (npk / 2048), 512u);
            break;
        default:
            hipLaunchKernelGGL((k_contig<C, 4, true, true, true, true>), dim3((unsigned) (npk / 1024)),
                               dim3(256), 0, s, in, io, 0, npk, npk * 4, 0u, prm,
                               (uint32_t) (npk / 1024), 256u);
    }
}

static double timeit(int grp, const float *in, float *io, uint64_t n, hipStream_t s)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch(grp, in, io, n, s);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 10; ++r)
        launch(grp, in, io, n, s);
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
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x, *y, *y2, *slab;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y, N * 4));
    CK(hipMalloc(&y2, N * 4));
    CK(hipMalloc(&slab, 3 * N * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, x, N, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, y, N, 2u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, slab, 3 * N, 3u);
    CK(hipStreamSynchronize(s));
    // same bits
    CK(hipMemcpyAsync(y2, y, N * 4, hipMemcpyDeviceToDevice, s));
    launch(0, x, y, N, s);
    launch(1, x, y2, N, s);
    CK(hipStreamSynchronize(s));
    std::vector<float> h1(1 << 20), h2(1 << 20);
    bool ok = true;
    for (uint64_t off : {(uint64_t) 0, N / 2, N - (1 << 20)}) {
        CK(hipMemcpy(h1.data(), y + off, 4 << 20, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), y2 + off, 4 << 20, hipMemcpyDeviceToHost));
        ok = ok && memcmp(h1.data(), h2.data(), 4 << 20) == 0;
    }
    struct P { const char *name; const float *in; float *io; };
    std::vector<P> ps = {{"separate", x, y},
                         {"slab+0", slab + N, slab},
                         {"slab+4KiB", slab + N + 1024, slab},
                         {"slab+64KiB", slab + N + 16384, slab}};
    printf("{\"ok\": %s", ok ? "true" : "false");
    const char *names[5] = {"alternating_u4", "grouped_u4", "grouped_u8", "grouped_u2",
                            "grouped_u4_b512"};
    for (auto &p : ps) {
        double t[5] = {0, 0, 0, 0, 0};
        for (int r = 0; r < 6; ++r)
            for (int v = 0; v < 5; ++v)
                t[v] += timeit(v, p.in, p.io, N, s);
        printf(", \"%s\": {", p.name);
        for (int v = 0; v < 5; ++v)
            printf("%s\"%s_ms\": %.4f", v ? ", " : "", names[v], t[v] / 6);
        printf("}");
    }
    printf("}\n");
    return ok ? 0 : 1;
}
