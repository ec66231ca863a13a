// small_block_probe.hip -- the shipped contiguous kernel (k_contig<FSum<float>,
// U, NT, NT>, grouped loads) at block sizes below the round-1 sweep (64 and
// 128 threads, U = 4 and 8) against the shipped 256 x U=4, 1 GiB fp32 SUM,
// interleaved in one process; separate allocations and one slab (+64 KiB).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Impich_amd/csrc -Iinclude \
//        -o tools/bin/small_block_probe tools/small_block_probe.hip
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

struct V { const char *name; int block, u; };
static const V kV[] = {{"b256_u4", 256, 4}, {"b128_u4", 128, 4}, {"b128_u8", 128, 8},
                       {"b64_u4", 64, 4}, {"b64_u8", 64, 8}};
constexpr int NV = sizeof kV / sizeof kV[0];

static void launch(int v, const float *in, float *io, uint64_t n, hipStream_t s)
{
    const uint64_t npk = n / 4;
    const Params prm{};
    const unsigned grid = (unsigned) (npk / ((uint64_t) kV[v].block * kV[v].u));
    if (kV[v].u == 4)
        hipLaunchKernelGGL((k_contig<C, 4, true, true>), dim3(grid), dim3(kV[v].block), 0, s, in, io,
                           (uint64_t) 0, npk, npk * 4, 0u, prm);
    else
        hipLaunchKernelGGL((k_contig<C, 8, true, true>), dim3(grid), dim3(kV[v].block), 0, s, in, io,
                           (uint64_t) 0, npk, npk * 4, 0u, prm);
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
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x, *y, *ref, *slab;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y, N * 4));
    CK(hipMalloc(&ref, N * 4));
    CK(hipMalloc(&slab, 2 * N * 4 + (1 << 20)));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, x, N, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, ref, N, 2u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, slab, 2 * N + (1 << 18), 3u);
    CK(hipStreamSynchronize(s));
    bool ok = true;     // every geometry: the same bits as the shipped one
    {
        std::vector<float> h0(N), h1(N);
        for (int v = 0; v < NV; ++v) {
            CK(hipMemcpyAsync(y, ref, N * 4, hipMemcpyDeviceToDevice, s));
            launch(v, x, y, N, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(v ? h1.data() : h0.data(), y, N * 4, hipMemcpyDeviceToHost));
            if (v)
                ok = ok && memcmp(h0.data(), h1.data(), N * 4) == 0;
        }
    }
    struct P { const char *name; const float *in; float *io; };
    std::vector<P> ps = {{"separate", x, y}, {"slab+64KiB", slab + N + 16384, slab}};
    printf("{\"ok\": %s", ok ? "true" : "false");
    for (auto &p : ps) {
        double t[NV] = {};
        for (int r = 0; r < 8; ++r)
            for (int v = 0; v < NV; ++v)
                t[v] += timeit(v, p.in, p.io, N, s);
        printf(", \"%s\": {", p.name);
        for (int v = 0; v < NV; ++v)
            printf("%s\"%s_ms\": %.4f", v ? ", " : "", kV[v].name, t[v] / 8);
        printf("}");
    }
    printf("}\n");
    return ok ? 0 : 1;
}
