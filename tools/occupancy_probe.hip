// occupancy_probe.hip -- do the ALU-heavier combiners lose to occupancy?
//
// The shipped k_contig (redop_kernels.h) needs 62-64 VGPRs for most
// combiners (8 waves per SIMD) but 71-74 for fp16 MAX/MIN, bf16 SUM, fp16
// complex PROD and fp32 complex PROD (7 waves), the rows that trail the 1 GiB
// per-type table.  This probe times, in one process and interleaved, the
// shipped kernel against a copy of its full-tile path built plain (check: it
// should match the shipped one) and with amdgpu_waves_per_eu(8) (the compiler
// then fits 64 VGPRs, spilling a few bytes to scratch).  1 GiB per operand,
// separate allocations; results checked bit-identical to the shipped kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//        -Impich_amd/csrc -Iinclude -o tools/bin/occupancy_probe tools/occupancy_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "redop_kernels.h"

using namespace mpix;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int U = 4;

// the shipped kernel's full-tile path (grouped loads, nt loads and stores);
// npk is a multiple of the tile here
#define TILE_BODY                                                                   \
    const uint64_t nt = blockDim.x;                                                 \
    const uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x;                \
    v4u a[U], b[U];                                                                 \
    _Pragma("unroll") for (int u = 0; u < U; ++u) a[u] = ld16<true>(io + i + u * nt); \
    _Pragma("unroll") for (int u = 0; u < U; ++u) b[u] = ld16<true>(in + i + u * nt); \
    _Pragma("unroll") for (int u = 0; u < U; ++u)                                   \
        st16<true>(io + i + u * nt, combine16<C>(a[u], b[u], prm));

template <class C>
__global__ void __launch_bounds__(1024) k_plain(const v4u *__restrict__ in, v4u *__restrict__ io,
                                                Params prm)
{
    TILE_BODY
}

template <class C>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8)))
k_occ8(const v4u *__restrict__ in, v4u *__restrict__ io, Params prm)
{
    TILE_BODY
}

template <class C>
static void launch(int v, const void *in, void *io, uint64_t bytes, hipStream_t s)
{
    using T = typename C::unit;
    const uint64_t npk = bytes / 16, tiles = npk / (256 * U);
    Params prm{};
    prm.ftrue = 1;
    const v4u *vin = static_cast<const v4u *>(in);
    v4u *vio = static_cast<v4u *>(io);
    if (v == 0)
        hipLaunchKernelGGL((k_contig<C, U, true, true, true, true>), dim3((unsigned) tiles), dim3(256),
                           0, s, static_cast<const T *>(in), static_cast<T *>(io), 0, npk,
                           npk * (16 / sizeof(T)), 0u, prm, (uint32_t) tiles, 256u);
    else if (v == 1)
        hipLaunchKernelGGL(k_plain<C>, dim3((unsigned) tiles), dim3(256), 0, s, vin, vio, prm);
    else
        hipLaunchKernelGGL(k_occ8<C>, dim3((unsigned) tiles), dim3(256), 0, s, vin, vio, prm);
}

template <class C>
static double timeit(int v, const void *in, void *io, uint64_t bytes, hipStream_t s)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch<C>(v, in, io, bytes, s);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 10; ++r)
        launch<C>(v, in, io, bytes, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / 10;
}

// small finite values in every 16-bit / 32-bit lane pattern the combiners read
__global__ void fill(uint32_t *p, uint64_t n, uint32_t seed)
{
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t) i * 2654435761u ^ seed;
        x ^= x >> 13;
        p[i] = (x & 0x3bff3bffu);   // fp16 halves below 1.0; fp32 / bf16 finite
    }
}

template <class C>
static bool run(const char *name, void *x, void *y, void *y2, void *y3, uint64_t bytes,
                hipStream_t s, bool first)
{
    // bit identity of the three kernels from the same inputs
    CK(hipMemcpyAsync(y2, y, bytes, hipMemcpyDeviceToDevice, s));
    CK(hipMemcpyAsync(y3, y, bytes, hipMemcpyDeviceToDevice, s));
    launch<C>(1, x, y2, bytes, s);
    launch<C>(2, x, y3, bytes, s);
    launch<C>(0, x, y, bytes, s);
    CK(hipStreamSynchronize(s));
    std::vector<char> h1(4 << 20), h2(4 << 20), h3(4 << 20);
    bool ok = true;
    for (uint64_t off : {(uint64_t) 0, bytes / 2, bytes - (4 << 20)}) {
        CK(hipMemcpy(h1.data(), (char *) y + off, 4 << 20, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), (char *) y2 + off, 4 << 20, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h3.data(), (char *) y3 + off, 4 << 20, hipMemcpyDeviceToHost));
        ok = ok && !memcmp(h1.data(), h2.data(), 4 << 20) && !memcmp(h1.data(), h3.data(), 4 << 20);
    }
    double t[3] = {0, 0, 0};
    for (int r = 0; r < 6; ++r)
        for (int v = 0; v < 3; ++v)
            t[v] += timeit<C>(v, x, y, bytes, s);
    printf("%s\"%s\": {\"bit_identical\": %s, \"shipped_ms\": %.4f, \"plain_copy_ms\": %.4f, "
           "\"waves8_ms\": %.4f}", first ? "" : ", ", name, ok ? "true" : "false", t[0] / 6,
           t[1] / 6, t[2] / 6);
    fflush(stdout);
    return ok;
}

int main()
{
    const uint64_t B = 1ull << 30;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void *x, *y, *y2, *y3;
    CK(hipMalloc(&x, B));
    CK(hipMalloc(&y, B));
    CK(hipMalloc(&y2, B));
    CK(hipMalloc(&y3, B));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, (uint32_t *) x, B / 4, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, (uint32_t *) y, B / 4, 2u);
    CK(hipStreamSynchronize(s));
    bool ok = true;
    printf("{");
    ok &= run<FSum<float>>("fp32_sum", x, y, y2, y3, B, s, true);
    ok &= run<FMax<_Float16>>("fp16_max", x, y, y2, y3, B, s, false);
    ok &= run<Bf16Sum>("bf16_sum", x, y, y2, y3, B, s, false);
    ok &= run<CProdHalf>("fp16_complex_prod", x, y, y2, y3, B, s, false);
    ok &= run<CProdAnnexG<float>>("fp32_complex_prod", x, y, y2, y3, B, s, false);
    printf("}\n");
    return ok ? 0 : 1;
}
