// stagger_probe.hip -- does de-correlating the two read streams help the
// placements where the combine runs slow (DRAM credit stalls,
// profiles/r02_split_rootcause.json)?  fp32 SUM, 1 GiB operands.
//   V0  the shipped shape: block b reads in[b] and io[b] (16 KiB tiles,
//       U = 4 packets per lane, non-temporal), combines, stores io[b]
//   V1  cross-half: block b owns tile b of the first half and tile b of the
//       second half; it issues in[A] with io[B] first and io[A] with in[B]
//       second, so the pairs in flight together are never the same index
//   V2  V0 with all `in` loads issued before all `io` loads (order only)
//   V3  V0 with all `io` loads issued before all `in` loads
// Operands: separate 1 GiB allocations, and one slab with `in` at 1 GiB +
// {0, 4 KiB, 64 KiB} from io.  Every variant's result is checked against V0's.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/stagger_probe tools/stagger_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int U = 4, T = 256;

__global__ void __launch_bounds__(256) v0(const f4 *__restrict__ in, f4 *__restrict__ io, uint64_t n4)
{
    uint64_t i = (uint64_t) blockIdx.x * T * U + threadIdx.x;
    f4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4) {
            a[u] = __builtin_nontemporal_load(io + i + u * T);
            b[u] = __builtin_nontemporal_load(in + i + u * T);
        }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            __builtin_nontemporal_store(a[u] + b[u], io + i + u * T);
}

__global__ void __launch_bounds__(256) v2(const f4 *__restrict__ in, f4 *__restrict__ io, uint64_t n4)
{
    uint64_t i = (uint64_t) blockIdx.x * T * U + threadIdx.x;
    f4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            b[u] = __builtin_nontemporal_load(in + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            a[u] = __builtin_nontemporal_load(io + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            __builtin_nontemporal_store(a[u] + b[u], io + i + u * T);
}

__global__ void __launch_bounds__(256) v3(const f4 *__restrict__ in, f4 *__restrict__ io, uint64_t n4)
{
    uint64_t i = (uint64_t) blockIdx.x * T * U + threadIdx.x;
    f4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            a[u] = __builtin_nontemporal_load(io + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            b[u] = __builtin_nontemporal_load(in + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * T < n4)
            __builtin_nontemporal_store(a[u] + b[u], io + i + u * T);
}

// n4 a multiple of 2 * T * U (1 GiB is)
__global__ void __launch_bounds__(256) v1(const f4 *__restrict__ in, f4 *__restrict__ io, uint64_t n4)
{
    const uint64_t half = n4 / 2;
    const uint64_t A = (uint64_t) blockIdx.x * T * U + threadIdx.x, B = A + half;
    f4 inA[U], ioB[U], ioA[U], inB[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        inA[u] = __builtin_nontemporal_load(in + A + u * T);
        ioB[u] = __builtin_nontemporal_load(io + B + u * T);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        ioA[u] = __builtin_nontemporal_load(io + A + u * T);
        inB[u] = __builtin_nontemporal_load(in + B + u * T);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        __builtin_nontemporal_store(ioA[u] + inA[u], io + A + u * T);
        __builtin_nontemporal_store(ioB[u] + inB[u], io + B + u * T);
    }
}

__global__ void fill(float *p, uint64_t n, uint32_t seed)
{
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t) i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        p[i] = (float) (x & 0xffff) / 65536.0f - 0.5f;
    }
}

static float run(int v, const float *in, float *io, uint64_t n, hipStream_t s)
{
    uint64_t n4 = n / 4;
    if (v == 1)
        hipLaunchKernelGGL(v1, dim3((unsigned) (n4 / 2 / (T * U))), dim3(T), 0, s, (const f4 *) in,
                           (f4 *) io, n4);
    else if (v == 3)
        hipLaunchKernelGGL(v3, dim3((unsigned) (n4 / (T * U))), dim3(T), 0, s, (const f4 *) in,
                           (f4 *) io, n4);
    else if (v == 2)
        hipLaunchKernelGGL(v2, dim3((unsigned) (n4 / (T * U))), dim3(T), 0, s, (const f4 *) in,
                           (f4 *) io, n4);
    else
        hipLaunchKernelGGL(v0, dim3((unsigned) (n4 / (T * U))), dim3(T), 0, s, (const f4 *) in,
                           (f4 *) io, n4);
    return 0.f;
}

static double timeit(int v, const float *in, float *io, uint64_t n, hipStream_t s, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    run(v, in, io, n, s);
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r)
        run(v, in, io, n, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

int main()
{
    const uint64_t N = 1ull << 28;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // correctness: every variant = V0 on the same inputs
    float *x, *y0, *y1;
    CK(hipMalloc(&x, N * 4));
    CK(hipMalloc(&y0, N * 4));
    CK(hipMalloc(&y1, N * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, x, N, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, y0, N, 2u);
    CK(hipStreamSynchronize(s));
    bool ok = true;
    for (int v = 1; v <= 3; ++v) {
        CK(hipMemcpy(y1, y0, N * 4, hipMemcpyDeviceToDevice));
        std::vector<float> h0(1 << 20), h1(1 << 20);
        CK(hipMemcpy(y1, y0, N * 4, hipMemcpyDeviceToDevice));
        float *yy;
        CK(hipMalloc(&yy, N * 4));
        CK(hipMemcpy(yy, y0, N * 4, hipMemcpyDeviceToDevice));
        CK(hipDeviceSynchronize());     // D2D hipMemcpy is asynchronous to the host
        run(0, x, yy, N, s);
        run(v, x, y1, N, s);
        CK(hipStreamSynchronize(s));
        for (uint64_t off : {(uint64_t) 0, N / 2 - (1 << 20), N - (1 << 20)}) {
            CK(hipMemcpy(h0.data(), yy + off, 4 << 20, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h1.data(), y1 + off, 4 << 20, hipMemcpyDeviceToHost));
            ok = ok && memcmp(h0.data(), h1.data(), 4 << 20) == 0;
        }
        CK(hipFree(yy));
    }
    CK(hipFree(y1));
    // placements: separate, and slab offsets
    float *slab;
    CK(hipMalloc(&slab, 3 * N * 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, slab, 3 * N, 3u);
    CK(hipStreamSynchronize(s));
    struct P { const char *name; const float *in; float *io; };
    std::vector<P> ps = {{"separate", x, y0},
                         {"slab+0", slab + N, slab},
                         {"slab+4KiB", slab + N + 1024, slab},
                         {"slab+64KiB", slab + N + 16384, slab}};
    printf("{\"ok\": %s", ok ? "true" : "false");
    for (auto &p : ps) {
        double best[4] = {1e9, 1e9, 1e9, 1e9}, sum[4] = {0, 0, 0, 0};
        const int rounds = 5;
        for (int r = 0; r < rounds; ++r)
            for (int v = 0; v < 4; ++v) {
                double t = timeit(v, p.in, p.io, N, s, 10);
                best[v] = std::min(best[v], t);
                sum[v] += t;
            }
        printf(", \"%s\": {\"v0_ms\": %.4f, \"v1_ms\": %.4f, \"v2_ms\": %.4f, \"v3_ms\": %.4f, "
               "\"v0_min\": %.4f, \"v1_min\": %.4f, \"v2_min\": %.4f, \"v3_min\": %.4f}",
               p.name, sum[0] / rounds, sum[1] / rounds, sum[2] / rounds, sum[3] / rounds,
               best[0], best[1], best[2], best[3]);
    }
    printf("}\n");
    return ok ? 0 : 1;
}
