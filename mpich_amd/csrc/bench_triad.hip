// bench_triad.hip -- measurement helper, not part of the product library.
// STREAM triad a[i] = b[i] + q*c[i] on fp32 with 16-byte loads/stores: the
// denominator BASELINE.json asks for ("fraction of a measured stream triad
// on the same GPU").  Same traffic shape as the local reduction (2 reads +
// 1 write per element) but three distinct arrays, as STREAM defines it.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(256) k_triad(f4 *__restrict__ a, const f4 *__restrict__ b,
                                               const f4 *__restrict__ c, float q, uint64_t n4)
{
    const uint64_t nt = blockDim.x;
    uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x;
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * nt < n4) {
            x[u] = __builtin_nontemporal_load(b + i + u * nt);
            y[u] = __builtin_nontemporal_load(c + i + u * nt);
        }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * nt < n4)
            __builtin_nontemporal_store(x[u] + q * y[u], a + i + u * nt);
}

extern "C" int mpix_bench_triad(float *a, const float *b, const float *c, float q, uint64_t n,
                                void *stream)
{
    if (n % 4 || ((uintptr_t) a | (uintptr_t) b | (uintptr_t) c) % 16)
        return 12;
    uint64_t n4 = n / 4;
    const int U = 4, T = 256;
    uint64_t grid = (n4 + (uint64_t) T * U - 1) / ((uint64_t) T * U);
    if (grid == 0)
        grid = 1;
    hipLaunchKernelGGL((k_triad<U>), dim3((unsigned) grid), dim3(T), 0, (hipStream_t) stream,
                       (f4 *) a, (const f4 *) b, (const f4 *) c, q, n4);
    return hipGetLastError() == hipSuccess ? 0 : 15;
}
