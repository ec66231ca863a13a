// bench_triad.hip -- measurement helper, not part of the product library.
// STREAM triad a[i] = b[i] + q*c[i] on fp32 with 16-byte loads/stores: the
// denominator BASELINE.json asks for ("fraction of a measured stream triad
// on the same GPU").  Same traffic shape as the local reduction (2 reads +
// 1 write per element) but three distinct arrays, as STREAM defines it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <time.h>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(1))) f4 gf4;

// xcd_mask: the blocks on these XCDs (HW_REG_XCC_ID) store write-through
// (sc0 sc1), the rest non-temporally -- the library's store policy, so the
// triad can be read with and without it (0: the plain STREAM triad)
template <int U>
__global__ void __launch_bounds__(256) k_triad(f4 *__restrict__ a, const f4 *__restrict__ b,
                                               const f4 *__restrict__ c, float q, uint64_t n4,
                                               unsigned xcd_mask)
{
    const uint64_t nt = blockDim.x;
    uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x;
    bool wt = false;
    if (xcd_mask) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        wt = (xcd_mask >> (x & 7)) & 1;
    }
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * nt < n4) {
            x[u] = __builtin_nontemporal_load(b + i + u * nt);
            y[u] = __builtin_nontemporal_load(c + i + u * nt);
        }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i + u * nt < n4) {
            if (wt)
                *(volatile gf4 *) (gf4 *) (a + i + u * nt) = x[u] + q * y[u];
            else
                __builtin_nontemporal_store(x[u] + q * y[u], a + i + u * nt);
        }
}

extern "C" int mpix_bench_triad_xcd(float *a, const float *b, const float *c, float q, uint64_t n,
                                    void *stream, unsigned xcd_mask)
{
    if (n % 4 || ((uintptr_t) a | (uintptr_t) b | (uintptr_t) c) % 16)
        return 12;
    uint64_t n4 = n / 4;
    const int U = 4, T = 256;
    uint64_t grid = (n4 + (uint64_t) T * U - 1) / ((uint64_t) T * U);
    if (grid == 0)
        grid = 1;
    hipLaunchKernelGGL((k_triad<U>), dim3((unsigned) grid), dim3(T), 0, (hipStream_t) stream,
                       (f4 *) a, (const f4 *) b, (const f4 *) c, q, n4, xcd_mask & 0xffu);
    return hipGetLastError() == hipSuccess ? 0 : 15;
}

extern "C" int mpix_bench_triad(float *a, const float *b, const float *c, float q, uint64_t n,
                                void *stream)
{
    return mpix_bench_triad_xcd(a, b, c, q, n, stream, 0);
}

// Per-call host time of a synchronous reduce entry point (passed as a
// function pointer, e.g. MPIX_Reduce_local), median over `reps` calls after
// one warm-up, timed in C so the figure carries no binding overhead.
typedef int (*sync_reduce_fn)(const void *, void *, int64_t, int, int);

extern "C" int mpix_bench_call_latency(void *fn, const void *in, void *io, int64_t count, int dt,
                                       int op, int reps, double *median_us, double *p90_us)
{
    if (!fn || reps < 1 || !median_us || !p90_us)
        return 12;
    sync_reduce_fn f = (sync_reduce_fn) fn;
    int rc = f(in, io, count, dt, op);
    if (rc)
        return rc;
    std::vector<double> t(reps);
    for (int i = 0; i < reps; ++i) {
        auto a = std::chrono::steady_clock::now();
        rc = f(in, io, count, dt, op);
        auto b = std::chrono::steady_clock::now();
        if (rc)
            return rc;
        t[i] = std::chrono::duration<double, std::micro>(b - a).count();
    }
    std::sort(t.begin(), t.end());
    *median_us = t[reps / 2];
    *p90_us = t[(reps * 9) / 10];
    return 0;
}

// `reps` back-to-back calls of a synchronous reduce entry point (the headline
// loop of bench.py: one MPIX_Reduce_local per step, issued from C as MPICH
// issues it, so no binding overhead sits between the calls); *total_s is the
// wall time of the whole loop.
extern "C" int mpix_bench_call_loop(void *fn, const void *in, void *io, int64_t count, int dt,
                                    int op, int reps, double *total_s)
{
    if (!fn || reps < 0 || !total_s)
        return 12;
    sync_reduce_fn f = (sync_reduce_fn) fn;
    auto a = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) {
        int rc = f(in, io, count, dt, op);
        if (rc)
            return rc;
    }
    auto b = std::chrono::steady_clock::now();
    *total_s = std::chrono::duration<double>(b - a).count();
    return 0;
}

// The same loop with every call's host entry and return stamped (CLOCK_MONOTONIC
// and CLOCK_BOOTTIME ns, t[4*i + 0..3] = mono in, mono out, boot in, boot out),
// to line the calls up with a rocprofv3 kernel trace (tools/sync_gap.py)
extern "C" int mpix_bench_call_loop_ts(void *fn, const void *in, void *io, int64_t count, int dt,
                                       int op, int reps, uint64_t *t)
{
    if (!fn || reps < 0 || !t)
        return 12;
    sync_reduce_fn f = (sync_reduce_fn) fn;
    auto ns = [](clockid_t c) {
        struct timespec ts;
        clock_gettime(c, &ts);
        return (uint64_t) ts.tv_sec * 1000000000ull + (uint64_t) ts.tv_nsec;
    };
    for (int i = 0; i < reps; ++i) {
        t[4 * i + 0] = ns(CLOCK_MONOTONIC);
        t[4 * i + 2] = ns(CLOCK_BOOTTIME);
        int rc = f(in, io, count, dt, op);
        t[4 * i + 1] = ns(CLOCK_MONOTONIC);
        t[4 * i + 3] = ns(CLOCK_BOOTTIME);
        if (rc)
            return rc;
    }
    return 0;
}

// The chunked regime of a pipelined collective (one combine per arriving
// chunk), issued from C: `count` elements of `elem_size` bytes cut into
// chunks of `chunk` elements, each enqueued through the stream-ordered entry
// point (e.g. MPIX_Reduce_local_async) back to back on `stream`, timed from
// the first issue to the stream draining.  *issue_s is the host time of the
// issue loop alone (per-call launch cost), *total_s the whole interval.
typedef int (*async_reduce_fn)(const void *, void *, int64_t, int, int, void *);

extern "C" int mpix_bench_chunked_async(void *fn, const void *in, void *io, int64_t count,
                                        int64_t chunk, int elem_size, int dt, int op, void *stream,
                                        double *issue_s, double *total_s)
{
    if (!fn || chunk < 1 || count < chunk || elem_size < 1 || !issue_s || !total_s)
        return 12;
    async_reduce_fn f = (async_reduce_fn) fn;
    hipStream_t s = (hipStream_t) stream;
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    const int64_t nch = count / chunk;
    auto a = std::chrono::steady_clock::now();
    for (int64_t k = 0; k < nch; ++k) {
        const int64_t off = k * chunk * elem_size;
        int rc = f((const char *) in + off, (char *) io + off, chunk, dt, op, stream);
        if (rc)
            return rc;
    }
    auto b = std::chrono::steady_clock::now();
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    auto c = std::chrono::steady_clock::now();
    *issue_s = std::chrono::duration<double>(b - a).count();
    *total_s = std::chrono::duration<double>(c - a).count();
    return 0;
}

__global__ void k_empty(int *p)
{
    if (p && threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345)
        p[1] = 0;
}

struct Args72 {
    uint64_t w[9];
};

__global__ void k_empty72(const float *a, float *b, uint64_t c, uint64_t d, uint64_t e,
                          uint32_t f, Args72 g)
{
    if (a && threadIdx.x == 0 && blockIdx.x == 0 && f == 12345u && g.w[0] == c + d + e)
        b[0] = a[0];
}

// Where the per-call host cost of an asynchronous reduce goes: mean host
// microseconds of (0) hipPointerGetAttributes on a device pointer, (1)
// hipPointerGetAttribute(MEMORY_TYPE), (2) issuing an empty kernel
// back to back, (3) issuing `fn` (MPIX_Reduce_local_async) back to back at
// `count`, (4) an empty kernel + hipStreamSynchronize round trip, (5) `fn` +
// hipStreamSynchronize round trip, (6) issuing an empty kernel with the
// contiguous kernel's 112-byte argument block.  out[7] holds the figures.
extern "C" int mpix_bench_launch_floor(void *fn, const void *in, void *io, int64_t count, int dt,
                                       int op, void *stream, int reps, double *out)
{
    if (!fn || reps < 1 || !out)
        return 12;
    async_reduce_fn f = (async_reduce_fn) fn;
    hipStream_t s = (hipStream_t) stream;
    using clk = std::chrono::steady_clock;
    auto us = [&](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count() / reps;
    };
    hipPointerAttribute_t attr;
    auto a = clk::now();
    for (int i = 0; i < reps; ++i)
        if (hipPointerGetAttributes(&attr, io) != hipSuccess)
            return 15;
    out[0] = us(a, clk::now());
    unsigned int mt = 0;
    a = clk::now();
    for (int i = 0; i < reps; ++i)
        if (hipPointerGetAttribute(&mt, HIP_POINTER_ATTRIBUTE_MEMORY_TYPE, (hipDeviceptr_t) io) !=
            hipSuccess)
            return 15;
    out[1] = us(a, clk::now());
    for (int pass = 0; pass < 2; ++pass) {      // pass 0 warms the launch path up
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
        a = clk::now();
        for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (int *) nullptr);
        out[2] = us(a, clk::now());
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
        a = clk::now();
        for (int i = 0; i < reps; ++i)
            if (int rc = f(in, io, count, dt, op, stream))
                return rc;
        out[3] = us(a, clk::now());
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
    }
    a = clk::now();
    for (int i = 0; i < reps; ++i) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (int *) nullptr);
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
    }
    out[4] = us(a, clk::now());
    a = clk::now();
    for (int i = 0; i < reps; ++i) {
        if (int rc = f(in, io, count, dt, op, stream))
            return rc;
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
    }
    out[5] = us(a, clk::now());
    Args72 g{};
    for (int pass = 0; pass < 2; ++pass) {
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
        a = clk::now();
        for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL(k_empty72, dim3(1), dim3(64), 0, s, (const float *) in, (float *) io,
                               (uint64_t) 1, (uint64_t) 2, (uint64_t) 3, 4u, g);
        out[6] = us(a, clk::now());
    }
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    return 0;
}

// Issue cost vs GPU cost of back-to-back calls, separated: calls are issued in
// bursts of `burst` (fewer than the stream's queue holds, so the host never
// waits for the GPU while issuing) and the stream is synchronised between
// bursts.  out[0]: host us per call to issue `fn` (MPIX_Reduce_local_async at
// `count`); out[1]: us per call of a whole burst including its drain; out[2],
// out[3]: the same for an empty one-block kernel; out[4 + j]: host us to issue
// an empty kernel with a j-th argument block size of kArgSizes (bytes).
template <int N> struct ArgBlock {
    uint64_t w[N / 8];
};
template <int N>
__global__ void k_empty_args(ArgBlock<N>)
{
}
template <int N>
static double issue_args_us(hipStream_t s, int burst, int rounds)
{
    ArgBlock<N> g{};
    double tot = 0;
    for (int r = 0; r < rounds; ++r) {
        if (hipStreamSynchronize(s) != hipSuccess)
            return -1;
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < burst; ++i)
            hipLaunchKernelGGL(k_empty_args<N>, dim3(1), dim3(64), 0, s, g);
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    if (hipStreamSynchronize(s) != hipSuccess)
        return -1;
    return tot / ((double) burst * rounds);
}

// An empty kernel with no kernel arguments at all: HIP skips the argument
// upload (the write to device memory and its visibility flush), so its issue
// time is the launch's own floor; issue of k_empty minus this = the upload.
__global__ void k_none() {}

extern "C" double mpix_bench_issue_noargs(void *stream, int burst, int rounds)
{
    hipStream_t s = (hipStream_t) stream;
    double tot = 0;
    for (int r = 0; r < rounds + 1; ++r) {      // round 0 warms up
        if (hipStreamSynchronize(s) != hipSuccess)
            return -1;
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < burst; ++i)
            hipLaunchKernelGGL(k_none, dim3(1), dim3(64), 0, s);
        if (r)
            tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    if (hipStreamSynchronize(s) != hipSuccess)
        return -1;
    return tot / ((double) burst * rounds);
}

// An empty kernel with k_contig's explicit argument size (104 B) that reads
// gridDim / blockDim, so its segment carries the hidden arguments too (360 B,
// as k_contig's does).
__global__ void k_empty_hidden(ArgBlock<104> g, int *p)
{
    if (p && gridDim.x == 12345u && g.w[0] == 1)
        p[0] = (int) blockDim.x;
}

// Two device pointers as plain kernel arguments, as the reduce kernels take
// their operands.
__global__ void k_empty_ptrs(const float *a, float *b)
{
    if (a == b && threadIdx.x == 0)
        b[0] = 0.f;
}

// out[0]: host us to issue an empty kernel with a 104-B argument block and no
// hidden arguments; out[1]: the same with the hidden arguments (360 B);
// out[2]: an empty kernel given the two device pointers p, q.
extern "C" int mpix_bench_issue_hidden(void *stream, int burst, int rounds, const void *p,
                                       void *q, double *out)
{
    if (burst < 1 || rounds < 1 || !out || !p || !q || p == q)
        return 12;
    hipStream_t s = (hipStream_t) stream;
    out[0] = issue_args_us<104>(s, burst, rounds);
    ArgBlock<104> g{};
    double tot = 0;
    for (int r = 0; r < rounds; ++r) {
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < burst; ++i)
            hipLaunchKernelGGL(k_empty_hidden, dim3(1), dim3(64), 0, s, g, (int *) nullptr);
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    out[1] = tot / ((double) burst * rounds);
    tot = 0;
    for (int r = 0; r < rounds; ++r) {
        if (hipStreamSynchronize(s) != hipSuccess)
            return 15;
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < burst; ++i)
            hipLaunchKernelGGL(k_empty_ptrs, dim3(1), dim3(64), 0, s, (const float *) p, (float *) q);
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
    }
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    out[2] = tot / ((double) burst * rounds);
    return out[0] < 0 ? 15 : 0;
}

// Host us per call of the HIP queries a stream-ordered reduce makes before
// its launch (redop_capi.cpp reachable()): out[0] hipPointerGetAttributes
// (made twice per call, once per operand), out[1] hipStreamGetDevice,
// out[2] hipGetLastError (once after the launch).
extern "C" int mpix_bench_query_us(const void *p, void *stream, int reps, double *out)
{
    if (!p || reps < 1 || !out)
        return 12;
    using clk = std::chrono::steady_clock;
    hipStream_t s = (hipStream_t) stream;
    hipPointerAttribute_t a;
    auto t0 = clk::now();
    for (int i = 0; i < reps; ++i)
        if (hipPointerGetAttributes(&a, p) != hipSuccess)
            return 15;
    auto t1 = clk::now();
    hipDevice_t d;
    for (int i = 0; i < reps; ++i)
        if (hipStreamGetDevice(s, &d) != hipSuccess)
            return 15;
    auto t2 = clk::now();
    int acc = 0;
    for (int i = 0; i < reps; ++i)
        acc |= (int) hipGetLastError();
    auto t3 = clk::now();
    if (acc)
        return 15;
    out[0] = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
    out[1] = std::chrono::duration<double, std::micro>(t2 - t1).count() / reps;
    out[2] = std::chrono::duration<double, std::micro>(t3 - t2).count() / reps;
    return 0;
}

extern "C" int mpix_bench_issue_burst(void *fn, const void *in, void *io, int64_t count, int dt,
                                      int op, void *stream, int burst, int rounds, double *out)
{
    if (!fn || burst < 1 || rounds < 2 || !out)
        return 12;
    async_reduce_fn f = (async_reduce_fn) fn;
    hipStream_t s = (hipStream_t) stream;
    using clk = std::chrono::steady_clock;
    for (int kind = 0; kind < 2; ++kind) {
        double issue = 0, whole = 0;
        for (int r = 0; r < rounds + 1; ++r) {      // round 0 warms up
            if (hipStreamSynchronize(s) != hipSuccess)
                return 15;
            auto a = clk::now();
            for (int i = 0; i < burst; ++i) {
                if (kind == 0) {
                    if (int rc = f(in, io, count, dt, op, stream))
                        return rc;
                } else {
                    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, (int *) nullptr);
                }
            }
            auto b = clk::now();
            if (hipStreamSynchronize(s) != hipSuccess)
                return 15;
            auto c = clk::now();
            if (r) {
                issue += std::chrono::duration<double, std::micro>(b - a).count();
                whole += std::chrono::duration<double, std::micro>(c - a).count();
            }
        }
        out[2 * kind] = issue / ((double) burst * rounds);
        out[2 * kind + 1] = whole / ((double) burst * rounds);
    }
    out[4] = issue_args_us<8>(s, burst, rounds);
    out[5] = issue_args_us<64>(s, burst, rounds);
    out[6] = issue_args_us<128>(s, burst, rounds);
    out[7] = issue_args_us<256>(s, burst, rounds);
    out[8] = issue_args_us<1024>(s, burst, rounds);
    out[9] = issue_args_us<2048>(s, burst, rounds);
    return 0;
}

// The chunked loop of mpix_bench_chunked_async, the chunks handed over
// `batch` at a time through MPIX_Reduce_local_batch_async (`fn`): what an
// engine with several ready chunks pays per chunk.
typedef int (*batch_reduce_fn)(const void *const *, void *const *, const int64_t *, int, int,
                               int, void *);
extern "C" int mpix_bench_chunked_batch(void *fn, const void *in, void *io, int64_t count,
                                        int64_t chunk, int elem_size, int dt, int op, void *stream,
                                        int batch, double *issue_s, double *total_s)
{
    if (!fn || chunk < 1 || count < chunk || elem_size < 1 || batch < 1 || batch > 64 ||
        !issue_s || !total_s)
        return 12;
    batch_reduce_fn f = (batch_reduce_fn) fn;
    hipStream_t s = (hipStream_t) stream;
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    const int64_t nch = count / chunk;
    std::vector<const void *> ins(64);
    std::vector<void *> ios(64);
    std::vector<int64_t> cnt(64, chunk);
    auto a = std::chrono::steady_clock::now();
    for (int64_t k = 0; k < nch; k += batch) {
        const int m = (int) std::min<int64_t>(batch, nch - k);
        for (int q = 0; q < m; ++q) {
            const int64_t off = (k + q) * chunk * elem_size;
            ins[q] = (const char *) in + off;
            ios[q] = (char *) io + off;
        }
        int rc = f(ins.data(), ios.data(), cnt.data(), m, dt, op, stream);
        if (rc)
            return rc;
    }
    auto b = std::chrono::steady_clock::now();
    if (hipStreamSynchronize(s) != hipSuccess)
        return 15;
    auto c = std::chrono::steady_clock::now();
    *issue_s = std::chrono::duration<double>(b - a).count();
    *total_s = std::chrono::duration<double>(c - a).count();
    return 0;
}

// A copy kernel of `blocks` workgroups (grid-stride, 16-byte packets): HBM
// traffic at a chosen fraction of the device's rate -- the stand-in for
// RCCL's point-to-point kernels (a few channels' worth of CUs writing what
// arrives over xGMI into HBM) next to a combine (tools/policy_concurrent.py).
__global__ void k_trickle(f4 *__restrict__ dst, const f4 *__restrict__ src, uint64_t n)
{
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[i];
}

extern "C" int mpix_bench_trickle_copy(void *dst, const void *src, uint64_t bytes, int blocks,
                                       void *stream)
{
    if (!dst || !src || blocks < 1 || (bytes & 15) || ((uintptr_t) dst & 15) || ((uintptr_t) src & 15))
        return 12;
    hipLaunchKernelGGL(k_trickle, dim3(blocks), dim3(256), 0, (hipStream_t) stream, (f4 *) dst,
                       (const f4 *) src, bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : 15;
}
