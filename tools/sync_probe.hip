// tools/sync_probe.hip -- completion-wait variants for the synchronous
// MPIX_Reduce_local, timed per call (median) for a 1-element and a 1 GiB
// fp32 SUM of the shipped packet kernel:
//   wv       launch, hipStreamWriteValue32 to a pinned host word, spin on it (shipped)
//   ext      hipExtLaunchKernelGGL with a stop event in the dispatch itself,
//            spin on hipEventQuery
//   extsync  the same, hipEventSynchronize
//   ev       launch, hipEventRecord, spin on hipEventQuery
//   kflag    a plain element-wise kernel whose last block (device-scope counter)
//            stores the sequence number to the pinned word itself, against
//            the same kernel followed by hipStreamWriteValue32 (kwv)
// Usage: sync_probe [reps_small=2000] [reps_big=50]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <functional>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
using C = FSum<float>;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_plain(const float *in, float *io, uint64_t n)
{
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x)
        io[i] += in[i];
}

__global__ void k_flag(const float *in, float *io, uint64_t n, uint32_t *flag, uint32_t *counter,
                       uint32_t seq)
{
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x)
        io[i] += in[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        uint32_t old = atomicAdd(counter, 1u);
        if (old == gridDim.x - 1) {
            *counter = 0;
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double med_us(const std::function<void()> &f, int reps)
{
    std::vector<double> t;
    f();
    for (int i = 0; i < reps; ++i) {
        auto a = std::chrono::steady_clock::now();
        f();
        auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv)
{
    int reps_small = argc > 1 ? atoi(argv[1]) : 2000;
    int reps_big = argc > 2 ? atoi(argv[2]) : 50;
    const uint64_t n = 1ull << 28;
    float *a, *b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev, stop;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&stop, hipEventDisableTiming));
    volatile uint32_t *flag = nullptr;
    CK(hipHostMalloc((void **) &flag, 64, hipHostMallocCoherent));
    *flag = 0;
    uint32_t seq = 0;
    const Params prm{1, 0};

    uint32_t *counter;
    CK(hipMalloc(&counter, 4));
    CK(hipMemset(counter, 0, 4));
    for (uint64_t count : {(uint64_t) 1, (uint64_t) 4096, (uint64_t) 65536, (uint64_t) 1 << 20}) {
        const unsigned g = (unsigned) std::min<uint64_t>((count + 1023) / 1024, 1024);
        double t_kwv = med_us([&] {
            ++seq;
            hipLaunchKernelGGL(k_plain, dim3(g), dim3(256), 0, s, b, a, count);
            hipStreamWriteValue32(s, (void *) flag, seq, 0);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
            }
        }, reps_small);
        double t_kflag = med_us([&] {
            ++seq;
            hipLaunchKernelGGL(k_flag, dim3(g), dim3(256), 0, s, b, a, count, (uint32_t *) flag,
                               counter, seq);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
            }
        }, reps_small);
        CK(hipStreamSynchronize(s));
        printf("plain kernel count %llu grid %u: kwv %.1f us  kflag %.1f us\n",
               (unsigned long long) count, g, t_kwv, t_kflag);
    }
    for (uint64_t count : {(uint64_t) 4, n}) {
        const uint64_t npk = count / 4;
        const unsigned grid = grid_for(256ull * 4, npk, 0);
        auto launch = [&] {
            hipLaunchKernelGGL((k_contig<C, 4, true, true>), dim3(grid), dim3(256), 0, s, b, a,
                               (uint64_t) 0, npk, npk * 4, (uint32_t) 0, prm);
        };
        auto ext = [&] {
            hipExtLaunchKernelGGL((k_contig<C, 4, true, true>), dim3(grid), dim3(256), 0, s,
                                  nullptr, stop, 0, (const float *) b, a, (uint64_t) 0, npk,
                                  npk * 4, (uint32_t) 0, prm);
        };
        int reps = count == n ? reps_big : reps_small;
        double t_wv = med_us([&] {
            ++seq;
            launch();
            hipStreamWriteValue32(s, (void *) flag, seq, 0);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
            }
        }, reps);
        double t_ext = med_us([&] {
            ext();
            while (hipEventQuery(stop) == hipErrorNotReady) {
            }
        }, reps);
        double t_extsync = med_us([&] {
            ext();
            hipEventSynchronize(stop);
        }, reps);
        double t_ev = med_us([&] {
            launch();
            hipEventRecord(ev, s);
            while (hipEventQuery(ev) == hipErrorNotReady) {
            }
        }, reps);
        // kernel alone, back to back, for reference
        CK(hipStreamSynchronize(s));
        auto k0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i)
            launch();
        CK(hipStreamSynchronize(s));
        auto k1 = std::chrono::steady_clock::now();
        double t_async = std::chrono::duration<double, std::micro>(k1 - k0).count() / reps;
        printf("count %llu: wv %.1f us  ext+query %.1f us  ext+sync %.1f us  ev %.1f us  "
               "(back-to-back async %.1f us/launch)\n", (unsigned long long) count, t_wv, t_ext,
               t_extsync, t_ev, t_async);
    }
    CK(hipStreamSynchronize(s));
    return 0;
}
