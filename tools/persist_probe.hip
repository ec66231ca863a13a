// tools/persist_probe.hip -- latency of a small synchronous fp32 SUM through a
// resident one-workgroup worker that polls a pinned host doorbell, against a
// normal launch whose kernel stores the completion word itself.
//
// Safety: the worker exits on an EXIT doorbell, and on its own once it has
// seen no work for kIdleTicks of the 100 MHz wall clock (200 ms) or polled
// kMaxPolls times in all, so no wave outlives the process even if the host
// never rings.  Progress goes to stderr unbuffered.
// Usage: persist_probe [reps=3000]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

struct Desc {
    const float *in;
    float *io;
    unsigned long long n;
};

constexpr uint32_t kExit = 0xffffffffu;
constexpr unsigned long long kIdleTicks = 20000000ull;     // 200 ms at 100 MHz
constexpr uint32_t kMaxPolls = 1u << 22;

__global__ void __launch_bounds__(256) k_worker(volatile uint32_t *bell, const Desc *desc,
                                                uint32_t *done, uint32_t *state, uint32_t start)
{
    __shared__ uint32_t s_seq;
    uint32_t last = start, polls = 0;
    if (threadIdx.x == 0)
        __hip_atomic_store(state, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t v;
            const unsigned long long t0 = wall_clock64();
            for (;;) {
                v = __hip_atomic_load((uint32_t *) bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v != last || ++polls >= kMaxPolls || wall_clock64() - t0 > kIdleTicks)
                    break;
                __builtin_amdgcn_s_sleep(1);
            }
            s_seq = (v != last) ? v : kExit;
            __hip_atomic_store(state + 1, polls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        const uint32_t seq = s_seq;
        __syncthreads();
        if (seq == kExit)
            break;
        last = seq;
        Desc d;
        d.in = (const float *) __hip_atomic_load((unsigned long long *) &desc->in, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM);
        d.io = (float *) __hip_atomic_load((unsigned long long *) &desc->io, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
        d.n = __hip_atomic_load((unsigned long long *) &desc->n, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM);
        for (unsigned long long i = threadIdx.x; i < d.n; i += blockDim.x)
            d.io[i] += d.in[i];
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(state, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(256) k_flag(const float *in, float *io, unsigned long long n,
                                              uint32_t *done, uint32_t seq)
{
    for (unsigned long long i = threadIdx.x; i < n; i += blockDim.x)
        io[i] += in[i];
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 1000;
    setvbuf(stdout, nullptr, _IONBF, 0);
    const size_t maxn = 4096;
    float *a, *b;
    CK(hipMalloc(&a, maxn * 4));
    CK(hipMalloc(&b, maxn * 4));
    std::vector<float> ones(maxn, 1.0f), back(maxn);
    CK(hipMemcpy(b, ones.data(), maxn * 4, hipMemcpyHostToDevice));
    uint32_t *bell, *done, *state;
    Desc *desc;
    CK(hipHostMalloc((void **) &bell, 64, hipHostMallocCoherent));
    CK(hipHostMalloc((void **) &done, 64, hipHostMallocCoherent));
    CK(hipHostMalloc((void **) &state, 64, hipHostMallocCoherent));
    CK(hipHostMalloc((void **) &desc, 64, hipHostMallocCoherent));
    *bell = 0;
    *done = 0;
    state[0] = state[1] = 0;
    hipStream_t s, ws;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ws, hipStreamNonBlocking));
    uint32_t seq = 0;
    for (size_t n : {(size_t) 1, (size_t) 256, (size_t) 4096}) {
        // normal launch, kernel-stored completion word
        CK(hipMemset(a, 0, maxn * 4));
        CK(hipDeviceSynchronize());
        std::vector<double> tl;
        for (int i = 0; i < reps; ++i) {
            ++seq;
            auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_flag, dim3(1), dim3(256), 0, s, b, a, (unsigned long long) n, done, seq);
            while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                    fprintf(stderr, "launch phase: completion word never arrived\n");
                    CK(hipStreamSynchronize(s));
                    return 4;
                }
            }
            tl.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        CK(hipStreamSynchronize(s));
        fprintf(stderr, "count %zu: launch phase done\n", n);
        // resident worker
        CK(hipMemset(a, 0, maxn * 4));
        CK(hipDeviceSynchronize());
        __atomic_store_n(state, 0u, __ATOMIC_RELEASE);
        const uint32_t start = __atomic_load_n(bell, __ATOMIC_ACQUIRE);
        hipLaunchKernelGGL(k_worker, dim3(1), dim3(256), 0, ws, (volatile uint32_t *) bell,
                           (const Desc *) desc, done, state, start);
        CK(hipGetLastError());
        // wait until the worker runs (bounded)
        auto w0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(state, __ATOMIC_ACQUIRE) != 1u) {
            if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(5)) {
                fprintf(stderr, "worker did not start\n");
                return 2;
            }
        }
        fprintf(stderr, "count %zu: worker running\n", n);
        std::vector<double> tw;
        int timeouts = 0;
        for (int i = 0; i < reps; ++i) {
            ++seq;
            auto t0 = std::chrono::steady_clock::now();
            desc->in = b;
            desc->io = a;
            desc->n = n;
            __atomic_store_n(bell, seq, __ATOMIC_RELEASE);
            while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                    ++timeouts;
                    break;
                }
            }
            tw.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            if (timeouts)
                break;
        }
        fprintf(stderr, "count %zu: %zu calls, %d timeouts, worker polls %u; ringing exit\n", n,
                tw.size(), timeouts, __atomic_load_n(state + 1, __ATOMIC_ACQUIRE));
        __atomic_store_n(bell, kExit, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(ws));
        fprintf(stderr, "count %zu: worker exited (state %u)\n", n, __atomic_load_n(state, __ATOMIC_ACQUIRE));
        __atomic_store_n(bell, seq, __ATOMIC_RELEASE);
        CK(hipMemcpy(back.data(), a, n * 4, hipMemcpyDeviceToHost));
        long wrong = 0;
        for (size_t i = 0; i < n; ++i)
            wrong += back[i] != (float) reps;
        std::sort(tl.begin(), tl.end());
        std::sort(tw.begin(), tw.end());
        printf("count %5zu: launch+kernel-flag median %6.2f us (p90 %6.2f) | resident worker median %6.2f us (p10 %6.2f p90 %6.2f)%s%s\n",
               n, tl[tl.size() / 2], tl[tl.size() * 9 / 10], tw[tw.size() / 2], tw[tw.size() / 10],
               tw[tw.size() * 9 / 10], timeouts ? " TIMEOUT" : "", wrong ? " WRONG" : " ok");
        if (timeouts)
            return 3;
    }
    return 0;
}
