// kernarg_probe.hip -- host issue cost of a kernel launch vs the size of its
// argument block (empty kernels, back-to-back on one stream, 1 block of 64
// threads): does the contiguous kernel's ~100-byte argument block cost the
// ~1 us over an empty launch seen in profiles/r02_launch_floor.json?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/kernarg_probe tools/kernarg_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

template <int N> struct Blob {
    uint64_t w[N];
};

template <int N> __global__ void k_args(Blob<N> b, uint64_t *sink)
{
    if (threadIdx.x == 0 && b.w[0] == 0x123456789ull)
        *sink = b.w[N - 1];
}

__global__ void k_none() {}

template <class F> static double issue_us(F launch, hipStream_t s, int reps)
{
    std::vector<double> t;
    for (int r = 0; r < 7; ++r) {
        (void) hipStreamSynchronize(s);
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i)
            launch();
        auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count() / reps);
    }
    (void) hipStreamSynchronize(s);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

template <int N> static void row(hipStream_t s, uint64_t *sink, bool *first)
{
    Blob<N> b{};
    double us = issue_us([&] { hipLaunchKernelGGL(k_args<N>, dim3(1), dim3(64), 0, s, b, sink); },
                         s, 2000);
    printf("%s{\"arg_bytes\": %d, \"issue_us\": %.3f}", *first ? "" : ", ", (int) (8 * N + 8), us);
    *first = false;
}

int main()
{
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return 1;
    uint64_t *sink;
    if (hipMalloc(&sink, 8) != hipSuccess)
        return 1;
    double none = issue_us([&] { hipLaunchKernelGGL(k_none, dim3(1), dim3(64), 0, s); }, s, 2000);
    printf("{\"no_args_issue_us\": %.3f, \"rows\": [", none);
    bool first = true;
    row<1>(s, sink, &first);
    row<3>(s, sink, &first);
    row<5>(s, sink, &first);
    row<7>(s, sink, &first);
    row<8>(s, sink, &first);
    row<9>(s, sink, &first);
    row<11>(s, sink, &first);
    row<13>(s, sink, &first);
    row<15>(s, sink, &first);
    row<31>(s, sink, &first);
    printf("]}\n");
    return 0;
}
