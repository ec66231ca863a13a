// tools/lat_probe.cpp -- host-side cost of the pieces of a synchronous
// MPIX_Reduce_local call (median ns over many iterations).
// Build: g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude \
//        tools/lat_probe.cpp -Lmpich_amd -lmpix_redop -L/opt/rocm/lib -lamdhip64 \
//        -Wl,-rpath,$PWD/mpich_amd -Wl,-rpath,/opt/rocm/lib -o /tmp/lat_probe
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <functional>
#include <vector>

#include "mpix_redop.h"

static double med_ns(const std::function<void()> &f, int reps = 2000)
{
    std::vector<double> t;
    f();
    for (int i = 0; i < reps; ++i) {
        auto a = std::chrono::steady_clock::now();
        f();
        auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::nano>(b - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main()
{
    float *a, *b, *h;
    hipMalloc(&a, 1 << 20);
    hipMalloc(&b, 1 << 20);
    hipHostMalloc(&h, 1 << 20, 0);
    std::vector<float> pageable(1 << 18);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    MPIX_Redop_init();
    hipPointerAttribute_t at;
    printf("hipPointerGetAttributes(device)   %8.0f ns\n", med_ns([&] { hipPointerGetAttributes(&at, a); }));
    printf("hipPointerGetAttributes(pinned)   %8.0f ns\n", med_ns([&] { hipPointerGetAttributes(&at, h); }));
    printf("hipPointerGetAttributes(pageable) %8.0f ns\n", med_ns([&] { hipPointerGetAttributes(&at, pageable.data()); (void) hipGetLastError(); }));
    int d;
    printf("hipGetDevice                      %8.0f ns\n", med_ns([&] { hipGetDevice(&d); }));
    printf("async launch count=1 (no wait)    %8.0f ns\n", med_ns([&] { MPIX_Reduce_local_async(b, a, 1, MPIX_MPI_FLOAT, MPIX_SUM, s); }));
    hipStreamSynchronize(s);
    printf("launch + event spin               %8.0f ns\n", med_ns([&] {
        MPIX_Reduce_local_async(b, a, 1, MPIX_MPI_FLOAT, MPIX_SUM, s);
        hipEventRecord(ev, s);
        while (hipEventQuery(ev) == hipErrorNotReady) {}
    }));
    printf("launch + hipStreamSynchronize     %8.0f ns\n", med_ns([&] {
        MPIX_Reduce_local_async(b, a, 1, MPIX_MPI_FLOAT, MPIX_SUM, s);
        hipStreamSynchronize(s);
    }));
    printf("MPIX_Reduce_local count=1 (%s)   %8.0f ns\n", getenv("MPIX_REDOP_SYNC") ? getenv("MPIX_REDOP_SYNC") : "event", med_ns([&] { MPIX_Reduce_local(b, a, 1, MPIX_MPI_FLOAT, MPIX_SUM); }));
    printf("MPIX_Reduce_local count=1         %8.0f ns\n", med_ns([&] { MPIX_Reduce_local(b, a, 1, MPIX_MPI_FLOAT, MPIX_SUM); }));
    printf("MPIX_Reduce_local count=1M/4      %8.0f ns\n", med_ns([&] { MPIX_Reduce_local(b, a, 1 << 18, MPIX_MPI_FLOAT, MPIX_SUM); }, 500));
    printf("empty event record+spin           %8.0f ns\n", med_ns([&] {
        hipEventRecord(ev, s);
        while (hipEventQuery(ev) == hipErrorNotReady) {}
    }));
    // completion through a value written to pinned host memory by the stream
    volatile uint32_t *flag = nullptr;
    hipHostMalloc((void **) &flag, 64, hipHostMallocCoherent);
    *flag = 0;
    uint32_t seq = 0;
    printf("launch + hipStreamWriteValue32    %8.0f ns\n", med_ns([&] {
        ++seq;
        MPIX_Reduce_local_async(b, a, 1, MPIX_MPI_FLOAT, MPIX_SUM, s);
        hipStreamWriteValue32(s, (void *) flag, seq, 0);
        while (*flag != seq) {}
    }));
    printf("empty hipStreamWriteValue32+spin  %8.0f ns\n", med_ns([&] {
        ++seq;
        hipStreamWriteValue32(s, (void *) flag, seq, 0);
        while (*flag != seq) {}
    }));
    hipStreamSynchronize(s);
    return 0;
}
