// tools/sync_latency.cpp -- per-call host time of the synchronous
// MPIX_Reduce_local (fp32 SUM, device-resident), median over repetitions, by
// count, under the completion mode MPIX_REDOP_SYNC selects (flag: the kernel
// stores the completion word when it runs as one workgroup; stream: the
// stream always writes it).  Each size is also checked: after r calls on
// zero-initialised inout with in = 1, inout must hold r everywhere.
// Build: g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude \
//        tools/sync_latency.cpp -Lmpich_amd -lmpix_redop -L/opt/rocm/lib -lamdhip64 \
//        -Wl,-rpath,$PWD/mpich_amd -Wl,-rpath,/opt/rocm/lib -o /tmp/sync_latency
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

#include "mpix_redop.h"

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 3000;
    const char *mode = getenv("MPIX_REDOP_SYNC") ? getenv("MPIX_REDOP_SYNC") : "flag";
    const long counts[] = {1, 16, 256, 1024, 4096, 4097, 8192, 65536, 1 << 20};
    float *a, *b;
    const size_t maxn = 1 << 20;
    if (hipMalloc(&a, maxn * 4) != hipSuccess || hipMalloc(&b, maxn * 4) != hipSuccess)
        return 1;
    std::vector<float> ones(maxn, 1.0f), back(maxn);
    hipMemcpy(b, ones.data(), maxn * 4, hipMemcpyHostToDevice);
    MPIX_Redop_init();
    int bad = 0;
    for (long n : counts) {
        hipMemset(a, 0, maxn * 4);
        hipDeviceSynchronize();
        std::vector<double> t;
        for (int i = 0; i < reps + 1; ++i) {
            auto t0 = std::chrono::steady_clock::now();
            int rc = MPIX_Reduce_local(b, a, n, MPIX_MPI_FLOAT, MPIX_SUM);
            auto t1 = std::chrono::steady_clock::now();
            if (rc)
                return 2;
            if (i)
                t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        // no device sync before the check: the call itself guarantees completion
        hipMemcpy(back.data(), a, n * 4, hipMemcpyDeviceToHost);
        long wrong = 0;
        for (long i = 0; i < n; ++i)
            wrong += back[i] != (float) (reps + 1);
        bad += wrong != 0;
        std::sort(t.begin(), t.end());
        printf("%-6s count %8ld: median %6.2f us  p10 %6.2f  p90 %6.2f  %s\n", mode, n,
               t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10], wrong ? "WRONG" : "ok");
    }
    return bad ? 3 : 0;
}
