// launch_probe.hip -- host cost per back-to-back async launch of a tiny
// combine kernel on one stream: hipLaunchKernelGGL (runtime resolves the
// host stub on every call) vs hipModuleLaunchKernel / hipExtLaunchKernel with
// a function handle resolved once by hipGetFuncBySymbol.  Measurement tool
// only; prints ns per launch for issue and issue+drain.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

__global__ void k_sum(const float *__restrict__ a, float *__restrict__ b, uint64_t n)
{
    uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        b[i] += a[i];
}

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                         \
        }                                                                     \
    } while (0)

int main()
{
    const uint64_t n = 1 << 14;     // 64 KiB of fp32 per call
    const int calls = 20000;
    float *a, *b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipFunction_t fn;
    CK(hipGetFuncBySymbol(&fn, (const void *) k_sum));
    const unsigned grid = (unsigned) ((n + 255) / 256);

    for (int mode = 0; mode < 3; ++mode) {
        for (int pass = 0; pass < 2; ++pass) {     // pass 0 warms up
            CK(hipStreamSynchronize(s));
            auto t0 = std::chrono::steady_clock::now();
            for (int c = 0; c < calls; ++c) {
                if (mode == 0) {
                    hipLaunchKernelGGL(k_sum, dim3(grid), dim3(256), 0, s, a, b, n);
                } else if (mode == 1) {
                    const float *pa = a;
                    float *pb = b;
                    uint64_t nn = n;
                    void *args[] = {&pa, &pb, &nn};
                    CK(hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, s, args, nullptr));
                } else {
                    struct {
                        const float *pa;
                        float *pb;
                        uint64_t nn;
                    } kargs = {a, b, n};
                    size_t sz = sizeof(kargs);
                    void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &kargs,
                                   HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
                    CK(hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, s, nullptr, cfg));
                }
            }
            auto t1 = std::chrono::steady_clock::now();
            CK(hipStreamSynchronize(s));
            auto t2 = std::chrono::steady_clock::now();
            CK(hipGetLastError());
            if (pass == 1) {
                double iss = std::chrono::duration<double, std::nano>(t1 - t0).count() / calls;
                double tot = std::chrono::duration<double, std::nano>(t2 - t0).count() / calls;
                static const char *names[] = {"hipLaunchKernelGGL", "hipModuleLaunchKernel(args)",
                                              "hipModuleLaunchKernel(extra)"};
                printf("%-30s issue %7.0f ns/launch  total %7.0f ns/launch\n", names[mode], iss,
                       tot);
            }
        }
    }
    float h = 0;
    CK(hipMemcpy(&h, b, 4, hipMemcpyDeviceToHost));
    printf("check b[0]=%g (expect 0)\n", h);
    return 0;
}
