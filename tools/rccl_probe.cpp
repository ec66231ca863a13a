// tools/rccl_probe.cpp -- can RCCL put two ranks on ONE GPU of this box?
// (decides whether the C collective schedules can be exercised with real
// RCCL transport on the 1-GPU test box).  One process, ncclCommInitAll over
// device list {0, 0}, one grouped send/recv exchange, result checked.
// Build: hipcc -O2 tools/rccl_probe.cpp -o /tmp/rccl_probe -lrccl
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <vector>

int main()
{
    const int P = 2;
    int devs[P] = {0, 0};
    ncclComm_t comms[P];
    ncclResult_t r = ncclCommInitAll(comms, P, devs);
    printf("ncclCommInitAll({0,0}) -> %d (%s)\n", (int) r, ncclGetErrorString(r));
    if (r != ncclSuccess)
        return 1;
    const size_t n = 1 << 20;
    float *buf[P], *rcv[P];
    hipStream_t st[P];
    for (int i = 0; i < P; ++i) {
        hipMalloc(&buf[i], n * 4);
        hipMalloc(&rcv[i], n * 4);
        hipStreamCreate(&st[i]);
        std::vector<float> h(n, (float) (i + 1));
        hipMemcpy(buf[i], h.data(), n * 4, hipMemcpyHostToDevice);
    }
    ncclGroupStart();
    for (int i = 0; i < P; ++i) {
        ncclSend(buf[i], n, ncclFloat, 1 - i, comms[i], st[i]);
        ncclRecv(rcv[i], n, ncclFloat, 1 - i, comms[i], st[i]);
    }
    r = ncclGroupEnd();
    printf("group send/recv -> %d (%s)\n", (int) r, ncclGetErrorString(r));
    for (int i = 0; i < P; ++i)
        hipStreamSynchronize(st[i]);
    int ok = 1;
    for (int i = 0; i < P; ++i) {
        std::vector<float> h(n);
        hipMemcpy(h.data(), rcv[i], n * 4, hipMemcpyDeviceToHost);
        for (size_t k = 0; k < n; ++k)
            if (h[k] != (float) (2 - i)) {
                ok = 0;
                break;
            }
    }
    printf("exchange %s\n", ok ? "OK" : "WRONG");
    for (int i = 0; i < P; ++i)
        ncclCommDestroy(comms[i]);
    return ok ? 0 : 1;
}
