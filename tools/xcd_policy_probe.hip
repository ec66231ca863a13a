// xcd_policy_probe.hip -- cache policies chosen per XCD for the 1 GiB fp32
// SUM stream (inout += in), beyond the shipped store policy (two of eight XCDs
// store write-through, profiles/r03_wt_probe_xcd.json): load flavours per XCD
// group, and the packets-per-lane unroll / block size under the store policy.
// Every variant is checked bit for bit against the plain kernel's result and
// timed with HIP events in one process, variants interleaved round by round.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xcd_policy_probe.hip -o tools/bin/xcd_policy_probe
// Run:   tools/bin/xcd_policy_probe   (one JSON object on stdout)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t _e = (x);                                                         \
        if (_e != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(_e)); \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;

__device__ __forceinline__ unsigned xcc()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7;
}

// load flavour: 0 nt, 1 plain, 2 sc0 sc1 (volatile global)
template <int M> __device__ __forceinline__ v4u ld(const v4u *p)
{
    if constexpr (M == 0)
        return __builtin_nontemporal_load(p);
    else if constexpr (M == 1)
        return *p;
    else
        return *(volatile const gv4u *) (const gv4u *) p;
}

// store flavour: 0 nt, 1 plain, 2 write-through (sc0 sc1)
template <int M> __device__ __forceinline__ void st(v4u *p, v4u v)
{
    if constexpr (M == 0)
        __builtin_nontemporal_store(v, p);
    else if constexpr (M == 1)
        *p = v;
    else
        *(volatile gv4u *) (gv4u *) p = v;
}

// ORD: 0 all inout loads then all in loads (shipped), 1 alternating, 2 in first
template <int U, int LA, int SA, int LB, int SB, int ORD = 0>
__device__ __forceinline__ void tile(const v4u *__restrict__ in, v4u *__restrict__ io, uint64_t npk,
                                     uint64_t i, uint64_t nt)
{
    if (i + (U - 1) * nt >= npk) {
        for (int u = 0; u < U; ++u) {
            uint64_t k = i + u * nt;
            if (k < npk) {
                float4 x = __builtin_bit_cast(float4, io[k]), y = __builtin_bit_cast(float4, in[k]);
                x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
                io[k] = __builtin_bit_cast(v4u, x);
            }
        }
        return;
    }
    v4u a[U], b[U];
    if constexpr (ORD == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = ld<LA>(io + i + u * nt);
#pragma unroll
        for (int u = 0; u < U; ++u)
            b[u] = ld<LA>(in + i + u * nt);
    } else if constexpr (ORD == 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = ld<LA>(io + i + u * nt);
            b[u] = ld<LA>(in + i + u * nt);
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
            b[u] = ld<LA>(in + i + u * nt);
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = ld<LA>(io + i + u * nt);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        float4 x = __builtin_bit_cast(float4, a[u]), y = __builtin_bit_cast(float4, b[u]);
        x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
        st<SA>(io + i + u * nt, __builtin_bit_cast(v4u, x));
    }
    (void) LB;
    (void) SB;
}

// group A = XCDs in `mask` (loads LA, stores SA), group B = the others (LB, SB)
template <int U, int LA, int SA, int LB, int SB, int ORD = 0>
__global__ void __launch_bounds__(1024) k_pol(const v4u *__restrict__ in, v4u *__restrict__ io,
                                              uint64_t npk, unsigned mask)
{
    const uint64_t nt = blockDim.x;
    const uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x;
    if (i >= npk)
        return;
    if ((mask >> xcc()) & 1)
        tile<U, LA, SA, LB, SB, ORD>(in, io, npk, i, nt);
    else
        tile<U, LB, SB, LA, SA, ORD>(in, io, npk, i, nt);
}

struct Var {
    std::string name;
    void (*launch)(const v4u *, v4u *, uint64_t, unsigned, int, hipStream_t);
    unsigned mask;
    int block;
    std::vector<float> ms;
};

template <int U, int LA, int SA, int LB, int SB, int ORD = 0>
void launch(const v4u *in, v4u *io, uint64_t npk, unsigned mask, int block, hipStream_t s)
{
    const uint64_t tile = (uint64_t) block * U;
    hipLaunchKernelGGL((k_pol<U, LA, SA, LB, SB, ORD>), dim3((unsigned) ((npk + tile - 1) / tile)),
                       dim3(block), 0, s, in, io, npk, mask);
}

int main()
{
    const size_t bytes = (size_t) 1 << 30;
    const uint64_t npk = bytes / 16;
    v4u *in, *io, *ref, *chk;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&io, bytes));
    CK(hipMalloc(&ref, bytes));
    CK(hipMalloc(&chk, bytes));
    {
        std::vector<float> h(bytes / 4);
        uint64_t x = 0x5EED0009ull;
        for (auto &v : h) {
            x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
            v = (float) ((x * 2685821657736338717ull) >> 40) / (1u << 24) - 0.5f;
        }
        CK(hipMemcpy(in, h.data(), bytes, hipMemcpyHostToDevice));
        for (auto &v : h)
            v = v * 0.25f + 1.0f;
        CK(hipMemcpy(io, h.data(), bytes, hipMemcpyHostToDevice));
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // L/S codes: 0 nt, 1 plain, 2 sc0 sc1.  Group A = XCDs 3 and 7 (0x88).
    std::vector<Var> V = {
        {"all_nt (session-1 kernel)", launch<4, 0, 0, 0, 0>, 0x00, 256, {}},
        {"store_wt_0x88 (shipped)", launch<4, 0, 2, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 + A loads plain", launch<4, 1, 2, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 + A loads sc", launch<4, 2, 2, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 + B loads plain", launch<4, 0, 2, 1, 0>, 0x88, 256, {}},
        {"store_plain_0x88", launch<4, 0, 1, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 + B stores plain", launch<4, 0, 2, 0, 1>, 0x88, 256, {}},
        {"store_wt_0x88 U=2", launch<2, 0, 2, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 U=8", launch<8, 0, 2, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 block 512", launch<4, 0, 2, 0, 0>, 0x88, 512, {}},
        {"store_wt_0x88 block 128", launch<4, 0, 2, 0, 0>, 0x88, 128, {}},
        {"store_wt_0x08 (one XCD)", launch<4, 0, 2, 0, 0>, 0x08, 256, {}},
        {"store_plain_0x08 (one XCD)", launch<4, 0, 1, 0, 0>, 0x08, 256, {}},
        {"store_plain_0x8c (three XCDs)", launch<4, 0, 1, 0, 0>, 0x8c, 256, {}},
        {"store_wt_0x88 U=4 block 192", launch<4, 0, 2, 0, 0>, 0x88, 192, {}},
        {"store_wt_0x88 loads alternating", launch<4, 0, 2, 0, 0, 1>, 0x88, 256, {}},
        {"store_wt_0x88 in loads first", launch<4, 0, 2, 0, 0, 2>, 0x88, 256, {}},
        {"all_nt loads alternating", launch<4, 0, 0, 0, 0, 1>, 0x00, 256, {}},
        {"store_wt_0x88 U=3", launch<3, 0, 2, 0, 0>, 0x88, 256, {}},
        {"store_wt_0x88 U=6", launch<6, 0, 2, 0, 0>, 0x88, 256, {}},
    };
    // parity: every variant from the same inout gives the plain kernel's bits
    // (device-to-device copies on the launch stream: a hipMemcpy D2D may
    // return before it completes, and `s` does not wait for the null stream)
    CK(hipMemcpyAsync(ref, io, bytes, hipMemcpyDeviceToDevice, s));
    launch<4, 1, 1, 1, 1>(in, ref, npk, 0, 256, s);
    CK(hipStreamSynchronize(s));
    bool all_ok = true;
    std::string bad;
    for (auto &v : V) {
        CK(hipMemcpyAsync(chk, io, bytes, hipMemcpyDeviceToDevice, s));
        v.launch(in, chk, npk, v.mask, v.block, s);
        CK(hipStreamSynchronize(s));
        std::vector<uint32_t> a(1 << 20), b(1 << 20);
        for (size_t off = 0; off < bytes; off += (size_t) 64 << 20) {   // 16 samples of 4 MiB
            CK(hipMemcpy(a.data(), (char *) ref + off, 4 << 20, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), (char *) chk + off, 4 << 20, hipMemcpyDeviceToHost));
            if (memcmp(a.data(), b.data(), 4 << 20)) {
                all_ok = false;
                bad += v.name + ";";
                break;
            }
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 4; ++round)
        for (auto &v : V) {
            v.launch(in, io, npk, v.mask, v.block, s);
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 10; ++r)
                v.launch(in, io, npk, v.mask, v.block, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / 10);
        }
    printf("{\"probe\": \"xcd_policy_probe\", \"bytes\": %zu, \"parity\": %s, \"bad\": \"%s\", \"kernel_ms\": {",
           bytes, all_ok ? "true" : "false", bad.c_str());
    for (size_t k = 0; k < V.size(); ++k) {
        auto m = V[k].ms;
        std::sort(m.begin(), m.end());
        printf("%s\"%s\": %.4f", k ? ", " : "", V[k].name.c_str(), (m[1] + m[2]) / 2);
    }
    printf("}}\n");
    return all_ok ? 0 : 5;
}
