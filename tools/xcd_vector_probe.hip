// xcd_vector_probe.hip -- the config-5 vector target (MPI_Type_vector(n, 1, 2,
// MPI_DOUBLE), inout[2j] += in[j], gaps never written) with the payload store
// flavour chosen per XCD group: the shipped k_vector_s2 stores write-through
// on every XCD (round 2: +5.8 %); here the two groups of the contiguous
// kernel's store policy (profiles/r03_wt_probe_xcd.json) get different
// flavours.  Bit-checked against the plain form, HIP events, one process.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xcd_vector_probe.hip -o tools/bin/xcd_vector_probe
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

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef double d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned xcc()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7;
}

// 0 nt, 1 plain, 2 write-through (sc0 sc1)
template <int M> __device__ __forceinline__ void st8(double *p, double v)
{
    unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    if constexpr (M == 0)
        __builtin_nontemporal_store(u, reinterpret_cast<unsigned long long *>(p));
    else if constexpr (M == 1)
        *reinterpret_cast<unsigned long long *>(p) = u;
    else
        *(volatile gu64 *) (gu64 *) reinterpret_cast<unsigned long long *>(p) = u;
}

template <int SA, int SB>
__global__ void __launch_bounds__(256) k_vs2(const double *__restrict__ in, double *__restrict__ io,
                                             uint64_t n, unsigned mask)
{
    const uint64_t j = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n)
        return;
    const bool a = (mask >> xcc()) & 1;
    double t;
    if (j + 1 < n)
        t = reinterpret_cast<const d2 *>(io)[j].x;      // the {payload, gap} pair in one load
    else
        t = io[2 * j];
    const double r = t + __builtin_nontemporal_load(in + j);
    if (a)
        st8<SA>(io + 2 * j, r);
    else
        st8<SB>(io + 2 * j, r);
}

struct Var {
    std::string name;
    void (*k)(const double *, double *, uint64_t, unsigned);
    unsigned mask;
    std::vector<float> ms;
};

template <int SA, int SB> void kl(const double *in, double *io, uint64_t n, unsigned mask)
{
    hipLaunchKernelGGL((k_vs2<SA, SB>), dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, 0, in,
                       io, n, mask);
}

int main()
{
    const uint64_t n = (uint64_t) 1 << 26;      // 512 MiB payload, 1 GiB span
    double *in, *io, *ref, *chk;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&io, n * 16));
    CK(hipMalloc(&ref, n * 16));
    CK(hipMalloc(&chk, n * 16));
    {
        std::vector<double> h(2 * n);
        uint64_t x = 0x5EED0005ull;
        for (auto &v : h) {
            x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
            v = (double) (x >> 11) / 9007199254740992.0 - 0.5;
        }
        CK(hipMemcpy(io, h.data(), n * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(in, h.data() + n / 2, n * 8, hipMemcpyHostToDevice));
    }
    std::vector<Var> V = {
        {"all_wt (shipped)", kl<2, 2>, 0x00, {}},
        {"all_nt", kl<0, 0>, 0x00, {}},
        {"all_plain", kl<1, 1>, 0x00, {}},
        {"wt, 0x88 nt", kl<0, 2>, 0x88, {}},
        {"wt, 0x88 plain", kl<1, 2>, 0x88, {}},
        {"nt, 0x88 wt", kl<2, 0>, 0x88, {}},
        {"plain, 0x88 wt", kl<2, 1>, 0x88, {}},
        {"wt, 0x08 nt", kl<0, 2>, 0x08, {}},
        {"wt, 0xcc nt", kl<0, 2>, 0xcc, {}},
    };
    CK(hipMemcpy(ref, io, n * 16, hipMemcpyDeviceToDevice));
    CK(hipDeviceSynchronize());
    kl<1, 1>(in, ref, n, 0);
    CK(hipDeviceSynchronize());
    bool ok = true;
    std::string bad;
    std::vector<char> a(64 << 20), b(64 << 20);
    for (auto &v : V) {
        CK(hipMemcpy(chk, io, n * 16, hipMemcpyDeviceToDevice));
        CK(hipDeviceSynchronize());
        v.k(in, chk, n, v.mask);
        CK(hipDeviceSynchronize());
        for (size_t off = 0; off < n * 16; off += (size_t) 256 << 20) {
            CK(hipMemcpy(a.data(), (char *) ref + off, a.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), (char *) chk + off, b.size(), hipMemcpyDeviceToHost));
            if (memcmp(a.data(), b.data(), a.size())) {
                ok = false;
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
            v.k(in, io, n, v.mask);
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < 10; ++r)
                v.k(in, io, n, v.mask);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / 10);
        }
    printf("{\"probe\": \"xcd_vector_probe\", \"payload_bytes\": %llu, \"parity\": %s, \"bad\": \"%s\", "
           "\"kernel_ms\": {", (unsigned long long) (n * 8), ok ? "true" : "false", bad.c_str());
    for (size_t k = 0; k < V.size(); ++k) {
        auto m = V[k].ms;
        std::sort(m.begin(), m.end());
        const double t = (m[1] + m[2]) / 2;
        printf("%s\"%s\": {\"ms\": %.4f, \"alg_GBs\": %.1f}", k ? ", " : "", V[k].name.c_str(), t,
               3.0 * n * 8 / (t * 1e-3) / 1e9);
    }
    printf("}}\n");
    return ok ? 0 : 5;
}
