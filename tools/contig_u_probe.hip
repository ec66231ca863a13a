// contig_u_probe.hip -- packets per lane (U) and block size of the headline
// kernel, k_contig<FSum<float>> in place, with the library's default store
// policy (blocks on XCDs 3 and 7 write through).
//
// tools/tree8_probe.hip found the fold-order tree at one or two packets per
// lane faster than the up-front forms, and k_contig itself at U = 1 ahead of
// the shipped U = 4 in the same process (6.93 vs 6.79 TB/s at 256 MiB, 6.84
// vs 6.64 at 1 GiB).  This probe times the headline shape only: 1 GiB fp32
// SUM per operand, U in {1, 2, 4} x block in {256, 512, 1024}, and at U = 1 the
// store-policy XCD masks and plain (not non-temporal) loads / stores, interleaved,
// 7 rounds of 10 launches, median; every form's result bit-identical to
// U = 4 / 256 (same combine per element, so it must be).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//        -Impich_amd/csrc -Iinclude -o tools/bin/contig_u_probe tools/contig_u_probe.hip
// usage: tools/bin/contig_u_probe [MiB per operand, default 1024]   (one JSON line)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "redop_kernels.h"

using namespace mpix;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef FSum<float> C;

__global__ void fill(float *p, uint64_t n, uint32_t seed)
{
    for (uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) (i * 2654435761u) ^ seed;
        h ^= h >> 13;
        h *= 0x5bd1e995u;
        h ^= h >> 15;
        p[i] = (float) (h & 0xffffff) / 16777216.0f - 0.5f;
    }
}

template <int U, unsigned MASK = 0x88, bool NTL = true, bool NTS = true, bool GRP = true>
void contig(const float *in, float *io, uint64_t npk, unsigned block, const Params &p, hipStream_t s)
{
    const unsigned g = grid_for((uint64_t) block * U, npk, 0);
    Params q = p;
    q.wt_xcd = MASK;
    hipLaunchKernelGGL((k_contig<C, U, NTL, NTS, true, GRP>), dim3(g), dim3(block), 0, s, in, io, 0, npk,
                       npk * 4, 0, q, g, block);
}

typedef void (*Fn)(const float *, float *, uint64_t, unsigned, const Params &, hipStream_t);

int main(int argc, char **argv)
{
    const uint64_t S = (uint64_t) (argc > 1 ? atoi(argv[1]) : 1024) << 20;
    const uint64_t n = S / 4, npk = n / 4;
    float *in, *io, *io0;
    CK(hipMalloc(&in, S));
    CK(hipMalloc(&io, S));
    CK(hipMalloc(&io0, S));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in, n, 0x1234u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, io0, n, 0x5678u);
    CK(hipDeviceSynchronize());
    Params prm{1, 0};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct V {
        const char *name;
        Fn fn;
        unsigned block;
    };
    std::vector<V> vs = {{"u4_b256", contig<4>, 256},  {"u2_b256", contig<2>, 256},
                         {"u1_b256", contig<1>, 256},  {"u4_b512", contig<4>, 512},
                         {"u2_b512", contig<2>, 512},  {"u1_b512", contig<1>, 512},
                         {"u1_b1024", contig<1>, 1024}, {"u2_b1024", contig<2>, 1024},
                         // one packet per lane: store policy masks and cache flavours
                         {"u1_b256_wt00", contig<1, 0x00>, 256}, {"u1_b256_wt08", contig<1, 0x08>, 256},
                         {"u1_b256_wt80", contig<1, 0x80>, 256}, {"u1_b256_wtAA", contig<1, 0xAA>, 256},
                         {"u1_b256_wtCC", contig<1, 0xCC>, 256}, {"u1_b256_wtFF", contig<1, 0xFF>, 256},
                         {"u1_b256_plainload", contig<1, 0x88, false, true>, 256},
                         {"u1_b256_plainstore", contig<1, 0x88, true, false>, 256},
                         {"u1_b128", contig<1>, 128}, {"u1_b64", contig<1>, 64},
                         {"u2_b128", contig<2>, 128},
                         // one-wave blocks (the round-5 default): policy masks, 2 packets
                         {"u1_b64_wt00", contig<1, 0x00>, 64}, {"u1_b64_wt08", contig<1, 0x08>, 64},
                         {"u1_b64_wt80", contig<1, 0x80>, 64}, {"u1_b64_wtCC", contig<1, 0xCC>, 64},
                         {"u1_b64_wt44", contig<1, 0x44>, 64}, {"u1_b64_wt11", contig<1, 0x11>, 64},
                         {"u2_b64", contig<2>, 64}, {"u2_b64_alt", contig<2, 0x88, true, true, false>, 64}};
    // bits: one launch of each on a fresh copy of io0, against u4_b256's
    std::vector<float> h_ref(n), h_got(n);
    std::vector<int> same(vs.size(), 1);
    for (size_t v = 0; v < vs.size(); ++v) {
        CK(hipMemcpy(io, io0, S, hipMemcpyDeviceToDevice));
        CK(hipDeviceSynchronize());     // the copy ran on the null stream, s does not wait for it
        vs[v].fn(in, io, npk, vs[v].block, prm, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(v ? h_got.data() : h_ref.data(), io, S, hipMemcpyDeviceToHost));
        if (v)
            same[v] = memcmp(h_ref.data(), h_got.data(), S) == 0;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> ms(vs.size());
    for (int round = 0; round < 7; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            vs[v].fn(in, io, npk, vs[v].block, prm, s);
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 10; ++r)
                vs[v].fn(in, io, npk, vs[v].block, prm, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / 10.0);
        }
    printf("{\"what\": \"k_contig fp32 SUM in place, %llu MiB per operand, store policy 0x88, HIP "
           "events, 7 interleaved rounds of 10; TB/s over 3 x S\", \"rows\": [",
           (unsigned long long) (S >> 20));
    for (size_t v = 0; v < vs.size(); ++v) {
        std::vector<double> m = ms[v];
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        printf("%s{\"form\": \"%s\", \"ms_median\": %.4f, \"ms_min\": %.4f, \"TBs\": %.3f, "
               "\"bit_identical\": %d}",
               v ? ", " : "", vs[v].name, med, m[0], 3.0 * S / (med * 1e-3) / 1e12, same[v]);
    }
    printf("]}\n");
    return 0;
}
