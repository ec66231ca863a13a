// multi_fold_probe.hip -- the in-order multi-input fold (the pipelined
// pairwise reduce-scatter's combine, k_contig_multi) by load placement.
//
// k_contig_multi runs at 6.46-6.50 TB/s for k = 3..15
// inputs with 1.0000x traffic while the 8-slot tree fold (9 streams, as the
// 7-input fold) reaches 6.94.  The association is fixed (inout, then inputs 0,
// 1, ... in order), so only where the loads sit can change.  Forms, one
// process, interleaved, fp32 SUM, S bytes per operand, in place into slot 0,
// one-wave blocks, the store policy on (XCDs 3, 7 write through):
//   ship        k_contig_multi<C, 1>: input q + 1 loaded before input q is
//               combined, a runtime loop over k
//   one         one input packet live beyond the accumulator: load q, combine q
//   unrollN     the fold unrolled over N = 4 / 8 / 16 compile-time slots,
//               guarded loads as reached (pairs)
//   clampN      unrolled over N slots, every load unconditional (an index past
//               the last input re-reads the last one, never combined): no
//               guard between a load and the combines after it
//   tree8       k_contig_tree_rec<C, 8, 1> (reference: 9 streams at k = 8)
//   _w6 / _w4   the same with dynamic LDS per block capping the waves per
//               SIMD at 6 / 4 (k_contig_tree_rec<8> uses 106 SGPRs: 6 waves)
//   contig      the headline kernel (k = 1 in place), uncapped and capped
// Every multi form's result is checked bit-identical to ship's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//        -Impich_amd/csrc -Iinclude -o tools/bin/multi_fold_probe tools/multi_fold_probe.hip
// usage: tools/bin/multi_fold_probe [MiB per operand, default 256]   (one JSON line)
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
constexpr unsigned B = 64;

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

// one packet per lane, no prefetch
__global__ void __launch_bounds__(64) k_one(MultiIn<float> ins, int k, float *io, uint64_t npk,
                                            Params prm, uint32_t nblk)
{
    v4u *vio = reinterpret_cast<v4u *>(io);
    const bool wt = wt_block(prm);
    for (uint64_t i = (uint64_t) blockIdx.x * B + threadIdx.x; i < npk; i += (uint64_t) nblk * B) {
        v4u acc = ld16<true>(vio + i);
        for (int q = 0; q < k; ++q)
            acc = combine16<C>(acc, ld16<true>(reinterpret_cast<const v4u *>(ins.p[q]) + i), prm);
        st16_pol<true>(vio + i, acc, wt);
    }
}

// unrolled over N slots, guarded loads as reached, in pairs
template <int N>
__global__ void __launch_bounds__(64) k_unroll(MultiIn<float> ins, int k, float *io, uint64_t npk,
                                               Params prm, uint32_t nblk)
{
    v4u *vio = reinterpret_cast<v4u *>(io);
    const bool wt = wt_block(prm);
    for (uint64_t i = (uint64_t) blockIdx.x * B + threadIdx.x; i < npk; i += (uint64_t) nblk * B) {
        v4u acc = ld16<true>(vio + i);
#pragma unroll
        for (int q = 0; q < N; q += 2) {
            v4u b0, b1;
            if (q < k)
                b0 = ld16<true>(reinterpret_cast<const v4u *>(ins.p[q]) + i);
            if (q + 1 < k)
                b1 = ld16<true>(reinterpret_cast<const v4u *>(ins.p[q + 1]) + i);
            if (q < k)
                acc = combine16<C>(acc, b0, prm);
            if (q + 1 < k)
                acc = combine16<C>(acc, b1, prm);
        }
        st16_pol<true>(vio + i, acc, wt);
    }
}

// unrolled over N slots, unconditional loads (clamped index), guarded combines
template <int N>
__global__ void __launch_bounds__(64) k_clamp(MultiIn<float> ins, int k, float *io, uint64_t npk,
                                              Params prm, uint32_t nblk)
{
    v4u *vio = reinterpret_cast<v4u *>(io);
    const bool wt = wt_block(prm);
    const v4u *p[N];
#pragma unroll
    for (int q = 0; q < N; ++q)
        p[q] = reinterpret_cast<const v4u *>(ins.p[q < k ? q : k - 1]);
    for (uint64_t i = (uint64_t) blockIdx.x * B + threadIdx.x; i < npk; i += (uint64_t) nblk * B) {
        v4u acc = ld16<true>(vio + i);
        v4u b[N];
#pragma unroll
        for (int q = 0; q < N; ++q)
            b[q] = ld16<true>(p[q] + i);
#pragma unroll
        for (int q = 0; q < N; ++q)
            acc = q < k ? combine16<C>(acc, b[q], prm) : acc;
        st16_pol<true>(vio + i, acc, wt);
    }
}

typedef void (*Fn)(const MultiIn<float> &, int, float *, uint64_t, const Params &, hipStream_t);

// dynamic LDS per one-wave block: caps the waves per SIMD (160 KiB of LDS per
// CU: 6656 B -> 24 blocks = 6 waves per SIMD, 10240 B -> 16 = 4); 0 = none
static unsigned g_lds = 0;

void ship(const MultiIn<float> &mi, int k, float *o, uint64_t npk, const Params &p, hipStream_t s)
{
    const unsigned g = grid_for(B, npk, 0, B);
    hipLaunchKernelGGL((k_contig_multi<C, 1>), dim3(g), dim3(B), g_lds, s, mi, k, o, 0, npk, npk * 4,
                       0, p, g, B);
}
void one(const MultiIn<float> &mi, int k, float *o, uint64_t npk, const Params &p, hipStream_t s)
{
    const unsigned g = grid_for(B, npk, 0, B);
    hipLaunchKernelGGL(k_one, dim3(g), dim3(B), g_lds, s, mi, k, o, npk, p, g);
}
template <int N> void unroll(const MultiIn<float> &mi, int k, float *o, uint64_t npk, const Params &p,
                             hipStream_t s)
{
    const unsigned g = grid_for(B, npk, 0, B);
    hipLaunchKernelGGL((k_unroll<N>), dim3(g), dim3(B), 0, s, mi, k, o, npk, p, g);
}
template <int N> void clamp(const MultiIn<float> &mi, int k, float *o, uint64_t npk, const Params &p,
                            hipStream_t s)
{
    const unsigned g = grid_for(B, npk, 0, B);
    hipLaunchKernelGGL((k_clamp<N>), dim3(g), dim3(B), g_lds, s, mi, k, o, npk, p, g);
}
// the headline kernel (k_contig, in place: o OP= input 0)
void contig(const MultiIn<float> &mi, int, float *o, uint64_t npk, const Params &p, hipStream_t s)
{
    const unsigned g = grid_for(B, npk, 0, B);
    hipLaunchKernelGGL((k_contig<C, 1, true, true, true>), dim3(g), dim3(B), g_lds, s, mi.p[0], o, 0,
                       npk, npk * 4, 0, p, g, B);
}
// LDS-capped form of F
template <Fn F, unsigned L> void cap(const MultiIn<float> &mi, int k, float *o, uint64_t npk,
                                     const Params &p, hipStream_t s)
{
    g_lds = L;
    F(mi, k, o, npk, p, s);
    g_lds = 0;
}

// the 8-slot tree (k + 1 = 8 slots: slot 0 the accumulator's role) into o
void tree8(const MultiIn<float> &mi, int k, float *o, uint64_t npk, const Params &p, hipStream_t s)
{
    MultiIn<float> t{};
    t.p[0] = o;
    for (int q = 0; q < 7; ++q)
        t.p[q + 1] = mi.p[q];
    hipLaunchKernelGGL((k_contig_tree_rec<C, 8, 1>), dim3(grid_for(B, npk, 0, B)), dim3(B), g_lds, s, t,
                       k + 1, (1u << (k + 1)) - 1, o, 0, npk, npk * 4, 0, p);
}

int main(int argc, char **argv)
{
    const uint64_t S = (uint64_t) (argc > 1 ? atoi(argv[1]) : 256) << 20;
    const uint64_t n = S / 4, npk = n / 4;
    std::vector<float *> slot(16);
    for (int q = 0; q < 16; ++q) {
        CK(hipMalloc(&slot[q], S));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, slot[q], n, 0x9e37u * (q + 1));
    }
    float *out, *ref, *init;
    CK(hipMalloc(&out, S));
    CK(hipMalloc(&ref, S));
    CK(hipMalloc(&init, S));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, init, n, 0x1234u);
    MultiIn<float> mi{};
    for (int q = 0; q < 16; ++q)
        mi.p[q] = slot[q];
    Params prm{1, 0};
    prm.wt_xcd = 0x88;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct V {
        const char *name;
        int k;
        Fn fn;
    };
    std::vector<V> vs;
    // round 6, second pass: the LDS cap swept (blocks per CU 29 / 26 / 24 /
    // 22 / 20, i.e. about 7 / 6.5 / 6 / 5.5 / 5 waves per SIMD) over the
    // shipped loop, one packet live, and the clamped unrolled form; the
    // headline kernel's and the tree's rows kept as references
    vs.push_back({"contig", 1, contig});
    vs.push_back({"contig_l6656", 1, cap<contig, 6656>});
    vs.push_back({"tree8", 7, tree8});
    for (int k : {1, 3, 7, 15}) {
        vs.push_back({"ship", k, ship});
        vs.push_back({"one", k, one});
        vs.push_back({"ship_l5632", k, cap<ship, 5632>});
        vs.push_back({"one_l5632", k, cap<one, 5632>});
        vs.push_back({"ship_l6144", k, cap<ship, 6144>});
        vs.push_back({"one_l6144", k, cap<one, 6144>});
        vs.push_back({"ship_l6656", k, cap<ship, 6656>});
        vs.push_back({"one_l6656", k, cap<one, 6656>});
        vs.push_back({"ship_l7168", k, cap<ship, 7168>});
        vs.push_back({"one_l7168", k, cap<one, 7168>});
        vs.push_back({"one_l8192", k, cap<one, 8192>});
        if (k <= 4) {
            vs.push_back({"clamp4", k, clamp<4>});
            vs.push_back({"clamp4_l6656", k, cap<clamp<4>, 6656>});
            vs.push_back({"clamp4_l5632", k, cap<clamp<4>, 5632>});
        }
    }
    // bits: every form against ship at the same k, from the same initial inout
    std::vector<int> same(vs.size(), -1);
    std::vector<float> h_ref(n), h_got(n);
    for (size_t v = 0; v < vs.size(); ++v) {
        if (!strncmp(vs[v].name, "contig", 6) || !strncmp(vs[v].name, "tree", 4))
            continue;
        size_t r = 0;
        while (r < vs.size() && (strcmp(vs[r].name, "ship") || vs[r].k != vs[v].k))
            ++r;
        if (r == v || r == vs.size())
            continue;
        CK(hipMemcpy(ref, init, S, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(out, init, S, hipMemcpyDeviceToDevice));
        CK(hipDeviceSynchronize());
        vs[r].fn(mi, vs[r].k, ref, npk, prm, s);
        vs[v].fn(mi, vs[v].k, out, npk, prm, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h_ref.data(), ref, S, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h_got.data(), out, S, hipMemcpyDeviceToHost));
        same[v] = memcmp(h_ref.data(), h_got.data(), S) == 0;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> ms(vs.size());
    for (int round = 0; round < 5; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            vs[v].fn(mi, vs[v].k, out, npk, prm, s);      // warm
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 10; ++r)
                vs[v].fn(mi, vs[v].k, out, npk, prm, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / 10.0);
        }
    printf("{\"what\": \"in-order multi-input fold by load placement, fp32 SUM, %llu MiB per operand, "
           "one-wave blocks, store policy 0x88, HIP events, 5 interleaved rounds of 10; TB/s over "
           "(k + 2) x S (k inputs + inout read + inout written); same = bits equal ship's\", "
           "\"rows\": [", (unsigned long long) (S >> 20));
    for (size_t v = 0; v < vs.size(); ++v) {
        std::vector<double> m = ms[v];
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        printf("%s{\"form\": \"%s\", \"k\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"TBs\": %.3f, "
               "\"same\": %d}", v ? ", " : "", vs[v].name, vs[v].k, med, m[0],
               (double) (vs[v].k + 2) * S / (med * 1e-3) / 1e12, same[v]);
    }
    printf("]}\n");
    return 0;
}
