// tree8_probe.hip -- the 8-slot tree fold (the P = 8 pull's combine) by form.
//
// k_contig_tree at k = 8 ran at 5.63 TB/s in its 16-slot,
// one-packet form.  This probe times, in one process and interleaved, fp32 SUM
// over 8 slots of S bytes into a separate output ((8 + 1) x S algorithmic):
//   slots16x1   k_contig_tree<C, 16, 1>   (round 4's form for k = 8)
//   slots8x2    k_contig_tree<C, 8, 2>    (all 16 loads per lane issued up front)
//   rec8xU      k_contig_tree_rec<C, 8, U> for U = 1, 2, 4 (the fold's pair order,
//               slots loaded as the recursion reaches them)
// plus the multi-input folds of 7 and 15 inputs (U = 2 shipped in round 4, and
// U = 1), the 2- and 4-slot forms, and each with the store policy (_wt).
// (Round 5 also timed the in-order multi-input fold unrolled over 8 / 16 slots,
// k_contig_multi_k, since removed: profiles/r05_multi_unrolled.json, source in
// git history.)
// Every tree form's output is checked bit-identical to the shipped form's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//        -Impich_amd/csrc -Iinclude -o tools/bin/tree8_probe tools/tree8_probe.hip
// usage: tools/bin/tree8_probe [MiB per operand, default 256]   (one JSON line)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
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

template <int KMAX, int U, unsigned B = 256> void tree(const MultiIn<float> &mi, int k, float *o,
                                                        uint64_t npk, const Params &p, hipStream_t s)
{
    hipLaunchKernelGGL((k_contig_tree<C, KMAX, U>), dim3(grid_for(B * U, npk, 0, B)), dim3(B), 0, s,
                       mi, k, (1u << k) - 1, o, 0, npk, npk * 4, 0, p);
}
template <int KMAX, int U, unsigned B = 256> void rec(const MultiIn<float> &mi, int k, float *o,
                                                       uint64_t npk, const Params &p, hipStream_t s)
{
    hipLaunchKernelGGL((k_contig_tree_rec<C, KMAX, U>), dim3(grid_for(B * U, npk, 0, B)), dim3(B), 0,
                       s, mi, k, (1u << k) - 1, o, 0, npk, npk * 4, 0, p);
}
template <int U, unsigned B = 256> void multi(const MultiIn<float> &mi, int k, float *o, uint64_t npk,
                                              const Params &p, hipStream_t s)
{
    // k - 1 inputs folded into o (which then holds garbage; timing only)
    MultiIn<float> m{};
    for (int q = 1; q < k; ++q)
        m.p[q - 1] = mi.p[q];
    const unsigned g = grid_for(B * U, npk, 0, B);
    hipLaunchKernelGGL((k_contig_multi<C, U>), dim3(g), dim3(B), 0, s, m, k - 1, o, 0, npk, npk * 4,
                       0, p, g, B);
}

// the headline kernel's form for comparison: o OP= slot 0 in place (k_contig, U packets per lane)
template <int U, unsigned B = 256> void contig(const MultiIn<float> &mi, int, float *o, uint64_t npk,
                                               const Params &p, hipStream_t s)
{
    const unsigned g = grid_for(B * U, npk, 0, B);
    hipLaunchKernelGGL((k_contig<C, U, true, true, true>), dim3(g), dim3(B), 0, s, mi.p[0], o, 0, npk,
                       npk * 4, 0, p, g, B);
}

typedef void (*LaunchFn)(const MultiIn<float> &, int, float *, uint64_t, const Params &, hipStream_t);

// the same launch with the library's default store policy (blocks on XCDs 3
// and 7 store write-through, Params::wt_xcd = 0x88)
template <LaunchFn F> void wt(const MultiIn<float> &mi, int k, float *o, uint64_t npk, const Params &p,
                              hipStream_t s)
{
    Params q = p;
    q.wt_xcd = 0x88;
    F(mi, k, o, npk, q, s);
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
    float *out, *ref;
    CK(hipMalloc(&out, S));
    CK(hipMalloc(&ref, S));
    MultiIn<float> mi{};
    for (int q = 0; q < 16; ++q)
        mi.p[q] = slot[q];
    Params prm{1, 0};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct V {
        const char *name;
        int k;
        LaunchFn fn;
        const char *ref;    // form whose bits it must equal (nullptr: not checked)
    };
    std::vector<V> vs = {
        {"k4_slots4x2", 4, tree<4, 2>, nullptr}, {"k4_rec4x1", 4, rec<4, 1>, "k4_slots4x2"},
        {"k4_rec4x2", 4, rec<4, 2>, "k4_slots4x2"},
        {"k8_slots8x2", 8, tree<8, 2>, nullptr}, {"k8_slots16x1", 8, tree<16, 1>, "k8_slots8x2"},
        {"k8_rec8x1", 8, rec<8, 1>, "k8_slots8x2"}, {"k8_rec8x2", 8, rec<8, 2>, "k8_slots8x2"},
        {"k16_slots16x1", 16, tree<16, 1>, nullptr}, {"k16_rec16x1", 16, rec<16, 1>, "k16_slots16x1"},
        {"k8_multi7_u2", 8, multi<2>, nullptr}, {"k8_multi7_u1", 8, multi<1>, nullptr},
        {"k16_multi15_u2", 16, multi<2>, nullptr}, {"k16_multi15_u1", 16, multi<1>, nullptr},
        {"k2_slots2x4_wt", 2, wt<tree<2, 4>>, nullptr}, {"k2_rec2x1_wt", 2, wt<rec<2, 1>>, "k2_slots2x4_wt"},
        {"k2_rec2x2_wt", 2, wt<rec<2, 2>>, "k2_slots2x4_wt"},
        {"k4_slots4x2_wt", 4, wt<tree<4, 2>>, "k4_slots4x2"}, {"k4_rec4x1_wt", 4, wt<rec<4, 1>>, "k4_slots4x2"},
        {"k8_rec8x1_wt", 8, wt<rec<8, 1>>, "k8_slots8x2"}, {"k16_rec16x1_wt", 16, wt<rec<16, 1>>, "k16_slots16x1"},
        {"k8_multi7_u2_wt", 8, wt<multi<2>>, nullptr}, {"k8_multi7_u1_wt", 8, wt<multi<1>>, nullptr},
        {"k16_multi15_u1_wt", 16, wt<multi<1>>, nullptr},
        {"k2_contig_u4_wt", 2, wt<contig<4>>, nullptr}, {"k2_contig_u2_wt", 2, wt<contig<2>>, nullptr},
        {"k2_contig_u1_wt", 2, wt<contig<1>>, nullptr},
        // 64-thread (one-wave) blocks
        {"k2_contig_u1_b64_wt", 2, wt<contig<1, 64>>, nullptr},
        {"k2_rec2x2_b64_wt", 2, wt<rec<2, 2, 64>>, "k2_slots2x4_wt"}, {"k2_rec2x1_b64_wt", 2, wt<rec<2, 1, 64>>, "k2_slots2x4_wt"},
        {"k4_slots4x2_b64_wt", 4, wt<tree<4, 2, 64>>, "k4_slots4x2"}, {"k4_rec4x1_b64_wt", 4, wt<rec<4, 1, 64>>, "k4_slots4x2"},
        {"k8_rec8x1_b64_wt", 8, wt<rec<8, 1, 64>>, "k8_slots8x2"}, {"k16_rec16x1_b64_wt", 16, wt<rec<16, 1, 64>>, "k16_slots16x1"},
        {"k8_multi7_u1_b64_wt", 8, wt<multi<1, 64>>, nullptr}, {"k16_multi15_u1_b64_wt", 16, wt<multi<1, 64>>, nullptr},
        // one-wave blocks at two packets per lane (2 KiB per stream per wave)
        {"k8_multi7_u2_b64_wt", 8, wt<multi<2, 64>>, nullptr}, {"k8_rec8x2_b64_wt", 8, wt<rec<8, 2, 64>>, "k8_slots8x2"},
        {"k4_multi3_u2_b64_wt", 4, wt<multi<2, 64>>, nullptr}, {"k4_multi3_u1_b64_wt", 4, wt<multi<1, 64>>, nullptr},
    };
    std::vector<int> same(vs.size(), -1);
    std::vector<float> h_ref(n), h_got(n);
    for (size_t v = 0; v < vs.size(); ++v) {
        if (!vs[v].ref)
            continue;
        size_t r = 0;
        while (strcmp(vs[r].name, vs[v].ref))
            ++r;
        // both start from slot 0 (the in-place multi forms fold into it; the
        // tree forms overwrite every element)
        CK(hipMemcpy(ref, slot[0], S, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(out, slot[0], S, hipMemcpyDeviceToDevice));
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
    printf("{\"what\": \"tree-fold and multi-input forms, fp32 SUM, %llu MiB per operand, HIP events, "
           "5 interleaved rounds of 10; TB/s over (k + 1) x S (tree, separate output; multi: k - 1 "
           "inputs + inout read + inout written)\", \"rows\": [", (unsigned long long) (S >> 20));
    for (size_t v = 0; v < vs.size(); ++v) {
        std::vector<double> m = ms[v];
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        printf("%s{\"form\": \"%s\", \"k\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"TBs\": %.3f, "
               "\"bit_identical_to\": %s%s%s, \"same\": %d}",
               v ? ", " : "", vs[v].name, vs[v].k, med, m[0],
               (double) (vs[v].k + 1) * S / (med * 1e-3) / 1e12, vs[v].ref ? "\"" : "",
               vs[v].ref ? vs[v].ref : "null", vs[v].ref ? "\"" : "", same[v]);
    }
    printf("]}\n");
    return 0;
}
