// valu_rate_probe.hip -- issue cost of the integer VALU instructions the
// soft-float fast paths are made of, relative to v_add_u32 (VERDICT r05
// item 5: the binary128 complex product is VALU-bound; which instructions
// its count should be cut in).  The VOP3 form of v_add_u32 and a VOP2 op with
// a 32-bit literal tell an encoding-size cost from a per-operation one.  Each kernel runs 8 waves per SIMD on every
// CU, each lane 8 independent chains of one instruction (inline asm, so the
// instruction is exactly the one named), 512 iterations; HIP events; the
// figure is kernel time / the v_add_u32 kernel's time.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_rate_probe tools/valu_rate_probe.hip
// usage: tools/bin/valu_rate_probe   (one JSON line)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 512;

#define KERNEL32(name, asmop)                                                                    \
    __global__ void __launch_bounds__(256) name(uint32_t *out, uint32_t seed)                    \
    {                                                                                            \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
        const uint32_t b = seed | 1, c = seed >> 3;                                              \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            asm volatile(asmop : "+v"(a0) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a1) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a2) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a3) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a4) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a5) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a6) : "v"(b), "v"(c) : "vcc");                                     \
            asm volatile(asmop : "+v"(a7) : "v"(b), "v"(c) : "vcc");                                     \
        }                                                                                        \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
    }

#define KERNEL64(name, asmop)                                                                    \
    __global__ void __launch_bounds__(256) name(uint32_t *out, uint32_t seed)                    \
    {                                                                                            \
        uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
        const uint32_t b = seed | 1, c = seed >> 3;                                              \
        const uint64_t d = ((uint64_t) seed << 32) | c;                                          \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            asm volatile(asmop : "+v"(a0) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a1) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a2) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a3) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a4) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a5) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a6) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
            asm volatile(asmop : "+v"(a7) : "v"(b), "v"(c), "v"(d) : "vcc");                             \
        }                                                                                        \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t) (a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    }

// the select and the rest without a vcc clobber: a clobber makes the compiler
// pad each following read of vcc with wait states (the first version's
// v_cndmask_b32 row, 8.7x, was that padding); the mask in an SGPR pair as
// compiled code has it after a v_cmp
#define KERNEL32S(name, asmop)                                                                   \
    __global__ void __launch_bounds__(256) name(uint32_t *out, uint32_t seed, uint64_t m)        \
    {                                                                                            \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
        const uint32_t b = seed | 1, c = seed >> 3;                                              \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            asm volatile(asmop : "+v"(a0) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a1) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a2) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a3) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a4) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a5) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a6) : "v"(b), "v"(c), "s"(m));                             \
            asm volatile(asmop : "+v"(a7) : "v"(b), "v"(c), "s"(m));                             \
        }                                                                                        \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
    }

#define KERNELF64(name, asmop)                                                                   \
    __global__ void __launch_bounds__(256) name(uint32_t *out, uint32_t seed, uint64_t m)        \
    {                                                                                            \
        double a0 = threadIdx.x + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,      \
               a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                            \
        const double b = 1.0 + seed * 1e-9, c = 1e-3;                                            \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            asm volatile(asmop : "+v"(a0) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a1) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a2) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a3) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a4) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a5) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a6) : "v"(b), "v"(c));                                     \
            asm volatile(asmop : "+v"(a7) : "v"(b), "v"(c));                                     \
        }                                                                                        \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t) (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7); \
    }

// a compare into an SGPR pair (%3, scratch) and a select reading it
#define KERNEL32T(name, asmop)                                                                   \
    __global__ void __launch_bounds__(256) name(uint32_t *out, uint32_t seed, uint64_t m)        \
    {                                                                                            \
        uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
        const uint32_t b = seed | 1, c = seed >> 3;                                              \
        uint64_t t;                                                                              \
        for (int i = 0; i < ITERS; ++i) {                                                        \
            asm volatile(asmop : "+v"(a0), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a1), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a2), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a3), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a4), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a5), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a6), "=&s"(t) : "v"(b), "v"(c));                           \
            asm volatile(asmop : "+v"(a7), "=&s"(t) : "v"(b), "v"(c));                           \
        }                                                                                        \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;             \
    }

KERNEL32(k_add_u32, "v_add_u32 %0, %0, %1")
KERNEL32(k_add_u32_e64, "v_add_u32_e64 %0, %0, %1")
KERNEL32(k_and_lit, "v_and_b32 %0, 0x7fffffff, %0")
KERNEL32(k_xor_e32, "v_xor_b32 %0, %0, %1")
KERNEL32(k_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
KERNEL32(k_lshl_or, "v_lshl_or_b32 %0, %0, 3, %1")
KERNEL32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
KERNEL32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
KERNEL32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL64(k_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %2, %0")
KERNEL64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %3")
KERNEL64(k_lshr_b64, "v_lshrrev_b64 %0, 3, %0")
KERNEL32(k_add_co_pair, "v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %2, vcc")
KERNEL32S(k_add_u32_s, "v_add_u32 %0, %0, %1")
KERNEL32S(k_cndmask_s, "v_cndmask_b32_e64 %0, %0, %1, %3")
KERNEL32S(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
KERNEL32S(k_mul_hi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
KERNEL32S(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL32S(k_bfe, "v_bfe_u32 %0, %0, %1, 7")
KERNEL32S(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL32S(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL32S(k_lshrrev_b32, "v_lshrrev_b32 %0, %1, %0")
KERNEL32S(k_mul_lo_u16, "v_mul_lo_u16 %0, %0, %1")
KERNEL32S(k_add_nop, "v_add_u32 %0, %0, %1\n\ts_nop 0")
KERNEL32S(k_cndmask_vcc, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL32S(k_addc_chain, "v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %2, vcc")
KERNEL32S(k_addc_chain_nop, "v_add_co_u32 %0, vcc, %0, %1\n\ts_nop 1\n\tv_addc_co_u32 %0, vcc, %0, %2, vcc")
KERNEL32(k_cmp_cndmask_vop2, "v_cmp_gt_u32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %1, vcc")
KERNEL32T(k_cmp_cndmask_e64, "v_cmp_gt_u32_e64 %1, %0, %2\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %0, %2, %1")
KERNEL32(k_cmp_vop2, "v_cmp_gt_u32 vcc, %0, %1\n\tv_add_u32 %0, %0, %1")
KERNELF64(k_fma_f64, "v_fma_f64 %0, %0, %1, %2")
KERNELF64(k_mul_f64, "v_mul_f64 %0, %0, %1")
KERNELF64(k_add_f64, "v_add_f64 %0, %0, %1")

typedef void (*K)(uint32_t *, uint32_t);
typedef void (*KS)(uint32_t *, uint32_t, uint64_t);

int main()
{
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 8;    // 256-thread blocks: 8 waves per SIMD
    uint32_t *out;
    CK(hipMalloc(&out, (size_t) blocks * 256 * 4));
    struct R {
        const char *name;
        K k;
        int per;    // instructions per asm statement
        KS ks = nullptr;
    } rs[] = {{"v_add_u32", k_add_u32, 1},           {"v_add_u32_e64 (VOP3 form)", k_add_u32_e64, 1},
              {"v_and_b32 + literal", k_and_lit, 1}, {"v_xor_b32", k_xor_e32, 1},
              {"v_alignbit_b32", k_alignbit, 1},
              {"v_lshl_or_b32", k_lshl_or, 1},       {"v_mul_lo_u32", k_mul_lo_u32, 1},
              {"v_mul_hi_u32", k_mul_hi_u32, 1},     {"v_cndmask_b32", k_cndmask, 1},
              {"v_mad_u64_u32", k_mad_u64_u32, 1},   {"v_lshl_add_u64", k_lshl_add_u64, 1},
              {"v_lshrrev_b64", k_lshr_b64, 1},      {"v_add_co_u32+v_addc_co_u32", k_add_co_pair, 2},
              {"v_add_u32 (no vcc clobber)", nullptr, 1, k_add_u32_s},
              {"v_cndmask_b32_e64 (SGPR mask)", nullptr, 1, k_cndmask_s},
              {"v_mul_u32_u24", nullptr, 1, k_mul_u24}, {"v_mul_hi_u32_u24", nullptr, 1, k_mul_hi_u24},
              {"v_mad_u32_u24", nullptr, 1, k_mad_u24}, {"v_bfe_u32", nullptr, 1, k_bfe},
              {"v_add3_u32", nullptr, 1, k_add3}, {"v_perm_b32", nullptr, 1, k_perm},
              {"v_lshrrev_b32", nullptr, 1, k_lshrrev_b32}, {"v_mul_lo_u16", nullptr, 1, k_mul_lo_u16},
              {"v_fma_f64", nullptr, 1, k_fma_f64}, {"v_mul_f64", nullptr, 1, k_mul_f64},
              {"v_add_f64", nullptr, 1, k_add_f64},
              {"v_add_u32 + s_nop 0 (per pair)", nullptr, 1, k_add_nop},
              {"v_cndmask_b32 vcc (no clobber)", nullptr, 1, k_cndmask_vcc},
              {"v_add_co_u32+v_addc_co_u32 (no clobber)", nullptr, 2, k_addc_chain},
              {"v_add_co_u32+s_nop 1+v_addc_co_u32 (per inst)", nullptr, 2, k_addc_chain_nop},
              {"v_cmp_gt_u32 vcc + v_cndmask_b32 vcc (per inst)", k_cmp_cndmask_vop2, 2},
              {"v_cmp_gt_u32_e64 s + v_cndmask_b32_e64 s (per inst)", nullptr, 2, k_cmp_cndmask_e64},
              {"v_cmp_gt_u32 vcc + v_add_u32 (per inst)", k_cmp_vop2, 2}};
    const int n = sizeof rs / sizeof rs[0];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best[64];
    for (int i = 0; i < n; ++i)
        best[i] = 1e30f;
    for (int round = 0; round < 5; ++round)
        for (int i = 0; i < n; ++i) {
            const uint64_t m = 0x5555aaaa3333ccccull;
            if (rs[i].ks)
                hipLaunchKernelGGL(rs[i].ks, dim3(blocks), dim3(256), 0, 0, out, 12345u + round, m);
            else
                hipLaunchKernelGGL(rs[i].k, dim3(blocks), dim3(256), 0, 0, out, 12345u + round);
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < 5; ++r)
                if (rs[i].ks)
                    hipLaunchKernelGGL(rs[i].ks, dim3(blocks), dim3(256), 0, 0, out, 777u + r, m);
                else
                    hipLaunchKernelGGL(rs[i].k, dim3(blocks), dim3(256), 0, 0, out, 777u + r);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            t /= 5;
            if (t < best[i])
                best[i] = t;
        }
    // wave-instructions per SIMD per launch: blocks * 4 waves * 8 chains * ITERS * per / SIMDs
    const double simds = prop.multiProcessorCount * 4.0;
    printf("{\"what\": \"integer VALU issue cost, 8 waves per SIMD, 8 independent chains per lane, "
           "best of 5 rounds of 5 launches; ns per wave-instruction per SIMD and the ratio to "
           "v_add_u32\", \"cus\": %d, \"rows\": [", prop.multiProcessorCount);
    for (int i = 0; i < n; ++i) {
        const double insts = blocks * 4.0 * 8 * ITERS * rs[i].per / simds;
        printf("%s{\"inst\": \"%s\", \"ms\": %.4f, \"ns_per_wave_inst\": %.4f, \"vs_v_add_u32\": %.3f}",
               i ? ", " : "", rs[i].name, best[i], best[i] * 1e6 / insts,
               (best[i] / rs[i].per) / best[0]);
    }
    printf("]}\n");
    return 0;
}
