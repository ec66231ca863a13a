// redop_kernels.h -- streaming kernels for the local reduction (gfx950).
//
// The combine is a pure HBM stream: per element 2 loads + 1 store and O(1)
// integer/fp work, so the kernels are built around the memory system, not
// the ALUs (no MFMA, no LDS on the contiguous path):
//   * both operands are read as 16-byte packets (global_load_dwordx4), each
//     lane keeping MPIX_REDOP_UNROLL packets per operand in flight before the
//     first combine, so a 256-thread block has 256*U*32 B outstanding (U = 1
//     since round 5: the latency is covered by waves, not by each wave's
//     loads -- 8 waves per SIMD at 1 GiB fp32 SUM ran 4.0 % faster than U = 4,
//     every config-3 row 2.8-8.2 % faster; tools/contig_u_probe.hip,
//     tools/gpu_u_ab.sh, profiles/r05_unroll_ab.json);
//   * inout is written back with 16-byte stores to the lines it just read;
//   * each packet holds 16/sizeof(unit) elements, combined in registers;
//   * elements before the first 16-byte boundary of inout (head) and after
//     the last full packet (tail) are done element-wise by block 0;
//   * if in and inout disagree modulo 16 bytes, `in` is read with unaligned
//     16-byte loads (gfx950 global loads take element-aligned addresses);
//     only buffers that are not even element-aligned fall back to an
//     element-wise grid-stride kernel.
// Launch geometry: one tile of blockDim*U packets per block, grid =
// ceil(npk / tile) (optionally capped, then grid-stride).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "redop_ops.h"

#ifndef MPIX_REDOP_UNROLL
#define MPIX_REDOP_UNROLL 1
#endif
#ifndef MPIX_REDOP_UNROLL32
// 32-byte units: 64-unit runs per lane per operand -- one since round 5 (two
// before): C_LONG_DOUBLE_COMPLEX and COMPLEX32 SUM +6-7 %, the pair types'
// MINLOC / MAXLOC and the complex PROD even (tools/gpu_u_ab.sh,
// profiles/r05_unroll32_ab.json)
#define MPIX_REDOP_UNROLL32 1
#endif
#ifndef MPIX_REDOP_NT_LOAD
#define MPIX_REDOP_NT_LOAD 1
#endif
#ifndef MPIX_REDOP_NT_STORE
#define MPIX_REDOP_NT_STORE 1
#endif
#ifndef MPIX_REDOP_GROUPED_LOADS
#define MPIX_REDOP_GROUPED_LOADS 1
#endif

namespace mpix {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT> __device__ __forceinline__ v4u ld16(const v4u *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NT> __device__ __forceinline__ void st16(v4u *p, v4u v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// the XCD this wave runs on (0-7; a hardware register, read-only)
__device__ __forceinline__ unsigned xcc_id()
{
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x;
}

// write-through 16-byte store (global_store_dwordx4 ... sc0 sc1)
__device__ __forceinline__ void st16_wt(v4u *p, v4u v)
{
    typedef __attribute__((address_space(1))) v4u gv4u;
    *(volatile gv4u *) (gv4u *) p = v;
}

// the store policy of this block (Params::wt_*): write-through or not,
// uniform per block
__device__ __forceinline__ bool wt_block(const Params &prm)
{
    bool wt = blockIdx.x >= prm.wt_from ||
              (prm.wt_every && blockIdx.x % prm.wt_every == prm.wt_phase);
    if (prm.wt_xcd)
        wt = wt || ((prm.wt_xcd >> (xcc_id() & 7)) & 1);
    return wt;
}

template <bool NT> __device__ __forceinline__ void st16_pol(v4u *p, v4u v, bool wt)
{
    if (wt)
        st16_wt(p, v);
    else
        st16<NT>(p, v);
}

// 16-byte load from an address that is only element-aligned: gfx950 global
// loads accept unaligned addresses, so this is still one global_load_dwordx4.
__device__ __forceinline__ v4u ld16u(const char *p)
{
    v4u v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

// 1-byte combiners may provide apply4(dword, dword): four elements at once
template <class C, class = void> struct HasApply4 {
    static constexpr bool value = false;
};
template <class C>
struct HasApply4<C, decltype((void) C::apply4(0u, 0u))> {
    static constexpr bool value = sizeof(typename C::unit) == 1;
};

// ... or apply4p(dword, dword, prm) when they need the runtime parameters
template <class C, class = void> struct HasApply4P {
    static constexpr bool value = false;
};
template <class C>
struct HasApply4P<C, decltype((void) C::apply4p(0u, 0u, *(const Params *) nullptr))> {
    static constexpr bool value = sizeof(typename C::unit) == 1;
};

template <class C> __device__ __forceinline__ v4u combine16(v4u a, v4u b, const Params &prm)
{
    if constexpr (HasApply4P<C>::value) {
        v4u r;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            r[e] = C::apply4p(a[e], b[e], prm);
        return r;
    }
    if constexpr (HasApply4<C>::value) {
        v4u r;
#pragma unroll
        for (int e = 0; e < 4; ++e)
            r[e] = C::apply4(a[e], b[e]);
        return r;
    }
    using T = typename C::unit;
    constexpr int E = 16 / sizeof(T);
    struct alignas(16) Pk { T u[E]; };
    static_assert(sizeof(Pk) == 16, "unit must divide 16 bytes");
    Pk pa = __builtin_bit_cast(Pk, a);
    Pk pb = __builtin_bit_cast(Pk, b);
#pragma unroll
    for (int e = 0; e < E; ++e)
        pa.u[e] = C::apply(pa.u[e], pb.u[e], prm);
    return __builtin_bit_cast(v4u, pa);
}

// AIN: `in` has the same 16-byte phase as `io` (packet loads); otherwise it
// is only element-aligned and its packets are read with unaligned loads
// (still one dwordx4 per lane; the lines are shared with the neighbours').
// GRP: issue all U `inout` packet loads, then all U `in` loads (instead of
// alternating them per packet)
// The body of one contiguous combine as block `bid` of `nblk` (k_contig: the
// launch's own block; k_batch: a block of its segment).
template <class C, int U, bool NTL, bool NTS, bool AIN, bool GRP>
__device__ __forceinline__ void
contig_body(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io,
            uint64_t head, uint64_t npk, uint64_t tail_start, uint32_t ntail, const Params &prm,
            uint64_t bid, uint64_t nblk, uint64_t nt)
{
    const v4u *__restrict__ vin = reinterpret_cast<const v4u *>(in + head);
    const char *__restrict__ cin = reinterpret_cast<const char *>(in + head);
    v4u *__restrict__ vio = reinterpret_cast<v4u *>(io + head);
    const uint64_t tile = nt * U;
    const uint64_t stride = nblk * tile;
    auto ldin = [&](uint64_t k) -> v4u {
        if constexpr (AIN)
            return ld16<NTL>(vin + k);
        else
            return ld16u(cin + 16 * k);
    };
    const bool wt = wt_block(prm);
    auto st = [&](v4u *p, v4u v) { st16_pol<NTS>(p, v, wt); };
    for (uint64_t i = bid * tile + threadIdx.x; i < npk; i += stride) {
        if (i + (U - 1) * nt < npk) {
            v4u a[U], b[U];
            if constexpr (GRP) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    a[u] = ld16<NTL>(vio + i + u * nt);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    b[u] = ldin(i + u * nt);
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    a[u] = ld16<NTL>(vio + i + u * nt);
                    b[u] = ldin(i + u * nt);
                }
            }
            // every load of the tile is issued before the first combine: left
            // alone, the scheduler sinks the last loads of the wider combiners
            // (1-byte ints, fp16 complex) below the first packet's combine, so
            // fewer bytes are in flight per wave (tools/isa_seq.py)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u)
                st(vio + i + u * nt, combine16<C>(a[u], b[u], prm));
        } else {
            for (int u = 0; u < U; ++u) {
                uint64_t k = i + u * nt;
                if (k < npk)
                    st16<NTS>(vio + k, combine16<C>(ld16<NTL>(vio + k), ldin(k), prm));
            }
        }
    }
    if (bid == 0) {
        for (uint64_t t = threadIdx.x; t < head; t += nt)
            io[t] = C::apply(io[t], in[t], prm);
        for (uint64_t t = threadIdx.x; t < ntail; t += nt)
            io[tail_start + t] = C::apply(io[tail_start + t], in[tail_start + t], prm);
    }
}

// The grid and block sizes come in as arguments (nblk, nt): a kernel that
// reads gridDim / blockDim gets the runtime's hidden-argument block appended
// to its kernel arguments (360 instead of 112 bytes here), which the host
// writes on every launch.
template <class C, int U, bool NTL, bool NTS, bool AIN = true, bool GRP = MPIX_REDOP_GROUPED_LOADS>
__global__ void __launch_bounds__(1024)
k_contig(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io,
         uint64_t head, uint64_t npk, uint64_t tail_start, uint32_t ntail, Params prm,
         uint32_t nblk, uint32_t nt)
{
    contig_body<C, U, NTL, NTS, AIN, GRP>(in, io, head, npk, tail_start, ntail, prm, blockIdx.x,
                                          nblk, nt);
    if (prm.done) {     // small synchronous call (launch_contig sets it)
        __threadfence();            // every wave: its stores complete
        __syncthreads();
        if (threadIdx.x == 0) {
            bool last = true;
            if (nblk > 1) {         // the last workgroup to arrive signals
                last = atomicAdd(prm.done_ctr, 1u) == nblk - 1;
                if (last)
                    *prm.done_ctr = 0;
            }
            if (last) {
                __threadfence_system();     // L2 written back for the host
                __hip_atomic_store(prm.done, prm.done_seq, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// Batch of independent contiguous combines in one launch
// (MPIX_Reduce_local_batch_async): segment s owns blocks [blk0, blk0 + nblk)
// of the grid, one tile each, laid out exactly as a k_contig launch of that
// segment alone would lay them out (same head / packets / tail split, same
// per-element combine), so the bits are those of one call per segment.
constexpr int kMaxBatch = kMaxBatchSegs;
struct BatchSeg {
    const void *in;
    void *io;
    uint64_t npk;
    uint8_t head, ntail, ain, pad[5];
};
struct BatchTab {
    uint32_t blk0[kMaxBatch];   // first block of each segment, ascending, blk0[0] = 0
    BatchSeg s[kMaxBatch];
};
static_assert(kMaxBatch <= 64, "one wave looks the segment up");

template <class C, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(1024)
k_batch(BatchTab tab, int nseg, Params prm, uint32_t nblk, uint32_t nt)
{
    using T = typename C::unit;
    constexpr uint64_t E = 16 / sizeof(T);
    const uint32_t b = blockIdx.x;
    // the segment of this block, the last with blk0 <= b: lane i of every
    // wave reads blk0[i], one ballot counts them (no serial scan of the table)
    const uint32_t lane = threadIdx.x & 63;
    const bool le = lane < (uint32_t) nseg && tab.blk0[lane] <= b;
    const int q = __popcll(__ballot(le)) - 1;
    const BatchSeg &g = tab.s[q];
    const uint32_t first = tab.blk0[q];
    const uint32_t next = q + 1 < nseg ? tab.blk0[q + 1] : nblk;
    const T *in = static_cast<const T *>(g.in);
    T *io = static_cast<T *>(g.io);
    const uint64_t tail_start = g.head + g.npk * E;
    if (g.ain)
        contig_body<C, U, NTL, NTS, true, MPIX_REDOP_GROUPED_LOADS>(
            in, io, g.head, g.npk, tail_start, g.ntail, prm, b - first, next - first, nt);
    else
        contig_body<C, U, NTL, NTS, false, MPIX_REDOP_GROUPED_LOADS>(
            in, io, g.head, g.npk, tail_start, g.ntail, prm, b - first, next - first, nt);
}

// Multi-input combine: inout = OP(...OP(OP(inout, in[0]), in[1])..., in[k-1]),
// i.e. k back-to-back MPIR_Reduce_local calls in that order -- the same
// association, so the same bits -- in ONE pass over HBM: (k+2) x bytes
// instead of 3k x bytes.  Used by the pairwise reduce-scatter, whose k
// received blocks arrive together.
constexpr int kMaxMulti = 16;
template <typename T> struct MultiIn {
    const T *p[kMaxMulti];
};

template <class C, int U>
__global__ void __launch_bounds__(1024)
k_contig_multi(MultiIn<typename C::unit> ins, int k, typename C::unit *__restrict__ io,
               uint64_t head, uint64_t npk, uint64_t tail_start, uint32_t ntail, Params prm,
               uint32_t nblk, uint32_t nthreads)
{
    v4u *__restrict__ vio = reinterpret_cast<v4u *>(io + head);
    const uint64_t nt = nthreads;
    const uint64_t tile = nt * U;
    const uint64_t stride = (uint64_t) nblk * tile;
    const bool wt = wt_block(prm);
    // one input packet live beside the accumulator: input q is loaded, then
    // combined, then input q + 1 (round 6; the round-5 form loaded q + 1
    // before combining q, and its copy forced a full wait anyway), with the
    // launch capping the waves per SIMD (launch_multi, kMultiLds)
    // (tools/multi_fold_probe.hip, profiles/r06_multi_fold_caps2.json)
    for (uint64_t i = (uint64_t) blockIdx.x * tile + threadIdx.x; i < npk; i += stride) {
        v4u acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * nt < npk)
                acc[u] = ld16<true>(vio + i + u * nt);
        for (int q = 0; q < k; ++q) {
            const v4u *__restrict__ vin = reinterpret_cast<const v4u *>(ins.p[q] + head);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (i + u * nt < npk)
                    acc[u] = combine16<C>(acc[u], ld16<true>(vin + i + u * nt), prm);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * nt < npk)
                st16_pol<true>(vio + i + u * nt, acc[u], wt);
    }
    if (blockIdx.x == 0) {
        for (uint64_t t = threadIdx.x; t < head; t += nt) {
            typename C::unit a = io[t];
            for (int q = 0; q < k; ++q)
                a = C::apply(a, ins.p[q][t], prm);
            io[t] = a;
        }
        for (uint64_t t = threadIdx.x; t < ntail; t += nt) {
            typename C::unit a = io[tail_start + t];
            for (int q = 0; q < k; ++q)
                a = C::apply(a, ins.p[q][tail_start + t], prm);
            io[tail_start + t] = a;
        }
    }
}

template <class C>
__global__ void __launch_bounds__(1024)
k_elem_multi(MultiIn<typename C::unit> ins, int k, typename C::unit *__restrict__ io, uint64_t n,
             Params prm, uint32_t nblk, uint32_t nt)
{
    const uint64_t stride = (uint64_t) nblk * nt;
    for (uint64_t i = (uint64_t) blockIdx.x * nt + threadIdx.x; i < n; i += stride) {
        typename C::unit a = io[i];
        for (int q = 0; q < k; ++q)
            a = C::apply(a, ins.p[q][i], prm);
        io[i] = a;
    }
}

// Tree combine: k = 2^L slots folded pairwise by levels, level m = 1, 2, 4,
// ...: slot s (bit m clear) = OP(inout = slot s, in = slot s + m), result =
// slot 0, written to `out` (which may be slot 0's buffer).  With the slots
// holding the peers of rank r in the order r ^ bitrev(s) this is the
// recursive-halving association of rank r's block (…recursive_halving.c:
// 164-229: each step the partner's partial is `in`, the own partial
// `inout`), computed in one pass that reads the k blocks (over xGMI for the
// peers') and writes one.  `pres` marks the slots that hold an operand: an
// absent slot's partner passes through unchanged (the reference's fold of a
// non-power-of-two world, where half of the first level has no partner).
// Unused slots (s >= k) are compile-time registers whose loads and combines
// are skipped by uniform branches, so one instantiation serves every k.
template <int KMAX, class V, class F>
__device__ __forceinline__ void tree_fold(V *v, int k, uint32_t pres, F f)
{
#pragma unroll
    for (int m = 1; m < KMAX; m <<= 1) {
#pragma unroll
        for (int q = 0; q < KMAX; q += 2 * m)
            if (q + m < k) {
                const bool a = (pres >> q) & 1u, b = (pres >> (q + m)) & 1u;
                if (a && b)
                    v[q] = f(v[q], v[q + m]);
                else if (b)
                    v[q] = v[q + m];
            }
        pres |= pres >> m;
    }
}

template <class C, int KMAX, int U>
__global__ void __launch_bounds__(256)
k_contig_tree(MultiIn<typename C::unit> ins, int k, uint32_t pres, typename C::unit *__restrict__ out,
              uint64_t head, uint64_t npk, uint64_t tail_start, uint32_t ntail, Params prm)
{
    using T = typename C::unit;
    v4u *vout = reinterpret_cast<v4u *>(out + head);
    // gridDim / blockDim kept here: the same kernel with the sizes as
    // arguments measured 2.5 % slower at k = 4 and 8 (tools/multi_probe.py)
    const uint64_t nt = blockDim.x;
    const uint64_t stride = (uint64_t) gridDim.x * nt * U;
    auto cv = [&](v4u a, v4u b) { return combine16<C>(a, b, prm); };
    auto ce = [&](T a, T b) { return C::apply(a, b, prm); };
    const bool wt = wt_block(prm);
    for (uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x; i < npk; i += stride) {
        v4u v[U][KMAX];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int q = 0; q < KMAX; ++q)
                if (q < k && ((pres >> q) & 1u) && i + u * nt < npk)
                    v[u][q] = ld16<true>(reinterpret_cast<const v4u *>(ins.p[q] + head) + i + u * nt);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + u * nt >= npk)
                continue;
            tree_fold<KMAX>(v[u], k, pres, cv);
            st16_pol<true>(vout + i + u * nt, v[u][0], wt);
        }
    }
    if (blockIdx.x == 0) {
        auto one = [&](uint64_t t) {
            T v[KMAX];
#pragma unroll
            for (int q = 0; q < KMAX; ++q)
                if (q < k && ((pres >> q) & 1u))
                    v[q] = ins.p[q][t];
            tree_fold<KMAX>(v, k, pres, ce);
            out[t] = v[0];
        };
        for (uint64_t t = threadIdx.x; t < head; t += nt)
            one(t);
        for (uint64_t t = threadIdx.x; t < ntail; t += nt)
            one(tail_start + t);
    }
}

// The same fold as a compile-time recursion over slot ranges [LO, LO + LEN):
// left half = inout, right half = in, an absent half passes the other through
// -- tree_fold's association exactly, with at most log2(KMAX) + 1 partial
// results live instead of KMAX slots (the 32-byte units would not fit the
// registers otherwise).  Returns whether any slot of the range is present.
template <int LO, int LEN, class T, class L, class F>
__device__ __forceinline__ bool tree_fold_rec(T &out, int k, uint32_t pres, L &load, F &f)
{
    if constexpr (LEN == 1) {
        if (LO < k && ((pres >> LO) & 1u)) {
            out = load(LO);
            return true;
        }
        return false;
    } else {
        T a, b;
        const bool ha = tree_fold_rec<LO, LEN / 2>(a, k, pres, load, f);
        if (LO + LEN / 2 >= k) {
            out = a;
            return ha;
        }
        const bool hb = tree_fold_rec<LO + LEN / 2, LEN / 2>(b, k, pres, load, f);
        out = (ha && hb) ? f(a, b) : (hb ? b : a);
        return ha || hb;
    }
}

// The tree fold in tree_fold_rec's order (pairs (0,1), (2,3), their sum, ...)
// with U packets per lane: the slots are loaded as the recursion reaches
// them, so the compiler may keep fewer of them live (more waves per SIMD)
// instead of issuing all KMAX x U loads up front as k_contig_tree does.
template <int U> struct PkU {
    v4u x[U];
};

template <class C, int KMAX, int U>
__global__ void __launch_bounds__(256)
k_contig_tree_rec(MultiIn<typename C::unit> ins, int k, uint32_t pres,
                  typename C::unit *__restrict__ out, uint64_t head, uint64_t npk,
                  uint64_t tail_start, uint32_t ntail, Params prm)
{
    using T = typename C::unit;
    v4u *vout = reinterpret_cast<v4u *>(out + head);
    const uint64_t nt = blockDim.x;
    const uint64_t stride = (uint64_t) gridDim.x * nt * U;
    const bool wt = wt_block(prm);
    for (uint64_t i = (uint64_t) blockIdx.x * nt * U + threadIdx.x; i < npk; i += stride) {
        auto load = [&](int q) {
            PkU<U> v;
            const v4u *p = reinterpret_cast<const v4u *>(ins.p[q] + head) + i;
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (i + u * nt < npk)
                    v.x[u] = ld16<true>(p + u * nt);
            return v;
        };
        auto f = [&](PkU<U> a, const PkU<U> &b) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                a.x[u] = combine16<C>(a.x[u], b.x[u], prm);
            return a;
        };
        PkU<U> r;
        tree_fold_rec<0, KMAX>(r, k, pres, load, f);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * nt < npk)
                st16_pol<true>(vout + i + u * nt, r.x[u], wt);
    }
    if (blockIdx.x == 0) {
        auto ce = [&](T a, T b) { return C::apply(a, b, prm); };
        auto one = [&](uint64_t t) {
            auto ld = [&](int q) { return ins.p[q][t]; };
            T r;
            tree_fold_rec<0, KMAX>(r, k, pres, ld, ce);
            out[t] = r;
        };
        for (uint64_t t = threadIdx.x; t < head; t += nt)
            one(t);
        for (uint64_t t = threadIdx.x; t < ntail; t += nt)
            one(tail_start + t);
    }
}

// the same fold element by element, for operands not sharing a 16-byte phase
// (and every 32-byte unit)
template <class C>
__global__ void __launch_bounds__(256)
k_elem_tree(MultiIn<typename C::unit> ins, int k, uint32_t pres, typename C::unit *__restrict__ out,
            uint64_t n, Params prm)
{
    using T = typename C::unit;
    auto ce = [&](T a, T b) { return C::apply(a, b, prm); };
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
        if constexpr (sizeof(T) > 16) {
            auto load = [&](int q) { return ins.p[q][t]; };
            T r;
            tree_fold_rec<0, kMaxMulti>(r, k, pres, load, ce);
            out[t] = r;
        } else {
            T v[kMaxMulti];
#pragma unroll
            for (int q = 0; q < kMaxMulti; ++q)
                if (q < k && ((pres >> q) & 1u))
                    v[q] = ins.p[q][t];
            tree_fold<kMaxMulti>(v, k, pres, ce);
            out[t] = v[0];
        }
    }
}

template <class C>
__global__ void __launch_bounds__(1024)
k_elem(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io, uint64_t n,
       Params prm, uint32_t nblk, uint32_t nt)
{
    const uint64_t stride = (uint64_t) nblk * nt;
    for (uint64_t i = (uint64_t) blockIdx.x * nt + threadIdx.x; i < n; i += stride)
        io[i] = C::apply(io[i], in[i], prm);
}

// 32-byte units (long double / binary128 pairs and complex), both operands
// 16-byte aligned.  Loads and stores stay k_contig's: lane l of a wave reads
// packets l and 64 + l of the wave's 128-packet (64-unit) run, so every
// instruction moves 1 KiB of whole lines (a unit per lane, its two packets 32
// bytes apart, would move half lines per instruction).  Adjacent lanes then
// swap one packet (DPP, no LDS): the even lane of a pair holds unit m of the
// run, the odd lane unit 32 + m; after the combine the same swap restores the
// packet layout for the stores.  U runs per lane per operand in flight, all
// loads of the tile before the first combine, the store policy per block.
// Full tiles only; the last partial tile goes a unit per lane.
struct alignas(16) Pk32 {
    v4u lo, hi;
};
#ifndef MPIX_REDOP_BLOCK32
#define MPIX_REDOP_BLOCK32 64       // k_contig32 / k_batch32 block
#endif
#ifdef MPIX_C32_WAVES_N
#define MPIX_C32_WAVES __attribute__((amdgpu_waves_per_eu(MPIX_C32_WAVES_N)))
#else
#define MPIX_C32_WAVES
#endif

// Split combiners (C::kSplit, the soft complex products): C::apply_fast(a, b,
// prm, ok) runs only the normal-operand fast paths and sets ok false when any
// of them declines (its result is then unspecified); the contiguous 32-byte
// kernel leaves such a unit as it was, records it in Params::fixup (one 64-bit word per 64 units, written
// for every group) and k_fixup32 combines the recorded units with the full
// C::apply in a second launch.  The general paths stay out of the streaming
// kernel, whose registers -- and so its waves per SIMD -- are the fast path's
// (QuadCProd: 107 VGPRs with the general paths inline, 70 without; it is
// VALU- and latency-bound).
template <class C, class = void> struct is_split : std::false_type {};
template <class C> struct is_split<C, std::void_t<decltype(C::kSplit)>>
    : std::integral_constant<bool, C::kSplit> {};

// the 64-bit lane mask of contig32's gathered layout (lane 2m holds unit m of
// the run, lane 2m + 1 unit 32 + m) in unit order
__device__ __forceinline__ uint64_t lanes_to_units(uint64_t m)
{
    auto even = [](uint64_t x) {
        x &= 0x5555555555555555ull;
        x = (x | (x >> 1)) & 0x3333333333333333ull;
        x = (x | (x >> 2)) & 0x0f0f0f0f0f0f0f0full;
        x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
        x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
        return (x | (x >> 16)) & 0x00000000ffffffffull;
    };
    return even(m) | (even(m >> 1) << 32);
}

// ok ? r : a, a component at a time (a select of the two aggregates compiles
// to a pointer select over stack copies: scratch)
__device__ __forceinline__ Pk32 select_pk(bool ok, const Pk32 &r, const Pk32 &a)
{
    Pk32 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        o.lo[e] = ok ? r.lo[e] : a.lo[e];
        o.hi[e] = ok ? r.hi[e] : a.hi[e];
    }
    return o;
}

// v from the other lane of each adjacent pair (quad_perm [1,0,3,2])
__device__ __forceinline__ v4u swap_pair(v4u v)
{
    v4u r;
#pragma unroll
    for (int e = 0; e < 4; ++e)
        r[e] = (unsigned) __builtin_amdgcn_mov_dpp((int) v[e], 0xB1, 0xF, 0xF, false);
    return r;
}

// Tile t (tile = nt * U units) of one 32-byte combine: a full tile through
// the packet loads and the lane swap, the last partial tile a unit per lane.
// Block-uniform: every lane of the block takes the same branch (the swap
// needs whole waves).
template <class C, int U, bool NTL, bool NTS>
__device__ __forceinline__ void contig32_tile(const typename C::unit *in, const typename C::unit *io,
                                              typename C::unit *out, uint64_t n, uint64_t t,
                                              uint64_t nt, bool wt, const Params &prm)
{
    using T = typename C::unit;
    static_assert(sizeof(T) == 32, "32-byte units");
    const v4u *vin = reinterpret_cast<const v4u *>(in);
    const v4u *vio = reinterpret_cast<const v4u *>(io);     // the inout role (read)
    v4u *vout = reinterpret_cast<v4u *>(out);               // io itself, or the tree's output
    constexpr bool split = is_split<C>::value;
    bool ok = true;
    auto f = [&](const Pk32 &a, const Pk32 &b) {
        if constexpr (split)
            return __builtin_bit_cast(Pk32, C::apply_fast(__builtin_bit_cast(T, a),
                                                          __builtin_bit_cast(T, b), prm, ok));
        else
            return __builtin_bit_cast(Pk32, C::apply(__builtin_bit_cast(T, a),
                                                     __builtin_bit_cast(T, b), prm));
    };
    // one fixup word per 64 units (every group written: the buffer is reused)
    auto record = [&](uint64_t unit0, uint64_t mask) {
        if constexpr (split)
            if ((threadIdx.x & 63) == 0)
                prm.fixup[unit0 >> 6] = mask;
    };
    const uint64_t tile = nt * U;
    // (the split combiners too: a unit per lane for every tile, two 16-byte
    // loads 16 bytes apart, saves the swaps' selects and DPP moves but ran
    // COMPLEX32 PROD 4.97 -> 4.51 and C_LONG_DOUBLE_COMPLEX PROD 6.24 -> 4.47
    // TB/s, profiles/r06_soft_rows_ab6.jsonl)
#ifndef MPIX_C32_LDS
#define MPIX_C32_LDS 1
#endif
    if ((t + 1) * tile <= n) {
        if constexpr (split && MPIX_C32_LDS) {
            // the split combiners are issue-bound: the packets go through LDS
            // (unit m of the run = packets 2m, 2m + 1 to lane m), which costs
            // no VALU, instead of the DPP swap and its selects; the lane's
            // unit is then in run order, so its ballot is the fixup word
            __shared__ v4u lds[MPIX_REDOP_BLOCK32 / 64][2][128];
            const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            v4u *la = lds[wave][0], *lb = lds[wave][1];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t run0 = t * tile + u * nt + wave * 64;
                const uint64_t q = 2 * run0 + lane;
                const v4u a0 = ld16<NTL>(vio + q), a1 = ld16<NTL>(vio + q + 64);
                const v4u b0 = ld16<NTL>(vin + q), b1 = ld16<NTL>(vin + q + 64);
                la[lane] = a0;
                la[lane + 64] = a1;
                lb[lane] = b0;
                lb[lane + 64] = b1;
                __syncthreads();
                const Pk32 r = f(Pk32{la[2 * lane], la[2 * lane + 1]},
                                 Pk32{lb[2 * lane], lb[2 * lane + 1]});
                __syncthreads();
                if (ok) {       // a declined unit stays as it was (k_fixup32 reads it)
                    la[2 * lane] = r.lo;
                    la[2 * lane + 1] = r.hi;
                }
                __syncthreads();
                st16_pol<NTS>(vout + q, la[lane], wt);
                st16_pol<NTS>(vout + q + 64, la[lane + 64], wt);
                record(run0, __ballot(!ok));
                __syncthreads();
            }
        } else {
            const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            const bool odd = lane & 1;
            // the unit a lane holds after the swap: run unit lane/2 (even) or 32 + lane/2 (odd)
            auto gather = [&](v4u p0, v4u p1) {
                const v4u y = swap_pair(odd ? p0 : p1);
                return odd ? Pk32{y, p1} : Pk32{p0, y};
            };
            v4u a0[U], a1[U], b0[U], b1[U];
            // run u of this wave: units [t*tile + u*nt + wave*64, +64) = packets from q
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t q = 2 * (t * tile + u * nt + wave * 64) + lane;
                a0[u] = ld16<NTL>(vio + q);
                a1[u] = ld16<NTL>(vio + q + 64);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t q = 2 * (t * tile + u * nt + wave * 64) + lane;
                b0[u] = ld16<NTL>(vin + q);
                b1[u] = ld16<NTL>(vin + q + 64);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const Pk32 ga = gather(a0[u], a1[u]);
                Pk32 r = f(ga, gather(b0[u], b1[u]));
                if constexpr (split)
                    r = select_pk(ok, r, ga);   // a declined unit stays as it was
                const v4u y = swap_pair(odd ? r.lo : r.hi);
                const uint64_t q = 2 * (t * tile + u * nt + wave * 64) + lane;
                st16_pol<NTS>(vout + q, odd ? y : r.lo, wt);
                st16_pol<NTS>(vout + q + 64, odd ? r.hi : y, wt);
                if constexpr (split)
                    record(t * tile + u * nt + wave * 64, lanes_to_units(__ballot(!ok)));
            }
        }
    } else {
        const uint64_t end = (t + 1) * tile < n ? (t + 1) * tile : n;    // this tile only
        for (uint64_t k = t * tile + threadIdx.x; k < end; k += nt) {
            const Pk32 a{ld16<NTL>(vio + 2 * k), ld16<NTL>(vio + 2 * k + 1)};
            Pk32 r = f(a, Pk32{ld16<NTL>(vin + 2 * k), ld16<NTL>(vin + 2 * k + 1)});
            if constexpr (split)
                r = select_pk(ok, r, a);    // a declined unit stays as it was
            st16_pol<NTS>(vout + 2 * k, r.lo, wt);
            st16_pol<NTS>(vout + 2 * k + 1, r.hi, wt);
            if constexpr (split)        // a unit per lane: the mask is in unit order
                record(k - (threadIdx.x & 63), __ballot(!ok));
        }
    }
}

template <class C, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) MPIX_C32_WAVES
k_contig32(const typename C::unit *in, const typename C::unit *io, typename C::unit *out, uint64_t n,
           Params prm, uint32_t nblk, uint32_t nthreads)
{
    const uint64_t tile = (uint64_t) nthreads * U;
    const uint64_t ntiles = (n + tile - 1) / tile;
    const bool wt = wt_block(prm);
    for (uint64_t t = blockIdx.x; t < ntiles; t += nblk)
        contig32_tile<C, U, NTL, NTS>(in, io, out, n, t, nthreads, wt, prm);
}

// The second launch of a split combiner: every unit the fast kernel recorded
// in the fixup words (it left them unchanged in `out`), combined with the full
// C::apply from the untouched operands (`io` is `out` in place, or the tree's
// separate inout role).  A wave loads 64 consecutive words (one per lane),
// skips them at once when all are zero (the usual case), and otherwise walks
// them in order: word j's units are combined by the lanes whose bit is set,
// lane l taking unit 64 (base + j) + l, so the loads and stores of a densely
// marked word are coalesced (a lane per word, walking its own 64 units, had
// each load hit 64 lines 2 KiB apart: real values stored as complex, where
// every unit declines, ran at 1.6 TB/s; profiles/r06_soft_zero_im.json).
template <class C>
__global__ void __launch_bounds__(256)
k_fixup32(const typename C::unit *in, const typename C::unit *io, typename C::unit *out, uint64_t n,
          Params prm, uint32_t nblk)
{
    const uint64_t nw = (n + 63) / 64;
    const unsigned lane = threadIdx.x & 63;
    for (uint64_t wb = (uint64_t) blockIdx.x * 256 + (threadIdx.x & ~63u); wb < nw;
         wb += (uint64_t) nblk * 256) {
        const uint64_t mine = wb + lane < nw ? prm.fixup[wb + lane] : 0;
        if (__ballot(mine != 0) == 0)
            continue;
        for (int j = 0; j < 64; ++j) {
            const uint32_t lo = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) mine, j);
            const uint32_t hi = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) (mine >> 32), j);
            const uint64_t m = ((uint64_t) hi << 32) | lo;
            if (m == 0)
                continue;
            const uint64_t u = (wb + j) * 64 + lane;
            if (((m >> lane) & 1) && u < n)
                out[u] = C::apply(io[u], in[u], prm);
        }
    }
}

// The batch entry's form for 32-byte units: segment s owns blocks [blk0,
// blk0 + its tiles), one tile each (BatchSeg::npk holds its count in units),
// each tile combined as k_contig32 combines it.
template <class C, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256)
k_batch32(BatchTab tab, int nseg, Params prm, uint32_t nt)
{
    using T = typename C::unit;
    const uint32_t b = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const bool le = lane < (uint32_t) nseg && tab.blk0[lane] <= b;
    const int q = __popcll(__ballot(le)) - 1;
    const BatchSeg &g = tab.s[q];
    contig32_tile<C, U, NTL, NTS>(static_cast<const T *>(g.in), static_cast<const T *>(g.io),
                                  static_cast<T *>(g.io), g.npk, b - tab.blk0[q], nt,
                                  wt_block(prm), prm);
}

// Vector target (typerep_op.c:115-150 for MPI_Type_vector(count, bl, stride)):
// packed source element j = b*bl + k lands on target element b*stride + k.
// Thread per source element: the source stream is fully coalesced, the
// target reads/writes are coalesced within each block run; gap elements are
// never loaded or stored.
template <class C>
__global__ void __launch_bounds__(1024)
k_vector(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io, uint64_t n,
         uint64_t bl, uint64_t st, Params prm, uint32_t nblk, uint32_t nt)
{
    const uint64_t stride = (uint64_t) nblk * nt;
    for (uint64_t j = (uint64_t) blockIdx.x * nt + threadIdx.x; j < n; j += stride) {
        uint64_t b = j / bl, k = j - b * bl;
        uint64_t t = b * st + k;
        io[t] = C::apply(io[t], in[j], prm);
    }
}

// bl == 1 specialisation: no division
template <class C>
__global__ void __launch_bounds__(1024)
k_vector1(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io, uint64_t n,
          uint64_t st, Params prm, uint32_t nblk, uint32_t nt)
{
    const uint64_t stride = (uint64_t) nblk * nt;
    for (uint64_t j = (uint64_t) blockIdx.x * nt + threadIdx.x; j < n; j += stride)
        io[j * st] = C::apply(io[j * st], in[j], prm);
}

// (bl, stride) = (1, 2), config 5: each lane loads the whole 2-element target
// pair {payload, gap} as one vector load (the line is fetched whole anyway,
// and one 16-B load per lane issues half the requests of two 8-B ones), then
// stores the payload element only; plain (non-temporal-free) policy so the
// half-line stores merge with the lines still held in L2 (measured: +10 %
// over 8-B target loads, non-temporal -25 %; profiles/r01_tune_vector.txt).
template <int N> struct RawOf;
template <> struct RawOf<2> { typedef unsigned short type; };
template <> struct RawOf<4> { typedef unsigned int type; };
template <> struct RawOf<8> { typedef unsigned int type __attribute__((ext_vector_type(2))); };
template <> struct RawOf<16> { typedef unsigned int type __attribute__((ext_vector_type(4))); };
template <> struct RawOf<32> { typedef unsigned int type __attribute__((ext_vector_type(8))); };

// Payload store of the stride-2 vector target, write-through (global_store
// sc0 sc1: the half-written line leaves L2 at once instead of waiting dirty
// for eviction) for 1..8-byte units: +1.9 % at the 2.5 GiB traffic floor of
// config 5, same FETCH/WRITE bytes (profiles/r02_tune_vector2.txt,
// tools/tune_vector2.hip S1 vs S0).  A relaxed system-scope atomic store is
// only the cache policy here: no ordering is asked of it.
template <typename T>
__device__ __forceinline__ void st_payload_wt(T *p, const T &v)
{
    if constexpr (sizeof(T) == 8) {
        unsigned long long u;
        __builtin_memcpy(&u, &v, 8);
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    } else if constexpr (sizeof(T) == 4) {
        unsigned int u;
        __builtin_memcpy(&u, &v, 4);
        __hip_atomic_store(reinterpret_cast<unsigned int *>(p), u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        *p = v;
    }
}

// Packed-source load of the stride-2 vector target, non-temporal for 4- and
// 8-byte units (read once, never revisited): with the write-through payload
// store +3.9 % over the default-policy source load at the same traffic
// (profiles/r02_tune_vector2b.txt, tools/tune_vector2.hip S6 vs S1).
template <typename T>
__device__ __forceinline__ T ld_source_nt(const T *p)
{
    if constexpr (sizeof(T) == 8) {
        unsigned long long u = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long *>(p));
        T v;
        __builtin_memcpy(&v, &u, 8);
        return v;
    } else if constexpr (sizeof(T) == 4) {
        unsigned int u = __builtin_nontemporal_load(reinterpret_cast<const unsigned int *>(p));
        T v;
        __builtin_memcpy(&v, &u, 4);
        return v;
    } else {
        return *p;
    }
}

template <class C>
__global__ void __launch_bounds__(256)
k_vector_s2(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io, uint64_t n,
            Params prm, uint32_t nblk, uint32_t nt)
{
    using T = typename C::unit;
    using R = typename RawOf<2 * sizeof(T)>::type;
    const uint64_t stride = (uint64_t) nblk * nt;
    for (uint64_t j = (uint64_t) blockIdx.x * nt + threadIdx.x; j < n; j += stride) {
        T t;
        if (j + 1 < n) {
            R raw = reinterpret_cast<const R *>(io)[j];
            __builtin_memcpy(&t, &raw, sizeof(T));
        } else {    // the last pair would reach one element past the type's span
            t = io[2 * j];
        }
        st_payload_wt(io + 2 * j, C::apply(t, ld_source_nt(in + j), prm));
    }
}

// General derived target given as its flattened iov (typerep_op.c:100-150):
// run s covers seg_off[s] (element offset into inout) .. + its count; its
// source elements start at src_off[s] of the packed source (runs are
// consumed in order, so src_off is the running prefix unless the host split
// the runs by alignment class).  prefix[s] = elements before run s in this
// launch (prefix[nseg] = total).  Thread per element, run found by binary
// search over the L2-resident prefix table.
template <class C>
__global__ void __launch_bounds__(256)
k_iov(const typename C::unit *__restrict__ in, typename C::unit *__restrict__ io,
      const int64_t *__restrict__ seg_off, const int64_t *__restrict__ prefix,
      const int64_t *__restrict__ src_off, int64_t nseg, uint64_t total, Params prm,
      uint32_t nblk)
{
    const uint64_t stride = (uint64_t) nblk * 256;        // 256-thread blocks (launch_iov)
    for (uint64_t j = (uint64_t) blockIdx.x * 256 + threadIdx.x; j < total; j += stride) {
        int64_t lo = 0, hi = nseg - 1;
        while (lo < hi) {               // last s with prefix[s] <= j
            int64_t mid = (lo + hi + 1) >> 1;
            if ((uint64_t) prefix[mid] <= j)
                lo = mid;
            else
                hi = mid - 1;
        }
        const int64_t k = (int64_t) (j - (uint64_t) prefix[lo]);
        const int64_t t = seg_off[lo] + k;
        io[t] = C::apply(io[t], in[src_off[lo] + k], prm);
    }
}

// The store policy (LaunchCfg::wt_*) of a launch of `grid` blocks.
inline void set_store_policy(Params &p, const LaunchCfg &cfg, unsigned grid)
{
    if (cfg.wt_tail > 0)
        p.wt_from = grid > (unsigned) cfg.wt_tail ? grid - (unsigned) cfg.wt_tail : 0u;
    p.wt_every = cfg.wt_every > 0 ? (unsigned) cfg.wt_every : 0u;
    p.wt_phase = (unsigned) cfg.wt_phase;
    p.wt_xcd = (unsigned) cfg.wt_xcd & 0xffu;
}

// k_contig32's block (its __launch_bounds__)
// One-wave blocks for the stride-2 vector target and the 32-byte units too
// (round 5, tools/gpu_u_ab.sh against 256 threads, profiles/r05_block64_vec32.json):
// config 5 0.449 -> 0.433 ms; LONG_DOUBLE_INT MINLOC / MAXLOC 6.74-6.78 ->
// 7.06-7.09 TB/s, the complex long double / binary128 rows even to +2 %
#ifndef MPIX_REDOP_VBLOCK
#define MPIX_REDOP_VBLOCK 64        // the stride-2 vector target's block
#endif
constexpr unsigned kContig32Block = MPIX_REDOP_BLOCK32;

// k_contig32 over 16-byte-aligned 32-byte units (`io` read in the inout
// role, the result to `out`: io itself, or the tree's output); a split
// combiner adds its fixup launch
template <class C>
hipError_t launch_contig32(const typename C::unit *in, const typename C::unit *io,
                           typename C::unit *out, uint64_t count, const Params &prm,
                           const LaunchCfg &cfg, hipStream_t s)
{
    constexpr int U32 = MPIX_REDOP_UNROLL32;
    const unsigned grid = grid_for((uint64_t) kContig32Block * U32, count, cfg.max_grid,
                                   kContig32Block);
    Params p = prm;
    p.done = nullptr;
    set_store_policy(p, cfg, grid);
    if constexpr (is_split<C>::value) {
        p.fixup = fixup_buffer(s, (count + 63) / 64 * sizeof(uint64_t));
        if (!p.fixup)
            return hipErrorOutOfMemory;
    }
    hipLaunchKernelGGL((k_contig32<C, U32, MPIX_REDOP_NT_LOAD, MPIX_REDOP_NT_STORE>), dim3(grid),
                       dim3(kContig32Block), 0, s, in, io, out, count, p, grid, kContig32Block);
    if constexpr (is_split<C>::value) {
        // a word per lane: the scan is one load per lane, mostly of zeros
        const unsigned g2 = grid_for(256, (count + 63) / 64, 0, 256);
        hipLaunchKernelGGL((k_fixup32<C>), dim3(g2), dim3(256), 0, s, in, io, out, count, p, g2);
    }
    return hipGetLastError();
}

// Contiguous launcher: chooses the packet or the element-wise kernel.
template <class C>
hipError_t launch_contig(const void *in, void *io, uint64_t count, const Params &prm,
                         const LaunchCfg &cfg, hipStream_t s)
{
    using T = typename C::unit;
    constexpr uint64_t E = sizeof(T) <= 16 ? 16 / sizeof(T) : 1;
    const T *tin = static_cast<const T *>(in);
    T *tio = static_cast<T *>(io);
    bool signalled = false;
    uintptr_t ai = reinterpret_cast<uintptr_t>(in), ao = reinterpret_cast<uintptr_t>(io);
    if constexpr (sizeof(T) > 16) {
        // 32-byte units (the long double / binary128 pairs and complex): two
        // units of two 16-byte packets per lane and operand, as many bytes in
        // flight as k_contig's four packets; operands off the 16-byte grid go
        // element-wise
        if (((ai | ao) & 15) == 0) {
            hipError_t e = launch_contig32<C>(tin, tio, tio, count, prm, cfg, s);
            if (e != hipSuccess)
                return e;
        } else {
            unsigned grid = grid_for((uint64_t) cfg.block * 4, count, cfg.max_grid, cfg.block);
            hipLaunchKernelGGL((k_elem<C>), dim3(grid), dim3(cfg.block), 0, s, tin, tio, count,
                               prm, grid, (uint32_t) cfg.block);
        }
    } else if ((ao % sizeof(T)) == 0 && (ai % sizeof(T)) == 0) {
        uint64_t head = ((16 - (ao & 15)) & 15) / sizeof(T);
        if (head > count)
            head = count;
        uint64_t npk = (count - head) / E;
        uint64_t tail_start = head + npk * E;
        uint32_t ntail = (uint32_t) (count - tail_start);
        const uint64_t tile = (uint64_t) cfg.block * MPIX_REDOP_UNROLL;
        unsigned grid = grid_for(tile, npk, cfg.max_grid, cfg.block);
        // up to kSignalMaxGrid workgroups (64 KiB per operand at the defaults): the
        // kernel stores the completion word itself (Params::done)
        Params p = prm;
        if (grid > (prm.done_ctr ? kSignalMaxGrid : 1u))
            p.done = nullptr;
        set_store_policy(p, cfg, grid);
        signalled = p.done != nullptr;
        if ((ai & 15) == (ao & 15))
            hipLaunchKernelGGL(
                (k_contig<C, MPIX_REDOP_UNROLL, MPIX_REDOP_NT_LOAD, MPIX_REDOP_NT_STORE, true>),
                dim3(grid), dim3(cfg.block), 0, s, tin, tio, head, npk, tail_start, ntail, p,
                grid, (uint32_t) cfg.block);
        else
            hipLaunchKernelGGL(
                (k_contig<C, MPIX_REDOP_UNROLL, MPIX_REDOP_NT_LOAD, MPIX_REDOP_NT_STORE, false>),
                dim3(grid), dim3(cfg.block), 0, s, tin, tio, head, npk, tail_start, ntail, p,
                grid, (uint32_t) cfg.block);
    } else {
        unsigned grid = grid_for((uint64_t) cfg.block * 4, count, cfg.max_grid, cfg.block);
        hipLaunchKernelGGL((k_elem<C>), dim3(grid), dim3(cfg.block), 0, s, tin, tio, count, prm,
                           grid, (uint32_t) cfg.block);
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && prm.done && !signalled)
        e = hipStreamWriteValue32(s, (void *) prm.done, prm.done_seq, 0);
    return e;
}

// LDS per 64 threads of a multi-input fold block: 160 KiB per CU / 6656 B =
// 24 one-wave blocks = 6 waves per SIMD (the kernel itself uses no LDS)
constexpr unsigned kMultiLds = 6656;

template <class C>
hipError_t launch_multi(const void *const *ins, int k, void *io, uint64_t count, const Params &prm,
                        const LaunchCfg &cfg, hipStream_t s)
{
    using T = typename C::unit;
    constexpr uint64_t E = sizeof(T) <= 16 ? 16 / sizeof(T) : 1;
    MultiIn<T> mi{};
    uintptr_t ao = reinterpret_cast<uintptr_t>(io);
    bool aligned = sizeof(T) <= 16 && (ao % sizeof(T)) == 0;
    for (int q = 0; q < k; ++q) {
        mi.p[q] = static_cast<const T *>(ins[q]);
        aligned = aligned && ((reinterpret_cast<uintptr_t>(ins[q]) & 15) == (ao & 15));
    }
    T *tio = static_cast<T *>(io);
    if constexpr (sizeof(T) > 16)
        aligned = false;
    if (aligned) {
        uint64_t head = ((16 - (ao & 15)) & 15) / sizeof(T);
        if (head > count)
            head = count;
        uint64_t npk = (count - head) / E;
        uint64_t tail_start = head + npk * E;
        uint32_t ntail = (uint32_t) (count - tail_start);
        // one packet per lane per input: 6.16 / 6.20 TB/s at k = 7 (256 MiB /
        // 1 GiB, store policy on) against 6.04 / 5.83 with two; 4 measured no
        // better than 2 (tools/tree8_probe.hip, tools/multi_probe.py)
        constexpr int U = 1;
        unsigned grid = grid_for((uint64_t) cfg.block * U, npk, cfg.max_grid, cfg.block);
        Params p = prm;
        set_store_policy(p, cfg, grid);
        // k >= 2 inputs: unused LDS per block caps the waves per SIMD at 6
        // (24 one-wave blocks per CU): with k + 2 streams per wave fewer
        // waves in flight run faster -- 256 MiB fp32, one-wave blocks, store
        // policy on: k = 3 6.53 -> 6.91, k = 7 6.53 -> 6.92, k = 15 6.38 ->
        // 6.65 TB/s against the round-5 form; the headline kernel (k = 1)
        // loses with any cap (7.04 -> 6.73) and keeps none
        // (profiles/r06_multi_fold_caps2.json)
        size_t lds = 0;
        if (k >= 2) {
            lds = (size_t) kMultiLds * ((unsigned) cfg.block / 64u);
            if (lds > 65536)
                lds = 0;
        }
        if constexpr (sizeof(T) <= 16)
            hipLaunchKernelGGL((k_contig_multi<C, U>), dim3(grid), dim3(cfg.block), lds, s, mi, k,
                               tio, head, npk, tail_start, ntail, p, grid, (uint32_t) cfg.block);
    } else {
        unsigned grid = grid_for((uint64_t) cfg.block * 4, count, cfg.max_grid, cfg.block);
        hipLaunchKernelGGL((k_elem_multi<C>), dim3(grid), dim3(cfg.block), 0, s, mi, k, tio, count,
                           prm, grid, (uint32_t) cfg.block);
    }
    return hipGetLastError();
}

// out = tree fold of ins[0..k-1] (k a power of two, 2..16; k_contig_tree);
// a NULL slot is absent (its partner passes through)
template <class C>
hipError_t launch_tree(const void *const *ins, int k, void *out, uint64_t count, const Params &prm,
                       const LaunchCfg &cfg, hipStream_t s)
{
    using T = typename C::unit;
    constexpr uint64_t E = sizeof(T) <= 16 ? 16 / sizeof(T) : 1;
    MultiIn<T> mi{};
    uintptr_t ao = reinterpret_cast<uintptr_t>(out);
    bool aligned = sizeof(T) <= 16 && (ao % sizeof(T)) == 0;
    uint32_t pres = 0;
    for (int q = 0; q < k; ++q) {
        mi.p[q] = static_cast<const T *>(ins[q]);
        if (!ins[q])
            continue;
        pres |= 1u << q;
        aligned = aligned && ((reinterpret_cast<uintptr_t>(ins[q]) & 15) == (ao & 15));
    }
    T *tout = static_cast<T *>(out);
    if constexpr (sizeof(T) > 16) {
        // out = slot 0 OP slot 1 on 32-byte units, all three 16-byte aligned:
        // k_contig32 with slot 0 in the inout role (recursive halving's
        // combine_to); other shapes go element-wise below
        if (k == 2 && pres == 3u &&
            ((ao | reinterpret_cast<uintptr_t>(ins[0]) | reinterpret_cast<uintptr_t>(ins[1])) & 15) ==
                0) {
            return launch_contig32<C>(mi.p[1], mi.p[0], tout, count, prm, cfg, s);
        }
    }
    if (aligned) {
        uint64_t head = ((16 - (ao & 15)) & 15) / sizeof(T);
        if (head > count)
            head = count;
        uint64_t npk = (count - head) / E;
        uint64_t tail_start = head + npk * E;
        uint32_t ntail = (uint32_t) (count - tail_start);
        Params p = prm;
        // forms by slot count (tools/tree8_probe.hip, profiles/r05_tree_forms.json;
        // fp32 SUM at 256 MiB / 1 GiB per operand, store policy on):
        //   k = 2   the fold order, 2 packets per lane     6.81 / 6.94 TB/s
        //           (all 4 x 2 loads up front: 6.44 / 6.84)
        //   k = 4   all 4 x 2 loads up front               6.40 / 6.61
        //           (the fold order, 1 packet: 6.34 / 6.53)
        //   k = 8   the fold order, 1 packet per lane      6.47 / 6.36
        //           (8 x 2 up front 5.79 / 5.43, 16 x 1 up front 5.68 / 5.22)
        //   k = 16  the fold order, 1 packet per lane      6.37 / 5.92
        //           (16 x 1 up front 5.86 / 5.50)
        // Loading slots only as the fold reaches them keeps 39 VGPRs live at
        // k = 8 (8 waves per SIMD) against 111 for the up-front form (4), and
        // with nine streams the waves, not each wave's bytes in flight, carry
        // the rate.  The store policy: +5 % at k = 2, +3.8 % at k = 4, neutral
        // above.
        // One-wave (64-thread) blocks, as the contiguous kernel: k = 2 / 4 / 8
        // / 16 at 6.84-6.96 / 6.48-6.61 / 6.58-6.67 / 6.06-6.45 TB/s against
        // 6.64-6.76 / 6.36-6.43 / 6.25-6.28 / 5.82-6.43 with 256 threads
        // (r05_tree_forms.json, last run).
        // The public entry takes k = 2, 4, 8, 16 only (the collectives pad an odd
        // world's fold with absent slots); a k between them runs the next
        // larger form, whose uniform branches skip the slots >= k.
        constexpr unsigned kTreeBlock = 64;
        const unsigned per = k <= 4 ? kTreeBlock * 2 : kTreeBlock;
        const unsigned grid = grid_for(per, npk, 0, kTreeBlock);
        set_store_policy(p, cfg, grid);
        if constexpr (sizeof(T) <= 16) {
            if (k <= 2)     // out = a OP b (recursive halving's combine_to)
                hipLaunchKernelGGL((k_contig_tree_rec<C, 2, 2>), dim3(grid), dim3(kTreeBlock), 0, s,
                                   mi, k, pres, tout, head, npk, tail_start, ntail, p);
            else if (k <= 4)
                hipLaunchKernelGGL((k_contig_tree<C, 4, 2>), dim3(grid), dim3(kTreeBlock), 0, s, mi,
                                   k, pres, tout, head, npk, tail_start, ntail, p);
            else if (k <= 8)    // the P = 8 pull's fold
                hipLaunchKernelGGL((k_contig_tree_rec<C, 8, 1>), dim3(grid), dim3(kTreeBlock), 0, s,
                                   mi, k, pres, tout, head, npk, tail_start, ntail, p);
            else
                hipLaunchKernelGGL((k_contig_tree_rec<C, kMaxMulti, 1>), dim3(grid), dim3(kTreeBlock),
                                   0, s, mi, k, pres, tout, head, npk, tail_start, ntail, p);
        }
    } else {
        hipLaunchKernelGGL((k_elem_tree<C>), dim3(grid_for(256 * 4, count, 0, 256)), dim3(256), 0, s,
                           mi, k, pres, tout, count, prm);
    }
    return hipGetLastError();
}

template <class C>
hipError_t launch_vector(const void *in, void *io, uint64_t count, uint64_t bl, uint64_t st,
                         const Params &prm, const LaunchCfg &cfg, hipStream_t s)
{
    using T = typename C::unit;
    uint64_t n = count * bl;
    if (n == 0)
        return hipSuccess;
    if (bl == st)       // contiguous after all
        return launch_contig<C>(in, io, n, prm, cfg, s);
    unsigned grid = grid_for((uint64_t) cfg.block * 4, n, cfg.max_grid, cfg.block);
    bool s2 = false;
    if constexpr (sizeof(T) <= 16)
        s2 = bl == 1 && st == 2 && (reinterpret_cast<uintptr_t>(io) % (2 * sizeof(T))) == 0;
    if (s2) {
        if constexpr (sizeof(T) <= 16) {
            constexpr unsigned kVb = MPIX_REDOP_VBLOCK;
            const unsigned g2 = grid_for(kVb, n, cfg.max_grid, kVb);
            hipLaunchKernelGGL((k_vector_s2<C>), dim3(g2), dim3(kVb), 0, s,
                               static_cast<const T *>(in), static_cast<T *>(io), n, prm, g2, kVb);
        }
    } else if (bl == 1)
        hipLaunchKernelGGL((k_vector1<C>), dim3(grid), dim3(cfg.block), 0, s,
                           static_cast<const T *>(in), static_cast<T *>(io), n, st, prm, grid,
                           (uint32_t) cfg.block);
    else
        hipLaunchKernelGGL((k_vector<C>), dim3(grid), dim3(cfg.block), 0, s,
                           static_cast<const T *>(in), static_cast<T *>(io), n, bl, st, prm, grid,
                           (uint32_t) cfg.block);
    return hipGetLastError();
}

template <class C>
hipError_t launch_iov(const void *in, void *io, const int64_t *d_seg_off, const int64_t *d_prefix,
                      const int64_t *d_src_off, int64_t nseg, uint64_t total, const Params &prm,
                      const LaunchCfg &cfg, hipStream_t s)
{
    using T = typename C::unit;
    if (total == 0 || nseg == 0)
        return hipSuccess;
    unsigned grid = grid_for(256ull * 4, total, cfg.max_grid, 256);
    hipLaunchKernelGGL((k_iov<C>), dim3(grid), dim3(256), 0, s, static_cast<const T *>(in),
                       static_cast<T *>(io), d_seg_off, d_prefix, d_src_off, nseg, total, prm, grid);
    return hipGetLastError();
}

// k independent contiguous combines (no operand range of one overlapping a
// target of another; the caller checked) in one k_batch launch; segments of
// zero count are skipped, segments whose operands are not element-aligned go
// to launch_contig's element-wise kernel, as do all of a 32-byte unit type
template <class C>
hipError_t launch_batch(const void *const *ins, void *const *ios, const uint64_t *counts, int k,
                        const Params &prm, const LaunchCfg &cfg, hipStream_t s)
{
    using T = typename C::unit;
    Params p = prm;
    p.done = nullptr;
    if constexpr (is_split<C>::value) {
        // a split combiner: each triple its own launches (launch_contig: the
        // fast kernel and its fixup)
        for (int i = 0; i < k; ++i)
            if (counts[i]) {
                hipError_t e = launch_contig<C>(ins[i], ios[i], counts[i], p, cfg, s);
                if (e != hipSuccess)
                    return e;
            }
        return hipSuccess;
    } else if constexpr (sizeof(T) > 16) {
        // 32-byte units: the 16-byte-aligned triples as one k_batch32 launch,
        // the others element-wise one launch each
        constexpr int U32 = MPIX_REDOP_UNROLL32;
        const uint64_t tile = (uint64_t) kContig32Block * U32;
        BatchTab tab;
        int n = 0;
        uint64_t blocks = 0;
        auto flush = [&]() -> hipError_t {
            if (!n)
                return hipSuccess;
            Params q = p;
            set_store_policy(q, cfg, (unsigned) blocks);
            hipLaunchKernelGGL((k_batch32<C, U32, MPIX_REDOP_NT_LOAD, MPIX_REDOP_NT_STORE>),
                               dim3((unsigned) blocks), dim3(kContig32Block), 0, s, tab, n, q,
                               kContig32Block);
            n = 0;
            blocks = 0;
            return hipGetLastError();
        };
        for (int i = 0; i < k; ++i) {
            const uint64_t count = counts[i];
            if (!count)
                continue;
            if (((reinterpret_cast<uintptr_t>(ins[i]) | reinterpret_cast<uintptr_t>(ios[i])) & 15) !=
                0) {
                hipError_t e = launch_contig<C>(ins[i], ios[i], count, p, cfg, s);
                if (e != hipSuccess)
                    return e;
                continue;
            }
            const uint64_t nb = (count + tile - 1) / tile;
            if (nb > max_blocks(kContig32Block)) {   // more tiles than one grid holds: a call of its own
                hipError_t e = launch_contig<C>(ins[i], ios[i], count, p, cfg, s);
                if (e != hipSuccess)
                    return e;
                continue;
            }
            if (blocks + nb > max_blocks(kContig32Block)) {
                hipError_t e = flush();
                if (e != hipSuccess)
                    return e;
            }
            tab.blk0[n] = (uint32_t) blocks;
            tab.s[n] = BatchSeg{ins[i], ios[i], count, 0, 0, 1, {0, 0, 0, 0, 0}};
            blocks += nb;
            ++n;
        }
        return flush();
    } else {
        constexpr uint64_t E = 16 / sizeof(T);
        const uint64_t tile = (uint64_t) cfg.block * MPIX_REDOP_UNROLL;
        BatchTab tab;
        int n = 0;
        uint64_t blocks = 0;
        auto flush = [&]() -> hipError_t {
            if (!n)
                return hipSuccess;
            Params q = p;
            set_store_policy(q, cfg, (unsigned) blocks);
            hipLaunchKernelGGL((k_batch<C, MPIX_REDOP_UNROLL, MPIX_REDOP_NT_LOAD, MPIX_REDOP_NT_STORE>),
                               dim3((unsigned) blocks), dim3(cfg.block), 0, s, tab, n, q,
                               (uint32_t) blocks, (uint32_t) cfg.block);
            n = 0;
            blocks = 0;
            return hipGetLastError();
        };
        for (int i = 0; i < k; ++i) {
            const uint64_t count = counts[i];
            if (!count)
                continue;
            const uintptr_t ai = reinterpret_cast<uintptr_t>(ins[i]);
            const uintptr_t ao = reinterpret_cast<uintptr_t>(ios[i]);
            if ((ai % sizeof(T)) || (ao % sizeof(T))) {
                hipError_t e = launch_contig<C>(ins[i], ios[i], count, p, cfg, s);
                if (e != hipSuccess)
                    return e;
                continue;
            }
            uint64_t head = ((16 - (ao & 15)) & 15) / sizeof(T);
            if (head > count)
                head = count;
            const uint64_t npk = (count - head) / E;
            const uint64_t ntail = count - head - npk * E;
            uint64_t nb = (npk + tile - 1) / tile;
            if (nb == 0)
                nb = 1;         // a segment of head / tail elements only
            if (nb > max_blocks(cfg.block)) {    // more tiles than one grid holds: launch_contig
                hipError_t e = launch_contig<C>(ins[i], ios[i], count, p, cfg, s);   // loops
                if (e != hipSuccess)
                    return e;
                continue;
            }
            if (blocks + nb > max_blocks(cfg.block)) {
                hipError_t e = flush();
                if (e != hipSuccess)
                    return e;
            }
            tab.blk0[n] = (uint32_t) blocks;
            tab.s[n] = BatchSeg{ins[i], ios[i], npk, (uint8_t) head, (uint8_t) ntail,
                                (uint8_t) ((ai & 15) == (ao & 15)), {0, 0, 0, 0, 0}};
            blocks += nb;
            ++n;
        }
        return flush();
    }
}

template <class C> constexpr Entry entry()
{
    return Entry{&launch_contig<C>, &launch_vector<C>, &launch_multi<C>, &launch_iov<C>,
                 &launch_tree<C>, &launch_batch<C>};
}

}  // namespace mpix
