// redop_soft.h -- x87 extended and IEEE binary128 SUM / PROD in integer
// arithmetic on gfx950 (no hardware for either format).
//
// MPI_LONG_DOUBLE on x86-64 is the x87 80-bit format in a 16-byte slot
// (MPIR_ALT_FLOAT128, mpir_datatype.h:82); MPI_REAL16 is binary128
// (MPIR_FLOAT128).  op_fns.c's `a[i] = a[i] + b[i]` / `a[i] * b[i]` on them
// is, as gcc builds MPICH on x86-64: fldt a; fldt b; faddp / fmulp; fstpt a
// (x87, precision control extended, round to nearest even) and
// __addtf3(a, b) / __multf3(a, b) (libgcc soft-fp, round to nearest even).
// Restated here bit for bit, checked against the oracle's gcc-built loops
// (tests/test_soft_fp_gpu.py):
//   * x87: an operand in an unsupported encoding (exponent != 0 with the
//     explicit integer bit J clear: unnormals, pseudo-infinities, pseudo-
//     NaNs) makes the result the "real indefinite" QNaN (sign 1, exponent
//     0x7fff, significand 0xC000...), NaN operands or not; of two NaNs the
//     one with the larger significand (a QNaN's is always the larger), on a
//     tie the positive one; a NaN result is quieted (bit 62); inf - inf and
//     0 * inf are the indefinite too.  Pseudo-denormals (exponent 0, J set)
//     are operands of exponent 1; results are normalised, denormal results
//     denormalised then rounded; `fstpt` stores 10 bytes, so the slot's
//     padding keeps inout's.
//   * binary128 (libgcc/config/i386/sfp-machine.h _FP_CHOOSENAN): of two
//     NaNs the larger fraction, on a tie the first operand (inout) for + and
//     *, the second for -; quieted; invalid results are the default NaN
//     (sign 1, quiet bit only).
// Both: exact result, then one rounding (RNE, gradual underflow).  Sums and
// products of two normal operands take a fast path that rounds at a fixed cut
// (the general path's shifts made constant; a near-cancelling sum is exact and
// only normalised); anything else -- specials, denormal or overflowing
// results, exact cancellation -- takes the general path.
#pragma once

#include <stdint.h>


#include "redop_dispatch.h"

// MPIX_SOFT_HOST: the same functions as plain host C++, for the CPU test that
// checks them against the oracle on millions of pairs without a GPU
// (tests/c/soft_check.cpp, tests/test_soft_fp.py)
#ifdef MPIX_SOFT_HOST
#define MPIX_SDEV inline
#else
#include <hip/hip_runtime.h>
#define MPIX_SDEV __device__ __forceinline__
#endif

namespace mpix {

typedef unsigned __int128 u128;

// x87 extended in a 16-byte slot
struct alignas(16) X87 {
    uint64_t m;     // significand, J = bit 63
    uint64_t se;    // bits 0-14 exponent, bit 15 sign, bits 16-63 padding
};

// IEEE binary128
struct alignas(16) Quad {
    uint64_t lo, hi;    // hi: sign, 15-bit exponent, top 48 fraction bits
};

// result classes (x87_class / quad_class); the compare-and-select combiners
// of redop_ops.h use kCmp* instead
enum SoftClass { kX87Bad = 0, kX87Nan, kX87Inf, kX87Zero, kX87Fin };

MPIX_SDEV int clz128(u128 x)
{
    const uint64_t hi = (uint64_t) (x >> 64), lo = (uint64_t) x;
    return hi ? __builtin_clzll(hi) : 64 + (lo ? __builtin_clzll(lo) : 64);
}

// Round the exact value S * 2^(E0 - 16383 - 126) (S != 0) to a significand of
// `bits` bits (64 for x87 with its explicit J bit, 113 for binary128 with the
// implicit one), round to nearest even, gradual underflow.  Out: *m the
// significand (leading bit at bits - 1 for a normal), *e the biased exponent
// (0: denormal or zero; 0x7fff: overflow to infinity, *m = the leading bit).
MPIX_SDEV void round_exact(u128 S, int64_t E0, int bits, u128 *m, int64_t *e)
{
    const int p = 127 - clz128(S);      // leading one of S
    int64_t E = E0 + p - 126;
    int64_t sh = p - (bits - 1);        // bits of S below the significand
    if (E < 1) {                        // denormal: the scale of exponent 1
        sh += 1 - E;
        E = 0;
    }
    u128 r;
    if (sh <= 0) {
        r = S << (int) (-sh);
    } else if (sh > 128) {
        r = 0;                          // below half of the smallest denormal
    } else if (sh == 128) {
        const u128 half = (u128) 1 << 127;
        r = S > half ? 1 : 0;           // a tie rounds to the even 0
    } else {
        r = S >> (int) sh;
        const u128 rest = S & (((u128) 1 << (int) sh) - 1);
        const u128 half = (u128) 1 << (int) (sh - 1);
        if (rest > half || (rest == half && (r & 1)))
            r += 1;
    }
    const u128 lead = (u128) 1 << (bits - 1);
    if (r >> bits) {                    // rounding carried out of the significand
        r >>= 1;
        E += 1;
    }
    if (E == 0 && (r & lead))           // a denormal rounded up into the normals
        E = 1;
    if (E >= 0x7fff) {
        r = lead;
        E = 0x7fff;
    }
    *m = r;
    *e = E;
}

// ---------------------------------------------------------------- x87

MPIX_SDEV int x87_class(uint64_t m, uint32_t e)
{
    const bool j = (m >> 63) != 0;
    if (e != 0 && !j)
        return kX87Bad;                 // unnormal, pseudo-infinity, pseudo-NaN
    if (e == 0x7fff)
        return (m << 1) ? kX87Nan : kX87Inf;
    if (e == 0 && m == 0)
        return kX87Zero;
    return kX87Fin;                     // normal, denormal, pseudo-denormal
}

// the 10 value bytes of a result, the slot's padding taken from `pad`
MPIX_SDEV X87 x87_make(const X87 &pad, bool s, uint32_t e, uint64_t m)
{
    X87 r;
    r.m = m;
    r.se = (pad.se & ~(uint64_t) 0xffff) | ((uint64_t) s << 15) | e;
    return r;
}

MPIX_SDEV X87 x87_indefinite(const X87 &pad)
{
    return x87_make(pad, true, 0x7fff, 0xC000000000000000ull);
}

// NaN result of a, b (at least one a NaN, neither unsupported)
MPIX_SDEV X87 x87_nan(const X87 &a, bool a_nan, const X87 &b, bool b_nan)
{
    const bool sa = (a.se >> 15) & 1, sb = (b.se >> 15) & 1;
    bool pick_a;
    if (a_nan && b_nan)
        pick_a = a.m != b.m ? a.m > b.m : !sa;
    else
        pick_a = a_nan;
    const X87 &n = pick_a ? a : b;
    return x87_make(a, pick_a ? sa : sb, 0x7fff, n.m | (1ull << 62));
}

MPIX_SDEV X87 x87_from_round(const X87 &pad, bool s, u128 S, int64_t E0)
{
    u128 m;
    int64_t e;
    round_exact(S, E0, 64, &m, &e);
    return x87_make(pad, s, (uint32_t) e, (uint64_t) m);
}

// ---------------------------------------------------------- 32-bit limbs
// The normal-operand fast paths work on 32-bit limbs (w[0] least
// significant): every step is a handful of 32-bit VALU operations (funnel
// shifts, carries, selects) instead of the 128-bit emulation a u128 shift by
// a variable amount or a u128 compare compiles to.  The complex products run
// four products and two sums per unit and are VALU-bound on gfx950 (round 5:
// 3.8 / 4.5 TB/s), so these instruction counts are their rate.

// ({hi, lo} >> (s & 31)) & 0xffffffff (v_alignbit_b32)
MPIX_SDEV uint32_t funnel_r(uint32_t hi, uint32_t lo, uint32_t s)
{
#ifdef MPIX_SOFT_HOST
    return (uint32_t) ((((uint64_t) hi << 32) | lo) >> (s & 31));
#else
    return __builtin_amdgcn_alignbit(hi, lo, s);
#endif
}

// ({hi, lo} << s) >> 32 for s in 0..31
MPIX_SDEV uint32_t funnel_l(uint32_t hi, uint32_t lo, uint32_t s)
{
    return (uint32_t) (((((uint64_t) hi << 32) | lo) << s) >> 32);
}

MPIX_SDEV uint32_t clz32(uint32_t x) { return x ? (uint32_t) __builtin_clz(x) : 32u; }

// x != 0 as 0 / 1: one full-rate v_min_u32 (a compare and a select otherwise)
MPIX_SDEV uint32_t nz32(uint32_t x) { return x < 1u ? x : 1u; }

// a + b + cin (cin 0 or 1), the carry out in *cout: one v_addc_co_u32 (the
// 64-bit accumulate-and-shift form compiles to an add, a select of the carry
// and a 64-bit add per limb)
MPIX_SDEV uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t *cout)
{
#ifdef MPIX_SOFT_HOST
    const uint64_t t = (uint64_t) a + b + cin;
    *cout = (uint32_t) (t >> 32);
    return (uint32_t) t;
#else
    unsigned c;
    const uint32_t r = __builtin_addc(a, b, cin, &c);
    *cout = c;
    return r;
#endif
}

// q += inc (inc 0 or 1) over four limbs; the carry out of q[3] is dropped
MPIX_SDEV void inc128(uint32_t q[4], uint32_t inc)
{
    uint32_t c;
    q[0] = addc32(q[0], inc, 0u, &c);
    q[1] = addc32(q[1], 0u, c, &c);
    q[2] = addc32(q[2], 0u, c, &c);
    q[3] = addc32(q[3], 0u, c, &c);
}

// z + x * y (v_mad_u64_u32): as a chain the compiler keeps in order -- left
// to itself it sums a column's products first and adds the carry with one more
// 64-bit add per column
MPIX_SDEV uint64_t mad64(uint32_t x, uint32_t y, uint64_t z)
{
#ifdef MPIX_SOFT_HOST
    return z + (uint64_t) x * y;
#else
    // the accumulator in place (dst = src2, as the compiler's own code has
    // it), early-clobber against the 32-bit sources; the carry-out pair is
    // never set (no overflow)
    uint64_t r = z, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+&v"(r), "=s"(carry) : "v"(x), "v"(y));
    return r;
#endif
}

// x * y as the first link of such a chain (the zero addend inline, not a
// register pair set to zero)
MPIX_SDEV uint64_t mul64(uint32_t x, uint32_t y)
{
#ifdef MPIX_SOFT_HOST
    return (uint64_t) x * y;
#else
    uint64_t r, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=&v"(r), "=s"(carry) : "v"(x), "v"(y));
    return r;
#endif
}

// v >>= d (d in 0..127); returns the OR of the bits shifted out
MPIX_SDEV uint32_t shr128_lost(uint32_t v[4], uint32_t d)
{
    const bool b64 = (d & 64) != 0, b32 = (d & 32) != 0;
    uint32_t lost = b64 ? (v[0] | v[1]) : 0u;
    const uint32_t t0 = b64 ? v[2] : v[0], t1 = b64 ? v[3] : v[1];
    const uint32_t t2 = b64 ? 0u : v[2], t3 = b64 ? 0u : v[3];
    lost |= b32 ? t0 : 0u;
    const uint32_t u0 = b32 ? t1 : t0, u1 = b32 ? t2 : t1, u2 = b32 ? t3 : t2, u3 = b32 ? 0u : t3;
    const uint32_t r = d & 31;
    lost |= u0 & ((1u << r) - 1u);
    v[0] = funnel_r(u1, u0, r);
    v[1] = funnel_r(u2, u1, r);
    v[2] = funnel_r(u3, u2, r);
    v[3] = u3 >> r;
    return lost;
}

// The sum of two normal operands, A (the larger magnitude) and B, both with
// their leading bit at 126 of a 128-bit limb vector, B's exponent d below A's
// (d clamped to 127: B then only leaves its sticky bit, as it did before it
// moved out of range).  B is aligned by d with the bits shifted out folded
// into its lowest bit (a sticky bit below every rounding position), added or
// (sub) subtracted, and the exact sum S rounded to BITS bits (RNE) at its
// leading bit: the cut sits lz bits lower than for a leading bit at 127, so
// the significand is S shifted right by 128 - BITS - lz, a funnel shift per
// limb -- no normalising shift.  A sum whose leading bit is not in the top
// limb (lz > 31: opposite signs cancelling 30 bits or more; for binary128
// lz > 15, where the significand would need a left shift) goes to the
// general path, as do a zero sum and a result that is not normal.  *q = the
// significand (limbs, leading bit at BITS - 1), *E its biased exponent for
// A's biased exponent xa.  round_exact's normal-result case.
template <int BITS>
MPIX_SDEV bool add_normal_limbs(const uint32_t A[4], uint32_t B[4], uint32_t d, bool sub, int32_t xa,
                                uint32_t q[4], int32_t *E)
{
    // exponents less than 32 apart (nearly every pair of products in a
    // complex product) need no limb selects: a branch a wave takes only when
    // one of its lanes is further apart
    uint32_t lost;
    if (d < 32u) {
        lost = B[0] & ((1u << d) - 1u);
        B[0] = funnel_r(B[1], B[0], d);
        B[1] = funnel_r(B[2], B[1], d);
        B[2] = funnel_r(B[3], B[2], d);
        B[3] >>= d;
    } else {
        lost = shr128_lost(B, d);
    }
    B[0] |= nz32(lost);
    // S = A + B, or A - B = A + ~B + 1 (A >= B, so no borrow out)
    const uint32_t m = sub ? 0xffffffffu : 0u;
    uint32_t S[4];
    uint32_t c = sub ? 1u : 0u;
    for (int i = 0; i < 4; ++i)
        S[i] = addc32(A[i], B[i] ^ m, c, &c);
    const uint32_t lz = clz32(S[3]);
    uint32_t rnd, sticky;
    if constexpr (BITS == 64) {
        // x87: q = S >> (64 - lz), lz in 0..31
        if (lz > 31)
            return false;
        const uint32_t r1 = funnel_l(S[1], S[0], lz);
        q[0] = funnel_l(S[2], S[1], lz);
        q[1] = funnel_l(S[3], S[2], lz);
        q[2] = q[3] = 0;
        rnd = r1 >> 31;
        sticky = (r1 & 0x7fffffffu) | (S[0] << lz);
    } else {
        static_assert(BITS == 113, "binary128");
        // q = S >> (15 - lz), lz in 0..15 (the cut in the lowest limb)
        if (lz > 15)
            return false;
        const uint32_t cut = 15u - lz;
        q[0] = funnel_r(S[1], S[0], cut);
        q[1] = funnel_r(S[2], S[1], cut);
        q[2] = funnel_r(S[3], S[2], cut);
        q[3] = S[3] >> cut;
        // the bits below the cut, left-aligned (none when cut = 0)
        const uint32_t low = funnel_r(S[0], 0u, cut);
        rnd = low >> 31;
        sticky = low << 1;
    }
    int32_t e = xa + 1 - (int32_t) lz;
    const uint32_t inc = rnd & (nz32(sticky) | (q[0] & 1u));
    inc128(q, inc);
    // carried out of the significand: it was all ones, it is now 2^BITS (the
    // limbs below the top one already zero)
    if constexpr (BITS == 64) {
        const uint32_t ovf = q[2] & 1u;
        q[1] |= ovf << 31;
        q[2] = 0;
        e += (int32_t) ovf;
    } else {
        const uint32_t ovf = q[3] >> (BITS - 96);
        q[3] >>= ovf;
        e += (int32_t) ovf;
    }
    *E = e;
    return e >= 1 && e <= 0x7ffe;
}

// a + b (sub: a - b), as fldt a; fldt b; faddp (fsubp); the result keeps a's
// padding.  FAST: both operands normal -> add_normal_limbs, the rest the general path.
// a + b (sub: a - b) of two normal operands whose sum is normal: *r and true;
// false for anything else (x87_add's general path decides)
MPIX_SDEV bool x87_add_fast(const X87 &a, const X87 &b, bool sub, X87 *r)
{
    const uint32_t ea = (uint32_t) a.se & 0x7fff, eb = (uint32_t) b.se & 0x7fff;
    if (!(ea - 1u < 0x7ffeu && eb - 1u < 0x7ffeu && (a.m >> 63) && (b.m >> 63)))
        return false;
    {
        // both normal: order by magnitude, align, add_normal_limbs
        const bool swap = ea < eb || (ea == eb && a.m < b.m);
        const bool sa0 = (a.se >> 15) & 1, sb0 = ((b.se >> 15) & 1) ^ (sub ? 1 : 0);
        const bool sa = swap ? sb0 : sa0, sb = swap ? sa0 : sb0;
        const uint64_t ma = swap ? b.m : a.m, mb = swap ? a.m : b.m;
        const uint32_t xa = swap ? eb : ea, d = swap ? eb - ea : ea - eb;
        // m << 63: the leading bit J at 126
        const uint32_t al = (uint32_t) ma, ah = (uint32_t) (ma >> 32);
        const uint32_t bl = (uint32_t) mb, bh = (uint32_t) (mb >> 32);
        const uint32_t A[4] = {0u, al << 31, funnel_r(ah, al, 1), ah >> 1};
        uint32_t B[4] = {0u, bl << 31, funnel_r(bh, bl, 1), bh >> 1};
        uint32_t q[4];
        int32_t e;
        if (!add_normal_limbs<64>(A, B, d < 127u ? d : 127u, sa != sb, (int32_t) xa, q, &e))
            return false;
        *r = x87_make(a, sa, (uint32_t) e, ((uint64_t) q[1] << 32) | q[0]);
        return true;
    }
}

template <bool FAST = true>
MPIX_SDEV X87 x87_add(const X87 &a, const X87 &b, bool sub)
{
    const uint32_t ea = (uint32_t) a.se & 0x7fff, eb = (uint32_t) b.se & 0x7fff;
    X87 r;
    if (FAST && x87_add_fast(a, b, sub, &r))
        return r;
    const int ca = x87_class(a.m, ea), cb = x87_class(b.m, eb);
    if (ca == kX87Bad || cb == kX87Bad)
        return x87_indefinite(a);
    if (ca == kX87Nan || cb == kX87Nan)
        return x87_nan(a, ca == kX87Nan, b, cb == kX87Nan);
    bool sa = (a.se >> 15) & 1, sb = ((b.se >> 15) & 1) ^ (sub ? 1 : 0);
    if (ca == kX87Inf || cb == kX87Inf) {
        if (ca == kX87Inf && cb == kX87Inf && sa != sb)
            return x87_indefinite(a);
        return x87_make(a, ca == kX87Inf ? sa : sb, 0x7fff, 1ull << 63);
    }
    if (ca == kX87Zero && cb == kX87Zero)
        return x87_make(a, sa && sb, 0, 0);
    // one zero, the other normal: that operand exactly (a denormal or
    // pseudo-denormal one goes on below, where rounding renormalises it)
    if (cb == kX87Zero && ea != 0)
        return x87_make(a, sa, ea, a.m);
    if (ca == kX87Zero && eb != 0)
        return x87_make(a, sb, eb, b.m);
    uint64_t ma = a.m, mb = b.m;
    int64_t xa = ea ? ea : 1, xb = eb ? eb : 1;
    if (xa < xb || (xa == xb && ma < mb)) {     // |a| >= |b|
        uint64_t t = ma; ma = mb; mb = t;
        int64_t u = xa; xa = xb; xb = u;
        bool v = sa; sa = sb; sb = v;
    }
    const u128 A = (u128) ma << 63;
    const int64_t d = xa - xb;
    u128 B = 0;
    if (d < 128) {
        const u128 full = (u128) mb << 63;
        B = full >> (int) d;
        if (d > 0 && (full & (((u128) 1 << (int) d) - 1)))
            B |= 1;                     // sticky
    } else if (mb) {
        B = 1;
    }
    const u128 S = sa == sb ? A + B : A - B;
    if (S == 0)
        return x87_make(a, false, 0, 0);        // exact cancellation: +0
    return x87_from_round(a, sa, S, xa);
}

// a * b of two normal operands whose product is normal: *r and true; false
// for anything else (x87_mul's general path decides)
MPIX_SDEV bool x87_mul_fast(const X87 &a, const X87 &b, X87 *r)
{
    const uint32_t ea = (uint32_t) a.se & 0x7fff, eb = (uint32_t) b.se & 0x7fff;
    if (!(ea - 1u < 0x7ffeu && eb - 1u < 0x7ffeu && (a.m >> 63) && (b.m >> 63)))
        return false;
    // both normal: the product of the significands is in [2^126, 2^128), so
    // its leading bit sits at 126 + top and the rounding cut at a fixed place
    // (the general path with its shifts constant), in 32-bit limbs w3..w0
    // from four multiply-adds.  A result that would be denormal or overflow
    // takes the general path.
    const uint32_t al = (uint32_t) a.m, ah = (uint32_t) (a.m >> 32);
    const uint32_t bl = (uint32_t) b.m, bh = (uint32_t) (b.m >> 32);
    const uint64_t p0 = mul64(al, bl);
    const uint64_t t1 = mad64(al, bh, p0 >> 32);
    const uint64_t t2 = mad64(ah, bl, (uint32_t) t1);
    const uint64_t t3 = mad64(ah, bh, (t1 >> 32) + (t2 >> 32));
    const uint32_t w0 = (uint32_t) p0, w1 = (uint32_t) t2;
    const uint32_t w2 = (uint32_t) t3, w3 = (uint32_t) (t3 >> 32);
    const uint32_t top = w3 >> 31;
    // the significand: {w3, w2} (top) or {w3, w2, w1} << 1; the bits below
    // the cut left-aligned in `low`, w0 under them
    uint32_t q0 = top ? w2 : funnel_r(w2, w1, 31);
    uint32_t q1 = top ? w3 : funnel_r(w3, w2, 31);
    const uint32_t low = w1 << (1u - top);
    const uint32_t rnd = low >> 31;
    const uint32_t inc = rnd & (nz32((low << 1) | w0) | (q0 & 1u));
    uint32_t c;
    q0 = addc32(q0, inc, 0u, &c);
    q1 = addc32(q1, 0u, c, &c);
    q1 |= c << 31;          // carried out of the significand: 2^64 -> 2^63, E + 1
    // denormal before rounding (E0 < 1: the cut is elsewhere) or overflowing
    const int32_t E0 = (int32_t) (ea + eb + top) - 16383, E = E0 + (int32_t) c;
    if (E0 < 1 || E > 0x7ffe)
        return false;
    *r = x87_make(a, ((a.se ^ b.se) >> 15) & 1, (uint32_t) E, ((uint64_t) q1 << 32) | q0);
    return true;
}

MPIX_SDEV X87 x87_mul(const X87 &a, const X87 &b)
{
    const uint32_t ea = (uint32_t) a.se & 0x7fff, eb = (uint32_t) b.se & 0x7fff;
    X87 r;
    if (x87_mul_fast(a, b, &r))
        return r;
    const int ca = x87_class(a.m, ea), cb = x87_class(b.m, eb);
    if (ca == kX87Bad || cb == kX87Bad)
        return x87_indefinite(a);
    if (ca == kX87Nan || cb == kX87Nan)
        return x87_nan(a, ca == kX87Nan, b, cb == kX87Nan);
    const bool s = ((a.se ^ b.se) >> 15) & 1;
    if (ca == kX87Inf || cb == kX87Inf) {
        if (ca == kX87Zero || cb == kX87Zero)
            return x87_indefinite(a);
        return x87_make(a, s, 0x7fff, 1ull << 63);
    }
    if (ca == kX87Zero || cb == kX87Zero)
        return x87_make(a, s, 0, 0);
    const int64_t xa = ea ? ea : 1, xb = eb ? eb : 1;
    // value = ma * mb * 2^(xa + xb - 2*16383 - 126) = S * 2^(E0 - 16383 - 126)
    return x87_from_round(a, s, (u128) a.m * b.m, xa + xb - 16383);
}

struct X87Sum {
    using unit = X87;
    static MPIX_SDEV X87 apply(X87 a, X87 b, const Params &) { return x87_add(a, b, false); }
};
struct X87Prod {
    using unit = X87;
    static MPIX_SDEV X87 apply(X87 a, X87 b, const Params &) { return x87_mul(a, b); }
};

// ----------------------------------------------------------- binary128
MPIX_SDEV int quad_class(const Quad &q)
{
    const uint32_t e = (uint32_t) (q.hi >> 48) & 0x7fff;
    const uint64_t fh = q.hi & 0xffffffffffffull;
    if (e == 0x7fff)
        return (fh | q.lo) ? kX87Nan : kX87Inf;
    if (e == 0 && !(fh | q.lo))
        return kX87Zero;
    return kX87Fin;
}

MPIX_SDEV Quad quad_make(bool s, uint32_t e, u128 frac)
{
    Quad r;
    r.lo = (uint64_t) frac;
    r.hi = ((uint64_t) s << 63) | ((uint64_t) e << 48) | ((uint64_t) (frac >> 64) & 0xffffffffffffull);
    return r;
}

// _FP_CHOOSENAN (i386): the larger fraction; a tie goes to x for + and *
// (x_on_tie), to y for -; the result quieted
MPIX_SDEV Quad quad_nan(const Quad &x, bool x_nan, const Quad &y, bool y_nan, bool x_on_tie)
{
    const u128 fx = ((u128) (x.hi & 0xffffffffffffull) << 64) | x.lo;
    const u128 fy = ((u128) (y.hi & 0xffffffffffffull) << 64) | y.lo;
    bool pick_x;
    if (x_nan && y_nan)
        pick_x = fx != fy ? fx > fy : x_on_tie;
    else
        pick_x = x_nan;
    const Quad &n = pick_x ? x : y;
    Quad r = n;
    r.hi |= 1ull << 47;
    return r;
}

MPIX_SDEV Quad quad_default_nan() { return quad_make(true, 0x7fff, (u128) 1 << 111); }

MPIX_SDEV void quad_parts(const Quad &q, bool *s, int64_t *x, u128 *m)
{
    const uint32_t e = (uint32_t) (q.hi >> 48) & 0x7fff;
    *s = q.hi >> 63;
    *x = e ? e : 1;
    *m = ((u128) (q.hi & 0xffffffffffffull) << 64) | q.lo;
    if (e)
        *m |= (u128) 1 << 112;
}

MPIX_SDEV Quad quad_from_round(bool s, u128 S, int64_t E0)
{
    u128 m;
    int64_t e;
    round_exact(S, E0, 113, &m, &e);
    return quad_make(s, (uint32_t) e, m & (((u128) 1 << 112) - 1));
}

// x + y (sub: x - y): __addtf3 / __subtf3
// A binary128 value in limbs: the significand q (implicit one at bit 112 of
// the four 32-bit limbs), its biased exponent e and sign s -- a product's
// result before it is packed, or an operand unpacked, for the sums
struct QLimbs {
    uint32_t q[4];
    uint32_t e, s;
};

MPIX_SDEV QLimbs quad_limbs(const Quad &x)
{
    QLimbs r;
    r.q[0] = (uint32_t) x.lo;
    r.q[1] = (uint32_t) (x.lo >> 32);
    r.q[2] = (uint32_t) x.hi;
    r.q[3] = ((uint32_t) (x.hi >> 32) & 0xffffu) | 0x10000u;
    r.e = (uint32_t) (x.hi >> 48) & 0x7fff;
    r.s = (uint32_t) (x.hi >> 63);
    return r;
}

// x + y (sub: x - y) of two normal values in limbs whose sum is normal: *r
// (packed) and true; false for anything else (quad_add's general path)
MPIX_SDEV bool quad_add_limbs(const QLimbs &x, const QLimbs &y, bool sub, Quad *r)
{
    // magnitudes ordered by (exponent, significand): two 64-bit keys each
    const uint64_t kx = ((uint64_t) ((x.e << 17) | x.q[3]) << 32) | x.q[2];
    const uint64_t ky = ((uint64_t) ((y.e << 17) | y.q[3]) << 32) | y.q[2];
    const uint64_t lx = ((uint64_t) x.q[1] << 32) | x.q[0], ly = ((uint64_t) y.q[1] << 32) | y.q[0];
    const bool swap = kx < ky || (kx == ky && lx < ly);
    const uint32_t sy = y.s ^ (sub ? 1u : 0u);
    const uint32_t sa = swap ? sy : x.s, sb = swap ? x.s : sy;
    const QLimbs &big = swap ? y : x, &small = swap ? x : y;
    const uint32_t xa = big.e, d = big.e - small.e;
    // significand << 14: the leading bit at 126
    // (a left funnel by 14 is a right funnel by 18: one v_alignbit_b32 a limb)
    const uint32_t A[4] = {big.q[0] << 14, funnel_r(big.q[1], big.q[0], 18),
                           funnel_r(big.q[2], big.q[1], 18), funnel_r(big.q[3], big.q[2], 18)};
    uint32_t B[4] = {small.q[0] << 14, funnel_r(small.q[1], small.q[0], 18),
                     funnel_r(small.q[2], small.q[1], 18), funnel_r(small.q[3], small.q[2], 18)};
    uint32_t q[4];
    int32_t e;
    if (!add_normal_limbs<113>(A, B, d < 127u ? d : 127u, sa != sb, (int32_t) xa, q, &e))
        return false;
    r->lo = ((uint64_t) q[1] << 32) | q[0];
    r->hi = ((uint64_t) sa << 63) | ((uint64_t) e << 48) | ((uint64_t) (q[3] & 0xffffu) << 32) | q[2];
    return true;
}

// x + y (sub: x - y) of two normal operands whose sum is normal: *r and
// true; false for anything else (quad_add's general path decides)
MPIX_SDEV bool quad_add_fast(const Quad &x, const Quad &y, bool sub, Quad *r)
{
    const uint32_t ex = (uint32_t) (x.hi >> 48) & 0x7fff, ey = (uint32_t) (y.hi >> 48) & 0x7fff;
    if (!(ex - 1u < 0x7ffeu && ey - 1u < 0x7ffeu))
        return false;
    return quad_add_limbs(quad_limbs(x), quad_limbs(y), sub, r);
}

template <bool FAST = true>
MPIX_SDEV Quad quad_add(const Quad &x, const Quad &y, bool sub)
{
    Quad r;
    if (FAST && quad_add_fast(x, y, sub, &r))
        return r;
    const int cx = quad_class(x), cy = quad_class(y);
    if (cx == kX87Nan || cy == kX87Nan)
        return quad_nan(x, cx == kX87Nan, y, cy == kX87Nan, !sub);
    bool sa, sb;
    int64_t xa, xb;
    u128 ma, mb;
    quad_parts(x, &sa, &xa, &ma);
    quad_parts(y, &sb, &xb, &mb);
    sb ^= sub;
    if (cx == kX87Inf || cy == kX87Inf) {
        if (cx == kX87Inf && cy == kX87Inf && sa != sb)
            return quad_default_nan();
        return quad_make(cx == kX87Inf ? sa : sb, 0x7fff, 0);
    }
    if (cx == kX87Zero && cy == kX87Zero)
        return quad_make(sa && sb, 0, 0);
    // one zero: the other operand exactly (soft-fp's NORMAL/ZERO cases copy
    // it; a denormal packs back to the same bits), y with the subtraction's
    // sign -- no alignment or rounding (real values stored as complex meet
    // this in every unit)
    if (cy == kX87Zero)
        return x;
    if (cx == kX87Zero) {
        Quad r = y;
        r.hi = (r.hi & ~(1ull << 63)) | ((uint64_t) sb << 63);
        return r;
    }
    if (xa < xb || (xa == xb && ma < mb)) {
        u128 t = ma; ma = mb; mb = t;
        int64_t u = xa; xa = xb; xb = u;
        bool v = sa; sa = sb; sb = v;
    }
    const u128 A = ma << 14;            // leading bit at 126, 14 guard bits
    const int64_t d = xa - xb;
    u128 B = 0;
    if (d < 128) {
        const u128 full = mb << 14;
        B = full >> (int) d;
        if (d > 0 && (full & (((u128) 1 << (int) d) - 1)))
            B |= 1;
    } else if (mb) {
        B = 1;
    }
    const u128 S = sa == sb ? A + B : A - B;
    if (S == 0)
        return quad_make(false, 0, 0);
    return quad_from_round(sa, S, xa);
}

// x * y of two normal operands whose product is normal, as four 64 x 64-bit
// partial products: *r and true; false for anything else (quad_mul's general
// path decides).  The shorter dependency chains of the two forms: the
// standalone MPI_REAL16 PROD row, bandwidth-bound, runs 6 % faster with it
// than with quad_mul_fast's digits (7.34-7.38 against 6.87-6.94 TB/s,
// profiles/r06_soft_rows_ab3.json)
MPIX_SDEV bool quad_mul_fast_wide(const Quad &x, const Quad &y, Quad *r)
{
    const uint32_t ex = (uint32_t) (x.hi >> 48) & 0x7fff, ey = (uint32_t) (y.hi >> 48) & 0x7fff;
    if (!(ex - 1u < 0x7ffeu && ey - 1u < 0x7ffeu))
        return false;
    // significands in [2^112, 2^113), the product in [2^224, 2^226) with its
    // leading bit at 224 + top, so the cut below the 113-bit result is at a
    // fixed place (the general path's shifts constant)
    const uint64_t a0 = x.lo, a1 = (x.hi & 0xffffffffffffull) | (1ull << 48);
    const uint64_t b0 = y.lo, b1 = (y.hi & 0xffffffffffffull) | (1ull << 48);
    const u128 p00 = (u128) a0 * b0, p01 = (u128) a0 * b1, p10 = (u128) a1 * b0;
    const u128 p11 = (u128) a1 * b1;
    const u128 mid = p01 + p10;     // a1, b1 < 2^49: no carry out
    const u128 lo = p00 + (mid << 64);
    const u128 hi = p11 + (mid >> 64) + (lo < p00 ? 1 : 0);
    const int top = (int) (hi >> 97) & 1;
    const u128 q112 = (hi << 16) | (lo >> 112);         // P >> 112
    const u128 rest = lo & (((u128) 1 << 112) - 1);
    const u128 q0 = top ? q112 >> 1 : q112;
    const bool rnd = top ? (q112 & 1) != 0 : ((rest >> 111) & 1) != 0;
    const bool sticky = top ? rest != 0 : (rest & (((u128) 1 << 111) - 1)) != 0;
    int64_t E = (int64_t) ex + ey - 16383 + top;
    if (E < 1)
        return false;
    u128 q = q0;
    if (rnd && (sticky || (q & 1))) {
        q += 1;
        if (q >> 113) {             // carried out of the significand
            q >>= 1;
            E += 1;
        }
    }
    if (E > 0x7ffe)
        return false;
    *r = quad_make(((x.hi ^ y.hi) >> 63) & 1, (uint32_t) E, q & (((u128) 1 << 112) - 1));
    return true;
}

// A binary128 operand as four 29-bit digits of its significand (the
// implicit one included: a[3] has 26 bits), biased exponent and sign
struct QDigits {
    uint32_t a[4];
    uint32_t e, s;
};

MPIX_SDEV QDigits quad_digits(const Quad &x)
{
    constexpr uint32_t M29 = (1u << 29) - 1u;
    const uint32_t x0 = (uint32_t) x.lo, x1 = (uint32_t) (x.lo >> 32), x2 = (uint32_t) x.hi;
    const uint32_t x3 = ((uint32_t) (x.hi >> 32) & 0xffffu) | 0x10000u;
    QDigits r;
    r.a[0] = x0 & M29;
    r.a[1] = funnel_r(x1, x0, 29) & M29;
    r.a[2] = funnel_r(x2, x1, 26) & M29;
    r.a[3] = funnel_r(x3, x2, 23);
    r.e = (uint32_t) (x.hi >> 48) & 0x7fff;
    r.s = (uint32_t) (x.hi >> 63);
    return r;
}

// The product of two normal operands' digits, rounded (RNE) to 113 bits, in
// limbs: *r and true when it is normal; false otherwise.  The significands
// in [2^112, 2^113), the product in [2^224, 2^226) with its leading bit at
// 224 + top, so the cut is at bit 112 + top.  A digit product is < 2^58, so a
// column of at most four sums in 64 bits with no carry between the 16
// multiply-adds; each column's chain starts from the previous column's
// carry, giving the product's digits d0..d7; the significand is four funnel
// shifts of the digits above 2^87 (V), those below only feed the sticky bit.
MPIX_SDEV bool quad_mul_digits(const QDigits &x, const QDigits &y, QLimbs *r)
{
    constexpr uint32_t M29 = (1u << 29) - 1u;
    // column c, with the carry of column c - 1 as the first addend of its
    // multiply-add chain: < 4 x 2^58 + 2^35 < 2^61
    uint32_t d[8];
    uint64_t t = 0;
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        t >>= 29;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (c - i >= 0 && c - i < 4)
                t = c == 0 ? mul64(x.a[i], y.a[c - i]) : mad64(x.a[i], y.a[c - i], t);
        d[c] = (uint32_t) t & M29;
    }
    d[7] = (uint32_t) (t >> 29);                // < 2^23
    // V = digits 3..7 as 32-bit words (bits 87.. of the product)
    const uint32_t v[5] = {d[3] | (d[4] << 29), (d[4] >> 3) | (d[5] << 26),
                           (d[5] >> 6) | (d[6] << 23), (d[6] >> 9) | (d[7] << 20), d[7] >> 12};
    const uint32_t top = d[7] >> 22;            // leading bit 225 (1) or 224 (0)
    const uint32_t c = 25u + top;               // the cut, bit 112 + top of the product
    uint32_t *q = r->q;
    q[0] = funnel_r(v[1], v[0], c);
    q[1] = funnel_r(v[2], v[1], c);
    q[2] = funnel_r(v[3], v[2], c);
    q[3] = funnel_r(v[4], v[3], c);
    const uint32_t low = v[0] << (32u - c);     // V's bits below the cut, left-aligned
    const uint32_t rnd = low >> 31;
    const uint32_t sticky = (low << 1) | d[2] | d[1] | d[0];
    inc128(q, rnd & (nz32(sticky) | (q[0] & 1u)));
    // carried out of the significand: 2^113 (q[0..2] are 0)
    const uint32_t ovf = q[3] >> 17;
    q[3] >>= ovf;
    const int32_t E = (int32_t) (x.e + y.e + top + ovf) - 16383;
    r->e = (uint32_t) E;
    r->s = x.s ^ y.s;
    return E >= 1 && E <= 0x7ffe;
}

// x * y of two normal operands whose product is normal: *r and true; false
// for anything else.  The same product as quad_mul_fast_wide in fewer
// instructions (quad_mul_digits)
MPIX_SDEV bool quad_mul_fast(const Quad &x, const Quad &y, Quad *r)
{
    const uint32_t ex = (uint32_t) (x.hi >> 48) & 0x7fff, ey = (uint32_t) (y.hi >> 48) & 0x7fff;
    if (!(ex - 1u < 0x7ffeu && ey - 1u < 0x7ffeu))
        return false;
    QLimbs p;
    if (!quad_mul_digits(quad_digits(x), quad_digits(y), &p))
        return false;
    r->lo = ((uint64_t) p.q[1] << 32) | p.q[0];
    r->hi = ((uint64_t) p.s << 63) | ((uint64_t) p.e << 48) | ((uint64_t) (p.q[3] & 0xffffu) << 32) |
            p.q[2];
    return true;
}

// x * y: __multf3 (the 226-bit product folded to 128 bits plus a sticky bit)
MPIX_SDEV Quad quad_mul(const Quad &x, const Quad &y)
{
    Quad r;
    if (quad_mul_fast_wide(x, y, &r))
        return r;
    const int cx = quad_class(x), cy = quad_class(y);
    if (cx == kX87Nan || cy == kX87Nan)
        return quad_nan(x, cx == kX87Nan, y, cy == kX87Nan, true);
    bool sa, sb;
    int64_t xa, xb;
    u128 ma, mb;
    quad_parts(x, &sa, &xa, &ma);
    quad_parts(y, &sb, &xb, &mb);
    const bool s = sa ^ sb;
    if (cx == kX87Inf || cy == kX87Inf) {
        if (cx == kX87Zero || cy == kX87Zero)
            return quad_default_nan();
        return quad_make(s, 0x7fff, 0);
    }
    if (cx == kX87Zero || cy == kX87Zero)
        return quad_make(s, 0, 0);
    // 256-bit product of two 113-bit significands, limbs of 64 bits
    const uint64_t a0 = (uint64_t) ma, a1 = (uint64_t) (ma >> 64);
    const uint64_t b0 = (uint64_t) mb, b1 = (uint64_t) (mb >> 64);
    const u128 p00 = (u128) a0 * b0, p01 = (u128) a0 * b1, p10 = (u128) a1 * b0;
    const u128 p11 = (u128) a1 * b1;
    const u128 mid = p01 + p10;         // a1, b1 < 2^49: no carry out
    u128 lo = p00 + (mid << 64);
    u128 hi = p11 + (mid >> 64) + (lo < p00 ? 1 : 0);
    // normalise: the leading one to bit 254 of (hi, lo), then fold
    const int lead = hi ? 255 - clz128(hi) : 127 - clz128(lo);
    const int k = 254 - lead;           // left shift, >= 0 (a product < 2^226)
    if (k >= 128) {
        hi = lo << (k - 128);
        lo = 0;
    } else if (k > 0) {
        hi = (hi << k) | (lo >> (128 - k));
        lo <<= k;
    }
    const u128 S = hi | (lo ? 1 : 0);
    // value = product * 2^(xa + xb - 2*16383 - 224), product = S * 2^(lead - 126)
    return quad_from_round(s, S, lead + xa + xb - 16383 - 224);
}

struct QuadSum {
    using unit = Quad;
    static MPIX_SDEV Quad apply(Quad a, Quad b, const Params &) { return quad_add(a, b, false); }
};
struct QuadProd {
    using unit = Quad;
    static MPIX_SDEV Quad apply(Quad a, Quad b, const Params &) { return quad_mul(a, b); }
};

// ------------------------------------------------------------ complex
// MPI_COMPLEX32 (MPIR_COMPLEX128): Fortran struct complex of binary128 parts,
// MPIR_OP_TYPE_GROUP(COMPLEX) (op_fns.c:26-42 component sums; :74-85
// re = c.re*b.re - c.im*b.im, im = c.im*b.re + c.re*b.im, each op soft-fp
// rounded).  MPI_C_LONG_DOUBLE_COMPLEX (MPIR_ALT_COMPLEX128): component
// sums of x87 parts, and the C99 product below.  32-byte units.
struct alignas(16) QuadC {
    Quad re, im;
};
struct QuadCSum {
    using unit = QuadC;
    static MPIX_SDEV QuadC apply(QuadC a, QuadC b, const Params &)
    {
        QuadC r;
        r.re = quad_add(a.re, b.re, false);
        r.im = quad_add(a.im, b.im, false);
        return r;
    }
};
// The complex products are split combiners (is_split, redop_kernels.h): the
// contiguous kernel runs apply_fast -- all six operations' normal-operand
// fast paths, one flag for the lot (the result unspecified when any declines:
// the kernel then leaves the unit as it was) -- and a second launch combines those units with apply, each operation's
// fast path or general path.  The general paths' registers stay out of the
// streaming kernel.
struct QuadCProd {
    using unit = QuadC;
    static constexpr bool kSplit = true;
    static MPIX_SDEV QuadC apply(QuadC c, QuadC b, const Params &)
    {
        QuadC r;
        r.re = quad_add(quad_mul(c.re, b.re), quad_mul(c.im, b.im), true);
        r.im = quad_add(quad_mul(c.im, b.re), quad_mul(c.re, b.im), false);
        return r;
    }
    static MPIX_SDEV QuadC apply_fast(QuadC c, QuadC b, const Params &, bool &ok)
    {
        // each operand's digits once (every one feeds two products), the
        // products kept in limbs for the sums (no pack / unpack between)
        const QDigits cr = quad_digits(c.re), ci = quad_digits(c.im);
        const QDigits br = quad_digits(b.re), bi = quad_digits(b.im);
        ok = cr.e - 1u < 0x7ffeu && ci.e - 1u < 0x7ffeu && br.e - 1u < 0x7ffeu &&
             bi.e - 1u < 0x7ffeu;
        QuadC r;
        QLimbs p0, p1, p2, p3;
        ok &= quad_mul_digits(cr, br, &p0);
        ok &= quad_mul_digits(ci, bi, &p1);
        ok &= quad_add_limbs(p0, p1, true, &r.re);
        ok &= quad_mul_digits(ci, br, &p2);
        ok &= quad_mul_digits(cr, bi, &p3);
        ok &= quad_add_limbs(p2, p3, false, &r.im);
        return r;
    }
};
struct alignas(16) X87C {
    X87 re, im;
};

// C `long double _Complex` product = libgcc's __mulxc3(a, b, c, d) (x = a+ib
// inout, y = c+id in): four x87 products, x = ac - bd, y = ad + bc, and when
// both come out NaN the C99 Annex G recovery of infinities (libgcc2.c), every
// operation an x87 one.  isnan is an unordered self-compare (true for NaNs
// and the unsupported encodings), isinf true for the infinity encoding only,
// copysign a sign-bit copy.
MPIX_SDEV bool x87_isnan(const X87 &v)
{
    const int c = x87_class(v.m, (uint32_t) v.se & 0x7fff);
    return c == kX87Nan || c == kX87Bad;
}
MPIX_SDEV bool x87_isinf(const X87 &v) { return x87_class(v.m, (uint32_t) v.se & 0x7fff) == kX87Inf; }
MPIX_SDEV X87 x87_signed(bool one, const X87 &sgn)      // copysign(one ? 1 : 0, sgn)
{
    X87 r;
    r.m = one ? 1ull << 63 : 0;
    r.se = (sgn.se & 0x8000) | (one ? 0x3fff : 0);
    return r;
}

struct X87CProd {
    using unit = X87C;
    static constexpr bool kSplit = true;
    // the six fast paths (as QuadCProd): finite results, so the Annex G
    // recovery of apply can never be needed where they all succeed
    static MPIX_SDEV X87C apply_fast(X87C x, X87C y, const Params &, bool &ok)
    {
        X87 ac, bd, ad, bc, re, im;
        ok = x87_mul_fast(x.re, y.re, &ac);
        ok &= x87_mul_fast(x.im, y.im, &bd);
        ok &= x87_mul_fast(x.re, y.im, &ad);
        ok &= x87_mul_fast(x.im, y.re, &bc);
        ok &= x87_add_fast(ac, bd, true, &re);
        ok &= x87_add_fast(ad, bc, false, &im);
        X87C r;     // stored with fstpt: each part keeps inout's padding
        r.re = x87_make(x.re, (re.se >> 15) & 1, (uint32_t) re.se & 0x7fff, re.m);
        r.im = x87_make(x.im, (im.se >> 15) & 1, (uint32_t) im.se & 0x7fff, im.m);
        return r;
    }
    static MPIX_SDEV X87C apply(X87C x, X87C y, const Params &)
    {
        X87 a = x.re, b = x.im, c = y.re, d = y.im;
        const X87 ac = x87_mul(a, c), bd = x87_mul(b, d), ad = x87_mul(a, d), bc = x87_mul(b, c);
        X87 re = x87_add(ac, bd, true), im = x87_add(ad, bc, false);
        if (x87_isnan(re) && x87_isnan(im)) {
            bool recalc = false;
            if (x87_isinf(a) || x87_isinf(b)) {
                a = x87_signed(x87_isinf(a), a);
                b = x87_signed(x87_isinf(b), b);
                if (x87_isnan(c)) c = x87_signed(false, c);
                if (x87_isnan(d)) d = x87_signed(false, d);
                recalc = true;
            }
            if (x87_isinf(c) || x87_isinf(d)) {
                c = x87_signed(x87_isinf(c), c);
                d = x87_signed(x87_isinf(d), d);
                if (x87_isnan(a)) a = x87_signed(false, a);
                if (x87_isnan(b)) b = x87_signed(false, b);
                recalc = true;
            }
            if (!recalc && (x87_isinf(ac) || x87_isinf(bd) || x87_isinf(ad) || x87_isinf(bc))) {
                if (x87_isnan(a)) a = x87_signed(false, a);
                if (x87_isnan(b)) b = x87_signed(false, b);
                if (x87_isnan(c)) c = x87_signed(false, c);
                if (x87_isnan(d)) d = x87_signed(false, d);
                recalc = true;
            }
            if (recalc) {
                X87 inf;
                inf.m = 1ull << 63;
                inf.se = 0x7fff;
                re = x87_mul(inf, x87_add(x87_mul(a, c), x87_mul(b, d), true));
                im = x87_mul(inf, x87_add(x87_mul(a, d), x87_mul(b, c), false));
            }
        }
        X87C r;     // stored with fstpt: each part keeps inout's padding
        r.re = x87_make(x.re, (re.se >> 15) & 1, (uint32_t) re.se & 0x7fff, re.m);
        r.im = x87_make(x.im, (im.se >> 15) & 1, (uint32_t) im.se & 0x7fff, im.m);
        return r;
    }
};
struct X87CSum {
    using unit = X87C;
    static MPIX_SDEV X87C apply(X87C a, X87C b, const Params &)
    {
        X87C r;
        r.re = x87_add(a.re, b.re, false);
        r.im = x87_add(a.im, b.im, false);
        return r;
    }
};

#undef MPIX_SDEV

}  // namespace mpix
