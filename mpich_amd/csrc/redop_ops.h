// redop_ops.h -- CDNA4 (gfx950) element combiners for the predefined MPI_Ops.
//
// One combiner per (op, element type).  Each has
//     using unit = <storage of one element, 1..16 bytes, or 32 for the
//                   long double / binary128 pairs (element-wise kernels)>;
//     static __device__ unit apply(unit a, unit b, const Params &p);
// computing the new inout element from a = inoutvec[i], b = invec[i], which is
// MPICH's operand order (src/include/mpir_op_util.h:46-53).  The semantics
// restate src/mpi/coll/op/op_fns.c; see DESIGN.md §Semantics for the full
// table and the oracle/ restatement they are checked against.
//
// Compile with -ffp-contract=off and no fast-math: every floating-point result
// must be the single IEEE-rounded operation the C loop performs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "redop_dispatch.h"
#include "redop_soft.h"     // X87 / Quad units and their SUM / PROD

namespace mpix {

#define MPIX_DEV __device__ __forceinline__

// ---------------------------------------------------------------- integers
// SUM/PROD are computed in an unsigned type at least int-wide and cast back:
// the reference's "(c_type_) (a OP b)" on promoted operands, i.e. wrap modulo
// 2^bits, without the signed-overflow UB.
template <typename T> struct Wide { using type = uint32_t; };
template <> struct Wide<int64_t> { using type = uint64_t; };
template <> struct Wide<uint64_t> { using type = uint64_t; };
template <> struct Wide<__int128> { using type = unsigned __int128; };
template <> struct Wide<unsigned __int128> { using type = unsigned __int128; };

// 1-byte MAX / MIN four per dword (combine16 uses apply4 for 1-byte
// combiners): a byte in the high half of a 16-bit lane whose low half is zero
// keeps its order as a 16-bit integer of the same signedness, so two packed
// 16-bit max / min (v_pk_max_[iu]16) do the odd and the even bytes and one
// v_perm_b32 interleaves them back -- 9 VALU per 4 elements.  Integers have no
// NaN or signed zero, so this is (a > b) ? a : b byte for byte
// (tests/test_swar.py checks every byte pair in every lane).
template <typename T, bool MAX> MPIX_DEV uint32_t minmax_bytes(uint32_t a, uint32_t b)
{
    typedef __attribute__((ext_vector_type(2)))
        typename std::conditional<std::is_signed<T>::value, short, unsigned short>::type v2;
    const uint32_t m = 0xff00ff00u;
    const v2 ao = __builtin_bit_cast(v2, a & m), bo = __builtin_bit_cast(v2, b & m);
    const v2 ae = __builtin_bit_cast(v2, (a << 8) & m), be = __builtin_bit_cast(v2, (b << 8) & m);
    uint32_t ro, re;
    if constexpr (MAX) {
        ro = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(ao, bo));
        re = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(ae, be));
    } else {
        ro = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(ao, bo));
        re = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(ae, be));
    }
    // bytes 0..3 = re.b1, ro.b1, re.b3, ro.b3 (selector 0-3: re, 4-7: ro)
    return __builtin_amdgcn_perm(ro, re, 0x07030501u);
}

template <typename T> struct IMax {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (a > b) ? a : b; }
    static MPIX_DEV uint32_t apply4(uint32_t a, uint32_t b) { return minmax_bytes<T, true>(a, b); }
};
template <typename T> struct IMin {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (a < b) ? a : b; }
    static MPIX_DEV uint32_t apply4(uint32_t a, uint32_t b) { return minmax_bytes<T, false>(a, b); }
};
template <typename T> struct ISum {
    using unit = T;
    using W = typename Wide<T>::type;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (T) ((W) a + (W) b); }
};
template <typename T> struct IProd {
    using unit = T;
    using W = typename Wide<T>::type;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (T) ((W) a * (W) b); }
};
// 1-byte logicals, four lanes per dword (SWAR, combine16 uses apply4 when a
// combiner has it): nz(x) sets bit 7 of every non-zero byte -- the low seven
// bits plus 0x7f carry into bit 7 exactly when one of them is set, or bit 7
// itself is -- so each op is 4-10 VALU per 4 elements instead of ~5 per byte.
// Byte for byte the same 0/1 results as apply().
MPIX_DEV uint32_t nz_bytes(uint32_t x) { return (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u; }

template <typename T> struct ILand {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (T) ((a != 0) & (b != 0)); }
    static MPIX_DEV uint32_t apply4(uint32_t a, uint32_t b) { return (nz_bytes(a) & nz_bytes(b)) >> 7; }
};
template <typename T> struct ILor {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (T) ((a != 0) | (b != 0)); }
    static MPIX_DEV uint32_t apply4(uint32_t a, uint32_t b) { return nz_bytes(a | b) >> 7; }
};
template <typename T> struct ILxor {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (T) ((a != 0) ^ (b != 0)); }
    static MPIX_DEV uint32_t apply4(uint32_t a, uint32_t b) { return (nz_bytes(a) ^ nz_bytes(b)) >> 7; }
};
template <typename T> struct IBand {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return a & b; }
};
template <typename T> struct IBor {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return a | b; }
};
template <typename T> struct IBxor {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return a ^ b; }
};

// Fortran logicals: MPII_FROM_FLOG(x) = (x == .FALSE. ? 0 : 1), compared after
// the usual promotion; MPII_TO_FLOG(c) = c ? .TRUE. : .FALSE. cast to T.
// The logical kinds are signed (int8..int128) and .FALSE. is an int
// (mpii_fortlogical.h:13), so the comparison is in int up to 4-byte kinds --
// exactly C's promotion, and one 32-bit compare per element instead of a
// sign-extended 64-bit one.
template <typename T> struct FlogW { using type = int; };
template <> struct FlogW<int64_t> { using type = long long; };
template <> struct FlogW<__int128> { using type = __int128; };
template <typename T> MPIX_DEV int flog_from(T x, const Params &p)
{
    using W = typename FlogW<T>::type;
    return ((W) x == (W) p.ffalse) ? 0 : 1;
}
template <typename T> MPIX_DEV T flog_to(int c, const Params &p)
{
    return (T) (c ? p.ftrue : p.ffalse);
}
// Kind-1 logicals four per dword (combine16 uses apply4p when a 1-byte
// combiner has it; the byte-array form needed scratch on gfx950): bit 7 of
// every byte that is .TRUE., i.e. differs from .FALSE. as flog_from compares
// (in int: a .FALSE. outside -128..127 equals no byte), and the results as
// the low bytes of .TRUE. / .FALSE. as flog_to casts them.  Byte for byte
// the same as apply() (tests/test_swar.py).
MPIX_DEV uint32_t flog_true_bytes(uint32_t x, const Params &p)
{
    const int f = (int) p.ffalse;
    if (f < -128 || f > 127)
        return 0x80808080u;
    return nz_bytes(x ^ ((uint32_t) (uint8_t) f * 0x01010101u));
}
MPIX_DEV uint32_t flog_to_bytes(uint32_t t, const Params &p)
{
    const uint32_t m = (t >> 7) * 0xffu;
    return ((uint32_t) (uint8_t) p.ftrue * 0x01010101u & m) |
           ((uint32_t) (uint8_t) p.ffalse * 0x01010101u & ~m);
}
template <typename T> struct FLand {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &p)
    {
        return flog_to<T>(flog_from(a, p) & flog_from(b, p), p);
    }
    static MPIX_DEV uint32_t apply4p(uint32_t a, uint32_t b, const Params &p)
    {
        return flog_to_bytes(flog_true_bytes(a, p) & flog_true_bytes(b, p), p);
    }
};
template <typename T> struct FLor {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &p)
    {
        return flog_to<T>(flog_from(a, p) | flog_from(b, p), p);
    }
    static MPIX_DEV uint32_t apply4p(uint32_t a, uint32_t b, const Params &p)
    {
        return flog_to_bytes(flog_true_bytes(a, p) | flog_true_bytes(b, p), p);
    }
};
template <typename T> struct FLxor {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &p)
    {
        return flog_to<T>(flog_from(a, p) ^ flog_from(b, p), p);
    }
    static MPIX_DEV uint32_t apply4p(uint32_t a, uint32_t b, const Params &p)
    {
        return flog_to_bytes(flog_true_bytes(a, p) ^ flog_true_bytes(b, p), p);
    }
};

// ------------------------------------------------------------ floating point
// MAX/MIN are MPL_MAX/MPL_MIN selects (src/mpl/include/mpl_base.h:105-106):
// with a NaN on either side the result is b, bit for bit; MAX(+0,-0) = -0.
// hipcc lowers these to v_cmp + v_cndmask (not v_max_*, whose NaN/zero
// rules differ).
template <typename T> struct FMax {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (a > b) ? a : b; }
};
template <typename T> struct FMin {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return (a < b) ? a : b; }
};
template <typename T> struct FSum {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return a + b; }
};
template <typename T> struct FProd {
    using unit = T;
    static MPIX_DEV T apply(T a, T b, const Params &) { return a * b; }
};

// bf16 SUM (op_fns.c:459-493): widen, fp32 add, store (u>>16) + ((u&0x8000)?1:0),
// i.e. round half away on the magnitude bits, no NaN special case.
struct Bf16Sum {
    using unit = uint16_t;
    static MPIX_DEV uint16_t apply(uint16_t a, uint16_t b, const Params &)
    {
        float fa = __builtin_bit_cast(float, (uint32_t) a << 16);
        float fb = __builtin_bit_cast(float, (uint32_t) b << 16);
        uint32_t u = __builtin_bit_cast(uint32_t, fa + fb);
        return (uint16_t) ((u >> 16) + ((u & 0x8000u) ? 1u : 0u));
    }
};

// ------------------------------------------------------------------ complex
template <typename R> struct alignas(2 * sizeof(R)) Cplx {
    R re, im;
};

// component-wise SUM (op_fns.c:27-42)
template <typename R> struct CSum {
    using unit = Cplx<R>;
    static MPIX_DEV unit apply(unit a, unit b, const Params &)
    {
        unit c;
        c.re = a.re + b.re;
        c.im = a.im + b.im;
        return c;
    }
};

// C-native complex product (MPIR_OP_TYPE_GROUP(C_COMPLEX), op_fns.c:61-71):
// what "a * b" on float/double _Complex computes under C99 Annex G -- the
// plain (ac-bd, ad+bc) and, only when both parts come out NaN, the
// infinity-recovery of G.5.1 (libgcc __mulsc3/__muldc3).  a = inout, b = in.
template <typename R> MPIX_DEV R cpsign(R mag, R sgn) { return __builtin_copysign(mag, sgn); }
template <> MPIX_DEV float cpsign<float>(float mag, float sgn) { return __builtin_copysignf(mag, sgn); }

template <typename R> struct CProdAnnexG {
    using unit = Cplx<R>;
    static MPIX_DEV unit apply(unit x, unit y, const Params &)
    {
        R a = x.re, b = x.im, c = y.re, d = y.im;
        R ac = a * c, bd = b * d, ad = a * d, bc = b * c;
        unit z;
        z.re = ac - bd;
        z.im = ad + bc;
        if (__builtin_expect(__builtin_isnan(z.re) && __builtin_isnan(z.im), 0))
            z = recover(a, b, c, d, ac, bd, ad, bc, z);
        return z;
    }
    static MPIX_DEV unit recover(R a, R b, R c, R d, R ac, R bd, R ad, R bc, unit z)
    {
        bool recalc = false;
        const R one = 1, zero = 0;
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = cpsign(__builtin_isinf(a) ? one : zero, a);
            b = cpsign(__builtin_isinf(b) ? one : zero, b);
            if (__builtin_isnan(c)) c = cpsign(zero, c);
            if (__builtin_isnan(d)) d = cpsign(zero, d);
            recalc = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = cpsign(__builtin_isinf(c) ? one : zero, c);
            d = cpsign(__builtin_isinf(d) ? one : zero, d);
            if (__builtin_isnan(a)) a = cpsign(zero, a);
            if (__builtin_isnan(b)) b = cpsign(zero, b);
            recalc = true;
        }
        if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) ||
                        __builtin_isinf(ad) || __builtin_isinf(bc))) {
            if (__builtin_isnan(a)) a = cpsign(zero, a);
            if (__builtin_isnan(b)) b = cpsign(zero, b);
            if (__builtin_isnan(c)) c = cpsign(zero, c);
            if (__builtin_isnan(d)) d = cpsign(zero, d);
            recalc = true;
        }
        if (recalc) {
            const R inf = __builtin_huge_val();
            R t0 = a * c, t1 = b * d, t2 = a * d, t3 = b * c;
            z.re = inf * (t0 - t1);
            z.im = inf * (t2 + t3);
        }
        return z;
    }
};

// struct complex (MPIR_OP_TYPE_GROUP(COMPLEX), op_fns.c:74-85) on fp16 parts:
// re = c.re*b.re - c.im*b.im; im = c.im*b.re + c.re*b.im, each fp16 op
// rounded (native _Float16, no excess precision on gfx950).
// The four products and the two sums as packed fp16 pairs (v_pk_mul_f16 /
// v_pk_add_f16 with operand selects): (p1, p3) = (re, im) * y.re, (p2, p4) =
// (im, re) * y.im, z = (p1 - p2, p3 + p4) -- each lane the same single
// correctly rounded fp16 op as the scalar form, 3 VALU per element instead of 7.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
struct CProdHalf {
    using unit = Cplx<_Float16>;
    static MPIX_DEV unit apply(unit x, unit y, const Params &)
    {
        const h2v xv = {x.re, x.im}, xs = {x.im, x.re};
        const h2v yr = {y.re, y.re}, yi = {y.im, y.im};
        const h2v a = xv * yr;          // (p1, p3)
        const h2v b = xs * yi;          // (p2, p4)
        const h2v sg = {(_Float16) -1, (_Float16) 1};
        const h2v z = a + b * sg;       // (p1 - p2, p3 + p4): * -1 is exact
        unit r;
        r.re = z.x;
        r.im = z.y;
        return r;
    }
};

// -------------------------------------------------------------- pair types
// MAXLOC/MINLOC (op_fns.c:299-435): if a.v < b.v (MAXLOC) take b's value and
// loc; else if a.v <= b.v (a tie) loc = MPL_MIN(a.loc, b.loc); NaN in either
// value leaves a unchanged.  Padding bytes of a are preserved.
template <typename V, typename L> struct alignas(sizeof(V) >= sizeof(L) ? sizeof(V) : sizeof(L)) BPair {
    V v;
    L l;
};
struct alignas(8) FloatInt { float v; int32_t l; };
struct alignas(8) DoubleIntBody { double v; int32_t l; int32_t pad; };
struct alignas(8) LongIntBody { int64_t v; int32_t l; int32_t pad; };
struct alignas(8) ShortInt { int16_t v; int16_t pad; int32_t l; };

template <typename P, bool IsMax> struct Loc {
    using unit = P;
    static MPIX_DEV P apply(P a, P b, const Params &)
    {
        bool take = IsMax ? (a.v < b.v) : (a.v > b.v);
        bool tie = IsMax ? (a.v <= b.v) : (a.v >= b.v);
        P r = a;
        if (take) {
            r.v = b.v;
            r.l = b.l;
        } else if (tie) {
            r.l = (a.l < b.l) ? a.l : b.l;
        }
        return r;
    }
};

// ------------------------------------------ x87 extended and IEEE binary128
// MPI_LONG_DOUBLE on x86-64 Linux is the x87 80-bit extended format in a
// 16-byte slot (MPIR_ALT_FLOAT128, mpir_datatype.h:82; MPIR_OP_TYPE_GROUP(
// FLOATING_POINT) lists it, mpir_op_util.h:211-217): bytes 0-7 the 64-bit
// significand with its explicit integer bit J (bit 63), bytes 8-9 sign and
// 15-bit exponent, bytes 10-15 padding.  MPI_REAL16 is IEEE binary128
// (MPIR_FLOAT128, __float128).  MAX/MIN/MAXLOC/MINLOC on them only compare and
// select, so they are done here in integer arithmetic, bit-exact with what gcc
// makes of op_fns.c on x86-64: fcomi's ordering, and for long double the
// result stored with fstpt -- the 10 value bytes, inout's padding kept.
// fcomi (and __gttf2/__lttf2 for binary128) report "unordered" for a NaN and,
// for x87, for the formats the 387 and later do not support: unnormals
// (exponent != 0 with J = 0), pseudo-infinities and pseudo-NaNs (exponent
// 0x7fff with J = 0).  Pseudo-denormals (exponent 0 with J = 1) compare as
// the normal of exponent 1 with the same significand, as do denormals by
// value (both are m * 2^(1 - 16383 - 63)); zeros of either sign are equal.
enum { kCmpLt = 0, kCmpEq = 1, kCmpGt = 2, kCmpUn = 3 };

MPIX_DEV int sign_mag_cmp(bool sa, bool sb, int mag, bool both_zero)
{
    if (both_zero)
        return kCmpEq;
    if (sa != sb)
        return sa ? kCmpLt : kCmpGt;
    if (mag == 0)
        return kCmpEq;
    return (mag < 0) != sa ? kCmpLt : kCmpGt;
}

MPIX_DEV int x87_cmp(const X87 &a, const X87 &b)
{
    const uint32_t ea = (uint32_t) a.se & 0x7fffu, eb = (uint32_t) b.se & 0x7fffu;
    const bool ja = (a.m >> 63) != 0, jb = (b.m >> 63) != 0;
    const bool bad_a = (ea != 0 && !ja) || (ea == 0x7fffu && (a.m << 1) != 0);
    const bool bad_b = (eb != 0 && !jb) || (eb == 0x7fffu && (b.m << 1) != 0);
    if (bad_a || bad_b)
        return kCmpUn;
    // magnitude key (max(e, 1), m); zero is (1, 0), below every other value
    const uint32_t ka = ea ? ea : 1u, kb = eb ? eb : 1u;
    const int mag = ka != kb ? (ka < kb ? -1 : 1) : (a.m != b.m ? (a.m < b.m ? -1 : 1) : 0);
    return sign_mag_cmp((a.se >> 15) & 1, (b.se >> 15) & 1, mag,
                        ea == 0 && eb == 0 && a.m == 0 && b.m == 0);
}

// `a = v` as fstpt does it: the 10 value bytes of v, a's padding kept
MPIX_DEV X87 x87_store(X87 a, const X87 &v)
{
    a.m = v.m;
    a.se = (a.se & ~(uint64_t) 0xffff) | (v.se & 0xffff);
    return a;
}

struct X87Max {
    using unit = X87;
    static MPIX_DEV X87 apply(X87 a, X87 b, const Params &)
    {
        return x87_cmp(a, b) == kCmpGt ? a : x87_store(a, b);
    }
};
struct X87Min {
    using unit = X87;
    static MPIX_DEV X87 apply(X87 a, X87 b, const Params &)
    {
        return x87_cmp(a, b) == kCmpLt ? a : x87_store(a, b);
    }
};

MPIX_DEV int quad_cmp(const Quad &a, const Quad &b)
{
    const uint64_t ma = a.hi & 0x7fffffffffffffffull, mb = b.hi & 0x7fffffffffffffffull;
    const uint64_t inf = 0x7fff000000000000ull;
    if (ma > inf || (ma == inf && a.lo) || mb > inf || (mb == inf && b.lo))
        return kCmpUn;
    const int mag = ma != mb ? (ma < mb ? -1 : 1) : (a.lo != b.lo ? (a.lo < b.lo ? -1 : 1) : 0);
    return sign_mag_cmp(a.hi >> 63, b.hi >> 63, mag, (ma | a.lo | mb | b.lo) == 0);
}

struct QuadMax {
    using unit = Quad;
    static MPIX_DEV Quad apply(Quad a, Quad b, const Params &) { return quad_cmp(a, b) == kCmpGt ? a : b; }
};
struct QuadMin {
    using unit = Quad;
    static MPIX_DEV Quad apply(Quad a, Quad b, const Params &) { return quad_cmp(a, b) == kCmpLt ? a : b; }
};

// MPI_LONG_DOUBLE_INT {long double; int} (pairtypes.c:15-21: extent 32, the
// int at 16, bytes 20-31 padding) and the builtin pair of binary128
// (MPIR_2FLOAT128, loc a binary128 too): the loop of op_fns.c:303-352 with
// the comparisons above.  32-byte units: element-wise kernels only.
struct alignas(16) LongDoubleInt {
    X87 v;
    int32_t l;
    int32_t pad[3];
};
template <bool IsMax> struct LocX87 {
    using unit = LongDoubleInt;
    static MPIX_DEV unit apply(unit a, unit b, const Params &)
    {
        const int c = x87_cmp(a.v, b.v);
        unit r = a;
        if (c == (IsMax ? kCmpLt : kCmpGt)) {
            r.v = x87_store(a.v, b.v);
            r.l = b.l;
        } else if (c == kCmpEq) {
            r.l = (a.l < b.l) ? a.l : b.l;
        }
        return r;
    }
};
struct alignas(16) QuadPair {
    Quad v, l;
};
template <bool IsMax> struct LocQuad {
    using unit = QuadPair;
    static MPIX_DEV unit apply(unit a, unit b, const Params &)
    {
        const int c = quad_cmp(a.v, b.v);
        unit r = a;
        if (c == (IsMax ? kCmpLt : kCmpGt)) {
            r.v = b.v;
            r.l = b.l;
        } else if (c == kCmpEq && quad_cmp(a.l, b.l) != kCmpLt) {
            r.l = b.l;      // MPL_MIN(a.l, b.l) on the binary128 locs
        }
        return r;
    }
};

#undef MPIX_DEV

}  // namespace mpix
