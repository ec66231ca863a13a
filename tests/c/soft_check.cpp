// Host build of mpich_amd/csrc/redop_soft.h (MPIX_SOFT_HOST): the software
// x87 / binary128 arithmetic the gfx950 kernels run, as C entry points over
// n elements, so tests/test_soft_fp.py can check it against the oracle's
// gcc-built loops on the CPU (x87 hardware, libgcc soft-fp).  Test
// infrastructure only.
#define MPIX_SOFT_HOST 1
#include "redop_soft.h"

#include <string.h>

using namespace mpix;

template <class C>
static void run(const void *in, void *inout, long n)
{
    typedef typename C::unit T;
    const Params prm{1, 0};
    for (long i = 0; i < n; ++i) {
        T a, b;
        memcpy(&a, (const char *) inout + i * sizeof(T), sizeof(T));
        memcpy(&b, (const char *) in + i * sizeof(T), sizeof(T));
        T r = C::apply(a, b, prm);
        memcpy((char *) inout + i * sizeof(T), &r, sizeof(T));
    }
}

// the sums through the general path only (x87_add / quad_add with FAST =
// false): the normal-operand fast paths must give the same bits
struct X87SumGeneral {
    using unit = X87;
    static X87 apply(X87 a, X87 b, const Params &) { return x87_add<false>(a, b, false); }
};
struct QuadSumGeneral {
    using unit = Quad;
    static Quad apply(Quad a, Quad b, const Params &) { return quad_add<false>(a, b, false); }
};

// a split combiner as the kernels run it: apply_fast, and where it declined
// (its result unspecified: the kernels keep the unit as it was) the full apply
template <class C>
static int run_split(const void *in, void *inout, long n)
{
    typedef typename C::unit T;
    const Params prm{1, 0};
    for (long i = 0; i < n; ++i) {
        T a, b;
        memcpy(&a, (const char *) inout + i * sizeof(T), sizeof(T));
        memcpy(&b, (const char *) in + i * sizeof(T), sizeof(T));
        bool ok = false;
        T r = C::apply_fast(a, b, prm, ok);
        if (!ok)
            r = C::apply(a, b, prm);
        memcpy((char *) inout + i * sizeof(T), &r, sizeof(T));
    }
    return 0;
}

// which: 0 x87 SUM, 1 x87 PROD, 2 binary128 SUM, 3 binary128 PROD,
// 4 binary128 complex SUM, 5 binary128 complex PROD, 6 x87 complex SUM, 7 x87 complex PROD,
// 8 x87 SUM general path only, 9 binary128 SUM general path only,
// 10 binary128 complex PROD split form, 11 x87 complex PROD split form
extern "C" int soft_reduce(int which, const void *in, void *inout, long n)
{
    switch (which) {
        case 0: run<X87Sum>(in, inout, n); return 0;
        case 1: run<X87Prod>(in, inout, n); return 0;
        case 2: run<QuadSum>(in, inout, n); return 0;
        case 3: run<QuadProd>(in, inout, n); return 0;
        case 4: run<QuadCSum>(in, inout, n); return 0;
        case 5: run<QuadCProd>(in, inout, n); return 0;
        case 6: run<X87CSum>(in, inout, n); return 0;
        case 7: run<X87CProd>(in, inout, n); return 0;
        case 8: run<X87SumGeneral>(in, inout, n); return 0;
        case 9: run<QuadSumGeneral>(in, inout, n); return 0;
        case 10: return run_split<QuadCProd>(in, inout, n);
        case 11: return run_split<X87CProd>(in, inout, n);
    }
    return -1;
}
