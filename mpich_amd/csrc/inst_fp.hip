// inst_fp.hip -- floating-point and complex combiners
// (MPIR_OP_TYPE_GROUP(FLOATING_POINT) / (C_COMPLEX) / (COMPLEX) and the bf16
// SUM helper, src/include/mpir_op_util.h:211-236, op_fns.c:19-91,459-493).
#include "redop_kernels.h"

namespace mpix {

namespace {

template <typename T>
const Entry *real_ops(int opi)
{
    static const Entry tab[4] = { entry<FMax<T>>(), entry<FMin<T>>(), entry<FSum<T>>(),
                                  entry<FProd<T>>() };
    return (opi >= 1 && opi <= 4) ? &tab[opi - 1] : nullptr;
}

template <typename R>
const Entry *cplx_ops(int opi)
{
    static const Entry tab[2] = { entry<CSum<R>>(), entry<CProdAnnexG<R>>() };
    return (opi == 3 || opi == 4) ? &tab[opi - 3] : nullptr;
}

const Entry *cplx_half_ops(int opi)
{
    static const Entry tab[2] = { entry<CSum<_Float16>>(), entry<CProdHalf>() };
    return (opi == 3 || opi == 4) ? &tab[opi - 3] : nullptr;
}

// MPI_LONG_DOUBLE (x87 in 16 bytes) and MPI_REAL16 (binary128): MAX / MIN
// compare and select in integer arithmetic (redop_ops.h), SUM / PROD in
// software extended / quad arithmetic (redop_soft.h)
template <class Max, class Min, class Sum, class Prod>
const Entry *soft_ops(int opi)
{
    static const Entry tab[4] = { entry<Max>(), entry<Min>(), entry<Sum>(), entry<Prod>() };
    return (opi >= 1 && opi <= 4) ? &tab[opi - 1] : nullptr;
}

// their complex forms: binary128 struct complex SUM / PROD, x87 C complex SUM / PROD
const Entry *quadc_ops(int opi)
{
    static const Entry tab[2] = { entry<QuadCSum>(), entry<QuadCProd>() };
    return (opi == 3 || opi == 4) ? &tab[opi - 3] : nullptr;
}

const Entry *x87c_ops(int opi)
{
    static const Entry tab[2] = { entry<X87CSum>(), entry<X87CProd>() };
    return (opi == 3 || opi == 4) ? &tab[opi - 3] : nullptr;
}

const Entry *bf16_ops(int opi)
{
    static const Entry e = entry<Bf16Sum>();
    return opi == 3 ? &e : nullptr;     // only MPIR_SUM handles MPIR_BFLOAT16
}

}  // namespace

const Entry *lookup_fp(int raw, int opi)
{
    switch ((unsigned) raw) {
        case 0x4c830200u: return real_ops<_Float16>(opi);
        case 0x4c830400u: return real_ops<float>(opi);
        case 0x4c830800u: return real_ops<double>(opi);
        case 0x4c840400u: return cplx_half_ops(opi);
        case 0x4c840800u: return cplx_ops<float>(opi);
        case 0x4c841000u: return cplx_ops<double>(opi);
        case 0x4c850200u: return bf16_ops(opi);
        case 0x4c851000u: return soft_ops<X87Max, X87Min, X87Sum, X87Prod>(opi);
        case 0x4c831000u: return soft_ops<QuadMax, QuadMin, QuadSum, QuadProd>(opi);
        case 0x4c842000u: return quadc_ops(opi);
        case 0x4c862000u: return x87c_ops(opi);
        default: return nullptr;
    }
}

int unroll() { return MPIX_REDOP_UNROLL; }

}  // namespace mpix

#define MPIX_STR2(x) #x
#define MPIX_STR(x) MPIX_STR2(x)
extern "C" const char *mpix_build_info(void)
{
    return "libmpix_redop gfx950 HIP " MPIX_STR(HIP_VERSION_MAJOR) "." MPIX_STR(HIP_VERSION_MINOR)
        " unroll=" MPIX_STR(MPIX_REDOP_UNROLL) " nt_load=" MPIX_STR(MPIX_REDOP_NT_LOAD)
        " nt_store=" MPIX_STR(MPIX_REDOP_NT_STORE) " grouped_loads=" MPIX_STR(MPIX_REDOP_GROUPED_LOADS);
}
