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
// only -- compare and select (redop_ops.h); SUM / PROD stay with the caller's
// CPU op table (MPIX_Redop_is_supported answers 0 for them)
template <class Max, class Min>
const Entry *select_ops(int opi)
{
    static const Entry tab[2] = { entry<Max>(), entry<Min>() };
    return (opi == 1 || opi == 2) ? &tab[opi - 1] : nullptr;
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
        case 0x4c851000u: return select_ops<X87Max, X87Min>(opi);
        case 0x4c831000u: return select_ops<QuadMax, QuadMin>(opi);
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
