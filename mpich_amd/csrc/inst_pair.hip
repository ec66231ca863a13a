// inst_pair.hip -- MAXLOC / MINLOC over builtin pairs {T v; T loc}
// (MPIR_2INT8.. MPIR_2FLOAT64, op_fns.c:303-330) and the struct pair types
// MPI_{FLOAT,DOUBLE,LONG,SHORT,LONG_DOUBLE}_INT {T v; int loc} (op_fns.c:337-352,
// pairtypes.c:15-121), and MPIR_2FLOAT128.
#include "redop_kernels.h"

namespace mpix {

namespace {

template <typename P>
const Entry *loc_ops(int opi)
{
    static const Entry tab[2] = { entry<Loc<P, false>>(), entry<Loc<P, true>>() };
    return (opi == 11 || opi == 12) ? &tab[opi - 11] : nullptr;     // MINLOC, MAXLOC
}

// the long double / binary128 pairs: their own comparisons (redop_ops.h)
template <template <bool> class L>
const Entry *loc_ops_cmp(int opi)
{
    static const Entry tab[2] = { entry<L<false>>(), entry<L<true>>() };
    return (opi == 11 || opi == 12) ? &tab[opi - 11] : nullptr;
}

}  // namespace

const Entry *lookup_pair(int raw, int opi)
{
    switch ((unsigned) raw) {
        case 0x4cc10200u: return loc_ops<BPair<int8_t, int8_t>>(opi);
        case 0x4cc10400u: return loc_ops<BPair<int16_t, int16_t>>(opi);
        case 0x4cc10800u: return loc_ops<BPair<int32_t, int32_t>>(opi);
        case 0x4cc11000u: return loc_ops<BPair<int64_t, int64_t>>(opi);
        case 0x4cc20200u: return loc_ops<BPair<uint8_t, uint8_t>>(opi);
        case 0x4cc20400u: return loc_ops<BPair<uint16_t, uint16_t>>(opi);
        case 0x4cc20800u: return loc_ops<BPair<uint32_t, uint32_t>>(opi);
        case 0x4cc21000u: return loc_ops<BPair<uint64_t, uint64_t>>(opi);
        case 0x4cc30400u: return loc_ops<BPair<_Float16, _Float16>>(opi);
        case 0x4cc30800u: return loc_ops<BPair<float, float>>(opi);
        case 0x4cc31000u: return loc_ops<BPair<double, double>>(opi);
        case 0x8c000000u: return loc_ops<FloatInt>(opi);
        case 0x8c000001u: return loc_ops<DoubleIntBody>(opi);
        case 0x8c000002u: return loc_ops<LongIntBody>(opi);
        case 0x8c000003u: return loc_ops<ShortInt>(opi);
        case 0x8c000004u: return loc_ops_cmp<LocX87>(opi);      // MPI_LONG_DOUBLE_INT
        case 0x4cc32000u: return loc_ops_cmp<LocQuad>(opi);     // MPIR_2FLOAT128
        default: return nullptr;
    }
}

}  // namespace mpix
