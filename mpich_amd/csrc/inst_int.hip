// inst_int.hip -- integer and Fortran-logical combiners
// (MPIR_OP_TYPE_GROUP(INTEGER) / (FORTRAN_LOGICAL), src/include/mpir_op_util.h:195-244).
#include "redop_kernels.h"

namespace mpix {

namespace {

template <typename S, typename U>
const Entry *int_ops(int opi)
{
    // SUM/PROD/bitwise/logical are sign-agnostic bit patterns: share the
    // unsigned instantiation; only MAX/MIN depend on signedness.
    static const Entry tab[11] = {
        Entry{nullptr, nullptr, nullptr, nullptr},
        entry<IMax<S>>(), entry<IMin<S>>(), entry<ISum<U>>(), entry<IProd<U>>(),
        entry<ILand<U>>(), entry<IBand<U>>(), entry<ILor<U>>(), entry<IBor<U>>(),
        entry<ILxor<U>>(), entry<IBxor<U>>(),
    };
    return (opi >= 1 && opi <= 10) ? &tab[opi] : nullptr;
}

template <typename U>
const Entry *uint_minmax(int opi)
{
    static const Entry tab[2] = { entry<IMax<U>>(), entry<IMin<U>>() };
    return (opi == 1 || opi == 2) ? &tab[opi - 1] : nullptr;
}

template <typename S>
const Entry *flog_ops(int opi)
{
    static const Entry tab[3] = { entry<FLand<S>>(), entry<FLor<S>>(), entry<FLxor<S>>() };
    switch (opi) {
        case 5: return &tab[0];
        case 7: return &tab[1];
        case 9: return &tab[2];
        default: return nullptr;
    }
}

}  // namespace

const Entry *lookup_int(int raw, int opi)
{
    switch ((unsigned) raw) {
        case 0x4c810100u: return int_ops<int8_t, uint8_t>(opi);
        case 0x4c810200u: return int_ops<int16_t, uint16_t>(opi);
        case 0x4c810400u: return int_ops<int32_t, uint32_t>(opi);
        case 0x4c810800u: return int_ops<int64_t, uint64_t>(opi);
        case 0x4c811000u: return int_ops<__int128, unsigned __int128>(opi);
        case 0x4c820100u: return (opi <= 2) ? uint_minmax<uint8_t>(opi) : int_ops<int8_t, uint8_t>(opi);
        case 0x4c820200u: return (opi <= 2) ? uint_minmax<uint16_t>(opi) : int_ops<int16_t, uint16_t>(opi);
        case 0x4c820400u: return (opi <= 2) ? uint_minmax<uint32_t>(opi) : int_ops<int32_t, uint32_t>(opi);
        case 0x4c820800u: return (opi <= 2) ? uint_minmax<uint64_t>(opi) : int_ops<int64_t, uint64_t>(opi);
        case 0x4c821000u:
            return (opi <= 2) ? uint_minmax<unsigned __int128>(opi)
                              : int_ops<__int128, unsigned __int128>(opi);
        case 0x4c870100u: return flog_ops<int8_t>(opi);
        case 0x4c870200u: return flog_ops<int16_t>(opi);
        case 0x4c870400u: return flog_ops<int32_t>(opi);
        case 0x4c870800u: return flog_ops<int64_t>(opi);
        case 0x4c871000u: return flog_ops<__int128>(opi);
        default: return nullptr;
    }
}

}  // namespace mpix
