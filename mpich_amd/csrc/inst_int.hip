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

// MPIX_EQUAL (src/mpi/coll/op/opequal.c:20-35): MPI_BYTE buffers whose first
// 8 bytes are an is_equal flag; inout's flag becomes 0 if either flag is not
// 1 or the payloads differ.  Not element-wise: a byte compare whose only
// effect is zeroing one word, so every wave that sees a difference stores the
// zero (idempotent, no atomics needed).
__global__ void __launch_bounds__(256)
k_equal(const unsigned char *__restrict__ in, unsigned char *__restrict__ io, uint64_t n)
{
    uint64_t hin, hio;
    __builtin_memcpy(&hin, in, 8);
    __builtin_memcpy(&hio, io, 8);
    const uint64_t zero = 0;
    if (hin != 1 || hio != 1) {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            __builtin_memcpy(io, &zero, 8);
        return;
    }
    const uint64_t data = n - 8, npk = data / 16;
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    bool diff = false;
    for (uint64_t k = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; k < npk; k += stride) {
        v4u a = ld16u(reinterpret_cast<const char *>(io) + 8 + 16 * k);
        v4u b = ld16u(reinterpret_cast<const char *>(in) + 8 + 16 * k);
        diff |= (a.x != b.x) | (a.y != b.y) | (a.z != b.z) | (a.w != b.w);
    }
    if (blockIdx.x == 0)
        for (uint64_t t = 8 + npk * 16 + threadIdx.x; t < n; t += blockDim.x)
            diff |= in[t] != io[t];
    if (diff)
        __builtin_memcpy(io, &zero, 8);
}

hipError_t launch_equal(const void *in, void *io, uint64_t n, hipStream_t s)
{
    uint64_t npk = (n - 8) / 16;
    unsigned grid = grid_for(256ull * 4, npk, 0, 256);
    hipLaunchKernelGGL(k_equal, dim3(grid), dim3(256), 0, s,
                       static_cast<const unsigned char *>(in), static_cast<unsigned char *>(io), n);
    return hipGetLastError();
}

// Up to kMaxMultiInputs independent copies in one launch (blockIdx.y picks
// the segment): the allgather step of a pull schedule reads P-1 peers' blocks
// over P-1 links at once instead of P-1 stream-serialised copies.  16-byte
// packets where source and destination share a 16-byte phase, bytes otherwise.
struct CopySegs {
    const unsigned char *src[kMaxMultiInputs];
    unsigned char *dst[kMaxMultiInputs];
    uint64_t bytes[kMaxMultiInputs];
};

// wt_xcd: the store policy of the contiguous kernel (blocks on these XCDs
// store write-through)
__global__ void __launch_bounds__(256) k_copy_multi(CopySegs sg, unsigned wt_xcd)
{
    const bool wt = wt_xcd && ((wt_xcd >> (xcc_id() & 7)) & 1);
    const int q = blockIdx.y;
    const unsigned char *src = sg.src[q];
    unsigned char *dst = sg.dst[q];
    const uint64_t n = sg.bytes[q];
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uintptr_t as = reinterpret_cast<uintptr_t>(src) & 15, ad = reinterpret_cast<uintptr_t>(dst) & 15;
    if (as == ad) {
        const uint64_t head = ((16 - ad) & 15) < n ? ((16 - ad) & 15) : n;
        const uint64_t npk = (n - head) / 16;
        const v4u *vs = reinterpret_cast<const v4u *>(src + head);
        v4u *vd = reinterpret_cast<v4u *>(dst + head);
        for (uint64_t k = t0; k < npk; k += stride)
            st16_pol<true>(vd + k, ld16<true>(vs + k), wt);
        if (blockIdx.x == 0) {
            for (uint64_t t = threadIdx.x; t < head; t += blockDim.x)
                dst[t] = src[t];
            for (uint64_t t = head + npk * 16 + threadIdx.x; t < n; t += blockDim.x)
                dst[t] = src[t];
        }
    } else {
        for (uint64_t k = t0; k < n; k += stride)
            dst[k] = src[k];
    }
}

hipError_t launch_copy_multi(const void *const *srcs, void *const *dsts, const uint64_t *bytes,
                             int n, hipStream_t s, unsigned wt_xcd)
{
    CopySegs sg{};
    uint64_t most = 0;
    for (int q = 0; q < n; ++q) {
        sg.src[q] = static_cast<const unsigned char *>(srcs[q]);
        sg.dst[q] = static_cast<unsigned char *>(dsts[q]);
        sg.bytes[q] = bytes[q];
        most = bytes[q] > most ? bytes[q] : most;
    }
    // about 2048 workgroups in all: each segment's share of the 256 CUs
    unsigned gx = grid_for(256ull * 16 * 4, most, (int) (2048 / (unsigned) n), 256);
    hipLaunchKernelGGL(k_copy_multi, dim3(gx, (unsigned) n), dim3(256), 0, s, sg, wt_xcd & 0xffu);
    return hipGetLastError();
}

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
