// redop_dispatch.h -- host-visible interface between the C-ABI
// (redop_capi.cpp, plain host C++) and the kernel instantiation units
// (inst_*.hip).  No device code here.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace mpix {

// Runtime parameters some combiners need (Fortran .TRUE./.FALSE.,
// src/include/mpii_fortlogical.h:15,28), and the completion word of a
// synchronous call: when `done` is set, the contiguous launcher guarantees
// that done_seq is stored to it once the combine is complete and visible to
// the host -- by the kernel itself when it runs as at most kSignalMaxGrid
// workgroups (the last one to finish, counted on done_ctr, stores it: no
// end-of-kernel + stream-packet round trip), else by a stream write after it.
struct Params {
    long long ftrue;
    long long ffalse;
    uint32_t *done = nullptr;       // pinned, fine-grained host word
    uint32_t *done_ctr = nullptr;   // device word, 0 between launches
    uint32_t done_seq = 0;
    // blocks from this index on store write-through (sc0 sc1: the line leaves
    // the XCD's L2 at once instead of staying dirty until the end-of-kernel
    // write-back); 0xffffffff = none (LaunchCfg::wt_tail)
    uint32_t wt_from = 0xffffffffu;
    uint32_t wt_every = 0;      // and blocks b with b % wt_every == wt_phase (0 = none)
    uint32_t wt_phase = 0;
    uint32_t wt_xcd = 0;        // and every block running on an XCD whose bit is set
    // split combiners (is_split, redop_kernels.h): one 64-bit word per 64
    // units, bit j set when unit 64 w + j left its fast path (fixup_buffer)
    uint64_t *fixup = nullptr;
};

constexpr unsigned kSignalMaxGrid = 64;     // 64 tiles of 64 x 1 packets: 64 KiB per operand

struct LaunchCfg {
    int block;          // threads per block (multiple of 64)
    int max_grid;       // 0 = no cap (one tile per block)
    int wt_tail;        // contiguous kernel: the last wt_tail blocks store write-through
    int wt_every;       // ... and blocks b with b % wt_every == wt_phase
    int wt_phase;
    int wt_xcd;         // ... and blocks on the XCDs (HW_REG_XCC_ID) of this bit mask
};

// One (op, type) pair: launchers for the contiguous and the vector-target form.
struct Entry {
    hipError_t (*contig)(const void *in, void *io, uint64_t count, const Params &,
                         const LaunchCfg &, hipStream_t);
    hipError_t (*vector)(const void *in, void *io, uint64_t count, uint64_t blocklen,
                         uint64_t stride, const Params &, const LaunchCfg &, hipStream_t);
    hipError_t (*multi)(const void *const *ins, int k, void *io, uint64_t count, const Params &,
                        const LaunchCfg &, hipStream_t);
    hipError_t (*iov)(const void *in, void *io, const int64_t *d_seg_off, const int64_t *d_prefix,
                      const int64_t *d_src_off, int64_t nseg, uint64_t total, const Params &,
                      const LaunchCfg &, hipStream_t);
    hipError_t (*tree)(const void *const *ins, int k, void *out, uint64_t count, const Params &,
                       const LaunchCfg &, hipStream_t);
    hipError_t (*batch)(const void *const *ins, void *const *ios, const uint64_t *counts, int k,
                        const Params &, const LaunchCfg &, hipStream_t);
};

// Most blocks one dispatch of `block`-thread workgroups may have: HIP caps a
// dispatch at UINT32_MAX work-items (gridDim.x * blockDim.x), so with one-wave
// blocks that is 2^26 - 1 blocks, not 2^31.  Every kernel
// launched through grid_for strides over the rest.
constexpr uint64_t max_blocks(uint64_t block)
{
    return 0xffffffffull / (block ? block : 1);
}

inline unsigned grid_for(uint64_t work_per_block_units, uint64_t n, int max_grid, uint64_t block)
{
    uint64_t g = (n + work_per_block_units - 1) / work_per_block_units;
    if (g == 0)
        g = 1;
    if (max_grid > 0 && g > (uint64_t) max_grid)
        g = (uint64_t) max_grid;
    if (g > max_blocks(block))
        g = max_blocks(block);
    return (unsigned) g;
}

constexpr int kMaxBatchSegs = 64;       // MPIX_BATCH_MAX

constexpr int kMaxMultiInputs = 16;

// Each instantiation unit resolves (raw internal type, op index) to an Entry
// or returns nullptr.  raw = handle & 0xffffff00 for builtins; struct pair
// handles 0x8c00000k are passed unchanged.
const Entry *lookup_int(int raw, int opi);
const Entry *lookup_fp(int raw, int opi);
const Entry *lookup_pair(int raw, int opi);

// MPIX_EQUAL on an MPI_BYTE buffer of n >= 8 bytes (opequal.c:20-35)
hipError_t launch_equal(const void *in, void *io, uint64_t n, hipStream_t s);

// up to kMaxMultiInputs independent device copies in one launch
// A device buffer of at least `bytes` for the split combiners' fixup words,
// one per (device, stream): stream order serialises its users; grown (after
// synchronising the stream) when a larger call comes; freed by
// MPIX_Redop_finalize.  nullptr when it cannot be allocated.
uint64_t *fixup_buffer(hipStream_t s, size_t bytes);

hipError_t launch_copy_multi(const void *const *srcs, void *const *dsts, const uint64_t *bytes,
                             int n, hipStream_t s, unsigned wt_xcd = 0);

// compile-time unroll of the packet kernel (packets per lane per operand)
int unroll();

}  // namespace mpix
