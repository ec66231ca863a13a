// redop_capi.cpp -- the C-ABI of libmpix_redop.so (include/mpix_redop.h).
//
// Host side of the drop-in for MPIR_Reduce_local
// (src/mpi/coll/reduce_local/reduce_local.c:53-96): handle decoding,
// (op, datatype) legality, pointer classification, the per-thread stream,
// host-buffer staging, and the dispatch to the gfx950 kernels instantiated in
// inst_{int,fp,pair}.hip.  There is no CPU compute path here: a combination
// the GPU path does not cover returns MPIX_REDOP_ERR_TYPE and
// MPIX_Redop_is_supported() says so, so the caller keeps its own op table
// for it (exactly how reduce_local.c:66-76 falls back when yaksa declines).
#include <hip/hip_runtime_api.h>
#include <immintrin.h>

#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "mpix_redop.h"
#include "redop_dispatch.h"

using mpix::Entry;
using mpix::LaunchCfg;
using mpix::Params;

namespace {

// ---------------------------------------------------------------- handles
// Builtin index -> internal type (raw, index bits clear) and the binding
// group used by MPIR_op_dt_check.  LP64 x86-64 with Fortran: INTEGER, REAL,
// LOGICAL 4 bytes; DOUBLE PRECISION 8; long double 16 (x87 80-bit); bool 1.
// Source: src/mpi/datatype/typeutil.c:29-109 resolved by configure.ac:3446-3609.
enum Group { GN = 0, GCI, GFI, GFP, GLOG, GCPX, GBYTE, GMULTI };

struct Builtin {
    uint32_t internal;
    uint8_t group;
};

constexpr uint32_t I8 = 0x4c810100u, I16 = 0x4c810200u, I32 = 0x4c810400u, I64 = 0x4c810800u,
    I128 = 0x4c811000u, U8 = 0x4c820100u, U16 = 0x4c820200u, U32 = 0x4c820400u,
    U64 = 0x4c820800u, F16 = 0x4c830200u, F32 = 0x4c830400u, F64 = 0x4c830800u,
    F128 = 0x4c831000u, C16 = 0x4c840400u, C32 = 0x4c840800u, C64 = 0x4c841000u,
    C128 = 0x4c842000u, BF16 = 0x4c850200u, LD = 0x4c851000u, LDC = 0x4c862000u,
    L8 = 0x4c870100u, L16 = 0x4c870200u, L32 = 0x4c870400u, L64 = 0x4c870800u,
    L128 = 0x4c871000u, FX0 = 0x4c800000u, FX8 = 0x4c800100u, P2I32 = 0x4cc10800u,
    P2F32 = 0x4cc30800u, P2F64 = 0x4cc31000u;

struct BuiltinTable {
    Builtin e[0x4d];
    BuiltinTable() : e()
    {
        auto set = [this](int i, uint32_t t, uint8_t g) { e[i] = Builtin{t, g}; };
        set(0x01, I8, GCI);    set(0x02, U8, GCI);    set(0x03, I16, GCI);   set(0x04, U16, GCI);
        set(0x05, I32, GCI);   set(0x06, U32, GCI);   set(0x07, I64, GCI);   set(0x08, U64, GCI);
        set(0x09, I64, GCI);   set(0x0a, F32, GFP);   set(0x0b, F64, GFP);   set(0x0c, LD, GFP);
        set(0x0d, U8, GBYTE);  set(0x0e, I32, GN);    set(0x0f, FX8, GN);    set(0x10, FX0, GN);
        set(0x11, FX0, GN);    set(0x16, P2I32, GN);  set(0x18, I8, GCI);    set(0x19, U64, GCI);
        set(0x1a, I8, GN);     set(0x1b, I32, GFI);   set(0x1c, F32, GFP);   set(0x1d, L32, GLOG);
        set(0x1e, C32, GCPX);  set(0x1f, F64, GFP);   set(0x20, P2I32, GN);  set(0x21, P2F32, GN);
        set(0x22, C64, GCPX);  set(0x23, P2F64, GN);  set(0x26, F16, GFP);   set(0x27, F32, GFP);
        set(0x28, C32, GCPX);  set(0x29, F64, GFP);   set(0x2a, C64, GCPX);  set(0x2b, F128, GFP);
        set(0x2c, C128, GCPX); set(0x2d, I8, GFI);    set(0x2e, C16, GCPX);  set(0x2f, I16, GFI);
        set(0x30, I32, GFI);   set(0x31, I64, GFI);   set(0x32, I128, GFI);  set(0x33, I8, GLOG);
        set(0x34, C32, GCPX);  set(0x35, C64, GCPX);  set(0x36, LDC, GCPX);  set(0x37, I8, GCI);
        set(0x38, I16, GCI);   set(0x39, I32, GCI);   set(0x3a, I64, GCI);   set(0x3b, U8, GCI);
        set(0x3c, U16, GCI);   set(0x3d, U32, GCI);   set(0x3e, U64, GCI);   set(0x3f, I8, GLOG);
        set(0x40, C32, GCPX);  set(0x41, C64, GCPX);  set(0x42, LDC, GCPX);  set(0x43, I64, GMULTI);
        set(0x44, I64, GMULTI); set(0x45, I64, GMULTI); set(0x46, F16, GFP); set(0x47, L8, GLOG);
        set(0x48, L16, GLOG);  set(0x49, L32, GLOG);  set(0x4a, L64, GLOG);  set(0x4b, L128, GLOG);
        set(0x4c, BF16, GFP);
    }
};
const BuiltinTable kBuiltins;

constexpr uint32_t kNull = 0x0c000000u;

inline bool is_builtin(uint32_t h) { return (h >> 30) == 1u; }
inline bool is_struct_pair(uint32_t h) { return (h & 0xffffff00u) == 0x8c000000u && (h & 0xff) < 5; }
inline bool is_builtin_op(uint32_t op) { return (op >> 24) == 0x58u; }

// MPIR_DATATYPE_REPLACE_BUILTIN (mpir_datatype.h:169-176)
uint32_t to_internal(uint32_t dt)
{
    if (!is_builtin(dt) || (dt & 0x800000u))
        return dt;
    uint32_t idx = dt & 0xff;
    if (idx == 0 || idx >= 0x4d || kBuiltins.e[idx].internal == 0)
        return kNull;
    return kBuiltins.e[idx].internal | idx;
}

// element extent in bytes (pair padding included; pairtypes.c:15-21)
uint64_t extent_of(uint32_t it)
{
    if (is_struct_pair(it)) {
        static const uint64_t ext[5] = {8, 16, 16, 8, 32};
        return ext[it & 0xff];
    }
    if (!is_builtin(it) || it == kNull)
        return 0;
    return (it >> 8) & 0xff;
}

bool is_pairtype(uint32_t it)
{
    return is_struct_pair(it) || (is_builtin(it) && (it & 0x400000u));
}

int hip_err(hipError_t e);

// Type map of the struct pairs (pairtypes.c:24-80: a struct {value @0,
// int @idx_offset}, extent = sizeof the C struct).  DOUBLE_INT, LONG_INT,
// SHORT_INT and LONG_DOUBLE_INT have size < extent: their padding is not
// part of the type map, so a typemap copy (MPIR_Localcopy) leaves it alone
// and typerep_op_fallback treats them as "pairtype" (typerep_op.c:88).
struct PairMap {
    uint32_t value_bytes, loc_off;
};
bool padded_pair(uint32_t it, PairMap *pm)
{
    static const PairMap m[5] = {{4, 4}, {8, 8}, {8, 8}, {2, 4}, {16, 16}};
    if (!is_struct_pair(it) || (it & 0xff) == 0)
        return false;
    *pm = m[it & 0xff];
    return true;
}

// MPIR_Datatype_get_size_macro: bytes of data in one element
uint64_t size_of(uint32_t it)
{
    PairMap pm;
    if (padded_pair(it, &pm))
        return pm.value_bytes + 4;
    return extent_of(it);
}

// MPI_REPLACE (op_fns.c:445-457) = MPIR_Localcopy: `rows` elements at the
// given pitches.  Contiguous types copy whole extents; padded pairs copy the
// value and the int of each element (two pitched copies), so inout keeps its
// padding bytes exactly as the typemap copy does.
int replace_rows(void *dst, size_t dpitch, const void *src, size_t spitch, uint64_t rows,
                 uint32_t it, uint64_t ext, hipStream_t s)
{
    if (rows == 0)
        return MPIX_REDOP_SUCCESS;
    PairMap pm;
    if (!padded_pair(it, &pm)) {
        if (dpitch == ext && spitch == ext)
            return hip_err(hipMemcpyAsync(dst, src, rows * ext, hipMemcpyDeviceToDevice, s));
        return hip_err(hipMemcpy2DAsync(dst, dpitch, src, spitch, ext, rows,
                                        hipMemcpyDeviceToDevice, s));
    }
    int rc = hip_err(hipMemcpy2DAsync(dst, dpitch, src, spitch, pm.value_bytes, rows,
                                      hipMemcpyDeviceToDevice, s));
    if (rc == MPIX_REDOP_SUCCESS)
        rc = hip_err(hipMemcpy2DAsync((char *) dst + pm.loc_off, dpitch,
                                      (const char *) src + pm.loc_off, spitch, 4, rows,
                                      hipMemcpyDeviceToDevice, s));
    return rc;
}

// MPIR_Internal_op_dt_check (mpir_datatype.h:870-933)
bool internal_ok(uint32_t op, uint32_t it)
{
    if (!is_builtin_op(op))
        return false;
    uint32_t opi = op & 0xf;
    if (opi == 11 || opi == 12)
        return is_pairtype(it);
    if (opi >= 13)
        return true;
    if (!is_builtin(it) || !(it & 0x800000u) || (it & 0x400000u))
        return false;
    uint32_t kind = it & 0x0f0000u;
    switch (opi) {
        case 1: case 2:
            return kind == 0x010000u || kind == 0x020000u || kind == 0x030000u || kind == 0x050000u;
        case 3: case 4:
            return kind >= 0x010000u && kind <= 0x060000u;
        case 5: case 7: case 9:
            return kind == 0x010000u || kind == 0x020000u || kind == 0x070000u;
        case 6: case 8: case 10:
            return kind == 0x010000u || kind == 0x020000u;
        default:
            return false;
    }
}

// MPIR_op_dt_check (mpir_datatype.h:780-868), builtin datatypes
bool binding_ok(uint32_t op, uint32_t dt)
{
    if (!is_builtin_op(op))
        return false;
    uint32_t opi = op & 0xf;
    if (opi == 11 || opi == 12)
        return is_pairtype(to_internal(dt));
    if (opi >= 13)
        return true;
    if (!is_builtin(dt))
        return false;
    if (dt & 0x800000u)
        return internal_ok(op, dt);
    uint32_t idx = dt & 0xff;
    if (idx == 0 || idx >= 0x4d || kBuiltins.e[idx].internal == 0)
        return false;
    uint8_t g = kBuiltins.e[idx].group;
    switch (opi) {
        case 1: case 2: return g == GCI || g == GFI || g == GFP || g == GMULTI;
        case 3: case 4: return g == GCI || g == GFI || g == GFP || g == GCPX || g == GMULTI;
        case 5: case 7: case 9: return g == GCI || g == GLOG || g == GMULTI;
        case 6: case 8: case 10: return g == GCI || g == GFI || g == GBYTE || g == GMULTI;
        default: return false;
    }
}

extern "C" const char *mpix_build_info(void);

const Entry *gpu_entry(uint32_t opi, uint32_t it)
{
    uint32_t raw = is_struct_pair(it) ? it : (it & 0xffffff00u);
    const Entry *e = mpix::lookup_fp((int) raw, (int) opi);
    if (!e)
        e = mpix::lookup_int((int) raw, (int) opi);
    if (!e)
        e = mpix::lookup_pair((int) raw, (int) opi);
    return e;
}

// ---------------------------------------------------------------- state
std::atomic<long long> g_ftrue{1}, g_ffalse{0};
// One-wave (64-thread) blocks of one packet per lane (round 5): kernel-trace
// durations of the synchronous 1 GiB fp32 SUM call 478 -> 460 us against
// 256-thread blocks, 448.7 against 480.6 us back to back; config-3 rows
// +3.3 % (median), the multi-input fold +4-8 % (tools/contig_u_probe.hip,
// tools/gpu_env_ab.sh, profiles/r05_block64_ab.json).
std::atomic<int> g_block{64}, g_max_grid{0};
// Grid cap of kernels reading page-locked host memory over PCIe (zero-copy):
// with one tile per block every block loads its whole tile (host to device)
// before it stores (device to host), and a grid of a few hundred blocks is
// one round, so the two link directions take turns.  Looping blocks keep
// both busy: with 4 packets per lane 32 blocks of 256 took 4 MiB 235 -> 186 us,
// 16 MiB 780 -> 655 us, 1 GiB 39.2 -> 38.1 ms (profiles/r04_pinned_grid.json);
// with one packet per lane (round 5) twice the lanes hold the same bytes in
// flight -- 64 blocks of 256: 1 MiB 69 -> 55 us, 4 MiB 238 -> 182 us, 16 MiB
// 769 -> 655 us, 256 MiB 10.1 -> 9.4 ms, where 32 gave 59 / 197 / 682 us /
// 9.8 ms (tools/pinned_grid.py, profiles/r05_pinned_grid.json).  The default
// cap is that many lanes (kZcLanes) in blocks of the current size;
// MPIX_REDOP_ZC_GRID sets it in blocks (0: uncapped).
constexpr int kZcLanes = 64 * 256;
constexpr int kZcAuto = -1;
std::atomic<int> g_zc_grid{kZcAuto};
// Store policy of the contiguous and multi-input kernels and the two-slot tree
// (MPIX_Redop_set_store_policy): the blocks running on the XCDs of g_wt_xcd
// store write-through (sc0 sc1), the others non-temporally.  Two XCDs of eight
// writing through make the 1 GiB fp32 SUM kernel 8-9 % faster at every operand
// placement tried, and every config-3 row 1-10 % faster (median 8 %); one XCD
// gains 4 %, three or four XCDs lose 1-5 %, all eight lose 3 %
// (profiles/r03_wt_probe_xcd.json, r03_wt_types_xcd88.json,
// r03_wt_sync_sweeps.txt).  Default: XCDs 3 and 7 on devices of 8 XCDs (SPX),
// off otherwise.  g_wt_every / g_wt_phase / g_wt_tail select blocks by index
// instead (the probes' forms).
// g_wt_xcd = kWtAuto until the first launch settles the default (resolve_wt,
// the only HIP query of the knobs: reading or setting them, and the support
// predicates, never start the HIP runtime).
constexpr int kWtAuto = -1;
std::atomic<int> g_wt_tail{0}, g_wt_every{0}, g_wt_phase{0}, g_wt_xcd{kWtAuto};
// The synchronous entry's own mask (MPIX_Redop_set_sync_store_policy, env
// MPIX_REDOP_WT_XCD_SYNC): MPIX_Reduce_local -- the MPIR_Reduce_local drop-in
// -- is timed by its callers call by call, each kernel starting from an idle
// GPU, and there XCDs 1 and 5 writing through (0x22) beat XCDs 3 and 7 (0x88)
// by 1.7-3.2 % per call on three boxes although the kernel alone is 2 %
// slower with it (profiles/r05_sync_xcd_masks.json).  The
// stream-ordered entries, whose kernels run back to back, keep g_wt_xcd.
// kWtAuto: an explicit g_wt_xcd if one was set, else the sync default.
std::atomic<int> g_wt_xcd_sync{kWtAuto};
std::once_flag g_wt_once;
// completion wait of the synchronous calls: 0 block (hipStreamSynchronize),
// 1 spin on an event, 2 spin on a pinned host word that a one-workgroup
// contiguous kernel stores itself and the stream writes after any other
// kernel (hipStreamWriteValue32; default), 3 the same word always written by
// the stream (10.1 vs 13.2 us for a 1-element call against the event,
// profiles/r01_lat_probe.txt) -- MPIX_REDOP_SYNC=block|event|flag|stream
std::atomic<int> g_sync{2};
std::atomic<bool> g_zero_copy{true}; // MPIX_REDOP_PINNED=stage stages pinned host memory too
std::once_flag g_env_once;
size_t g_stage_chunk = (size_t) 64 << 20;
// pageable operands up to this many bytes are copied (host memcpy) into a
// pinned bounce buffer the kernel reads and writes over PCIe, instead of three
// pageable hipMemcpy calls (each a driver-side bounce of its own);
// MPIX_REDOP_BOUNCE_BYTES, 0 disables
size_t g_bounce_bytes = (size_t) 1 << 20;
// large pageable operands (at least two chunks in the wave form below, two
// chunks per worker in the worker form): this many host threads copy chunks
// of g_pipe_chunk bytes into pinned buffers that zero-copy kernels combine
// (MPIX_REDOP_PAGEABLE_THREADS, 0 = always stream the chunks through device
// scratch with hipMemcpyAsync; MPIX_REDOP_PAGEABLE_CHUNK).  Wave form, 8 x
// 64 MiB: 1 GiB in 45-46 ms, 0.88 x the pinned zero-copy call
// (profiles/r03_pageable_wave_ramp.jsonl)
std::atomic<int> g_pipe_threads{8};
std::atomic<size_t> g_pipe_chunk{(size_t) 64 << 20};
// Worker form only: with MPIX_REDOP_PAGEABLE_DB=1 each worker keeps two slots
// and copies chunk k + W into one while the kernel of chunk k reads the other
// (default one slot: measured no faster, twice the pinned memory,
// profiles/r03_pageable_sweep.jsonl).  Both forms: the workers can be pinned
// to the CPUs of the GPU's own NUMA node (MPIX_REDOP_PAGEABLE_AFFINITY=gpu, or
// an explicit cpulist such as "64-127"; default "none" leaves them where the
// scheduler puts them -- pinning measured no faster either)
std::atomic<bool> g_pipe_db{false};
std::string g_pipe_affinity = "none";
// Pageable form (MPIX_REDOP_PAGEABLE_MODE): "wave" (default) -- all workers
// copy the same chunk in together (each a slice), ONE zero-copy kernel per
// chunk runs while they copy the next one in and the one before out, three
// pinned chunk buffers in rotation, chunk sizes ramped at both ends.  A
// zero-copy kernel pays a ramp of ~0.16 ms however large
// (profiles/r03_pinned_chunks.json), so large chunks win, and the ramped ends
// keep the pipeline fill short: 1 GiB in 45-46 ms at 8 x 64 MiB against
// 53 ms for the worker form (profiles/r03_pageable_wave_ramp.jsonl).
// "worker": each worker copies, combines and copies back chunks of its own.
std::atomic<int> g_pipe_wave{1};
// Support-predicate knobs, the pattern of MPIR_CVAR_ENABLE_YAKSA_REDUCTION and
// MPIR_CVAR_YAKSA_REDUCTION_THRESHOLD (typerep_yaksa_pack.c:44-64,229-240):
// MPIX_REDOP_ENABLE=0 makes every predicate answer 0 (the caller keeps its CPU
// op table); MPIX_REDOP_THRESHOLD > 0 declines calls whose packed size
// (count * type size) exceeds it (default -1, no limit).  The pointer-aware
// predicate also declines operands that are BOTH host-resident below a floor
// (MPIX_REDOP_HOST_FLOOR for pageable memory, MPIX_REDOP_PINNED_FLOOR for
// page-locked memory, bytes per operand): there one core's op_fns.c loop beats
// the PCIe round trip (crossover measured by bench.py's host_crossover leg).
std::atomic<bool> g_enable{true};
std::atomic<long long> g_threshold{-1};
// defaults from the crossover on MI355X + EPYC 9575F boxes, including the
// driver's (BENCH_r03 host_crossover, profiles/r04_pageable_swing.json): one
// core matches the pageable path up to 64 MiB per operand (the staged form at
// 1.00-1.05 x its time) and loses to it from 128 MiB on (0.4-0.8 x).  The
// page-locked zero-copy call lost to one core at 4 MiB (236 vs 216 us on the
// driver's box) until its kernel was capped to looping blocks (g_zc_grid):
// 169 vs 219 us at 4 MiB, even at 1 MiB (profiles/r04_bench_n1_zc.json).
// Below the floors MPICH keeps its op_fns.c loop.
std::atomic<long long> g_host_floor{(long long) 128 << 20};
std::atomic<long long> g_pinned_floor{(long long) 4 << 20};
// MPIX_Op_table entries return void, like MPIR_op_function: a call the GPU
// path declines aborts by default, as op_fns.c's MPIR_Assert(0) does
// (op_fns.c:51-53); MPIX_REDOP_OPFN_ABORT=0 only records the error
// (MPIX_Redop_last_error)
std::atomic<bool> g_opfn_abort{true};

void read_env()
{
    if (const char *s = getenv("MPIX_REDOP_BLOCK")) {
        int b = atoi(s);
        if (b >= 64 && b <= 1024 && b % 64 == 0)
            g_block = b;
    }
    if (const char *s = getenv("MPIX_REDOP_WT_TAIL"))
        g_wt_tail = atoi(s) > 0 ? atoi(s) : 0;
    if (const char *s = getenv("MPIX_REDOP_WT_EVERY"))
        g_wt_every = atoi(s) > 0 ? atoi(s) : 0;
    if (const char *s = getenv("MPIX_REDOP_WT_PHASE"))
        g_wt_phase = atoi(s) > 0 ? atoi(s) : 0;
    if (g_wt_every > 0)
        g_wt_phase = g_wt_phase % g_wt_every;
    if (const char *s = getenv("MPIX_REDOP_WT_XCD"))
        g_wt_xcd = (int) (strtol(s, nullptr, 0) & 0xff);
    if (const char *s = getenv("MPIX_REDOP_WT_XCD_SYNC"))
        g_wt_xcd_sync = (int) (strtol(s, nullptr, 0) & 0xff);
    if (const char *s = getenv("MPIX_REDOP_MAXGRID"))
        g_max_grid = atoi(s) > 0 ? atoi(s) : 0;
    if (const char *s = getenv("MPIX_REDOP_ZC_GRID"))
        g_zc_grid = atoi(s) > 0 ? atoi(s) : 0;
    if (const char *s = getenv("MPIX_REDOP_SYNC"))
        g_sync = strcmp(s, "block") == 0 ? 0
               : strcmp(s, "flag") == 0  ? 2
               : strcmp(s, "stream") == 0 ? 3
                                          : 1;
    if (const char *s = getenv("MPIX_REDOP_PINNED"))
        g_zero_copy = strcmp(s, "stage") != 0;
    if (const char *s = getenv("MPIX_REDOP_STAGE_CHUNK")) {
        long long c = atoll(s);
        if (c >= 4096)
            g_stage_chunk = (size_t) c;
    }
    if (const char *s = getenv("MPIX_REDOP_PAGEABLE_THREADS")) {
        int t = atoi(s);
        if (t >= 0 && t <= 16)
            g_pipe_threads = t;
    }
    if (const char *s = getenv("MPIX_REDOP_PAGEABLE_DB"))
        g_pipe_db = atoi(s) != 0;
    if (const char *s = getenv("MPIX_REDOP_PAGEABLE_MODE"))
        g_pipe_wave = strcmp(s, "worker") != 0;
    if (const char *s = getenv("MPIX_REDOP_PAGEABLE_AFFINITY"))
        g_pipe_affinity = s;
    if (const char *s = getenv("MPIX_REDOP_PAGEABLE_CHUNK")) {
        long long c = atoll(s);
        if (c >= 65536 && c <= (256ll << 20))
            g_pipe_chunk = (size_t) c;
    }
    if (const char *s = getenv("MPIX_REDOP_ENABLE"))
        g_enable = atoi(s) != 0;
    if (const char *s = getenv("MPIX_REDOP_THRESHOLD"))
        g_threshold = atoll(s);
    if (const char *s = getenv("MPIX_REDOP_HOST_FLOOR"))
        g_host_floor = atoll(s);
    if (const char *s = getenv("MPIX_REDOP_PINNED_FLOOR"))
        g_pinned_floor = atoll(s);
    if (const char *s = getenv("MPIX_REDOP_OPFN_ABORT"))
        g_opfn_abort = atoi(s) != 0;

    if (const char *s = getenv("MPIX_REDOP_BOUNCE_BYTES")) {
        long long c = atoll(s);
        if (c >= 0 && c <= (64ll << 20))
            g_bounce_bytes = (size_t) c;
    }
}

thread_local int t_last_error = 0;

constexpr int kMaxDev = 64;
constexpr int kSyncTimingMax = 1 << 16;    // calls one MPIX_Redop_sync_timing covers
struct DevState {
    bool init = false;
    hipStream_t s[2] = {nullptr, nullptr};
    hipEvent_t done = nullptr;          // completion marker for the spin wait
    volatile uint32_t *flag = nullptr;  // pinned host word for MPIX_REDOP_SYNC=flag
    uint32_t *flag_ctr = nullptr;       // device word: workgroups done (Params::done_ctr)
    uint32_t seq = 0;
    void *scratch = nullptr;    // 2 slots x (in chunk + inout chunk)
    size_t scratch_bytes = 0;
    // iov run tables, two slots used in turn, so back-to-back iov calls only
    // wait for the call before the previous one
    struct IovSlot {
        int64_t *tab = nullptr;     // device copy of the run table
        int64_t *host = nullptr;    // its pinned host staging copy
        size_t cap = 0;             // capacity of both in int64 entries
        hipEvent_t done = nullptr;  // recorded after the launches that read it
    } iov[2];
    uint32_t iov_next = 0;
    char *bounce = nullptr;     // pinned host: in half + inout half, bounce_half bytes each
    char *bounce_dev = nullptr; // its device mapping
    size_t bounce_half = 0;
    // MPIX_Redop_sync_timing: an event pair around the launch of each of the
    // next t_cap synchronous calls on s[0] (t_used recorded so far)
    std::vector<hipEvent_t> tev;
    int t_cap = 0, t_used = 0;
};

// Large pageable operands: one stream + pinned slot pair per host worker, ONE
// set per device for the whole process (not per calling thread), so the
// pinned footprint is workers x 2 x chunk (256 MiB at the defaults) per device
// however many MPI_THREAD_MULTIPLE threads call in.  A call that finds the set
// busy stages its operands instead (same kernel, same bits).
struct PipeSlot {
    hipStream_t s = nullptr;
    char *host = nullptr;   // nbuf buffers of (in half + inout half), half bytes each
    char *dev = nullptr;    // its device mapping
    hipEvent_t ev[2] = {nullptr, nullptr};   // kernel of the chunk in buffer 0 / 1 done
};
struct PipeSet {
    std::mutex mu;
    PipeSlot slot[16];
    // wave mode: 3 chunk buffers (in half + inout half each), one stream
    char *ring = nullptr, *ring_dev = nullptr;
    size_t ring_half = 0;
    hipStream_t ring_s = nullptr;
    hipEvent_t ring_ev[3] = {nullptr, nullptr, nullptr};
    size_t half = 0;        // slot half size; slots [0, threads) hold host != nullptr
    int nbuf = 0;           // buffers per worker (2: double-buffered)
    bool cpus_known = false;
    std::vector<int> cpus;  // worker CPUs (empty: no pinning)
};
PipeSet *g_pipes = new PipeSet[64];     // per device; never destroyed (finalize frees the memory)
// Per-thread device state (streams, flag word, scratch).  A thread that exits
// hands its array to a process-wide pool and the next new thread takes it over
// instead of creating streams of its own, so MPI_THREAD_MULTIPLE codes that
// spawn and join worker threads keep a bounded set of HIP streams.  The hand-off
// makes no HIP call (it may run at process exit); work still queued on the
// streams stays ordered ahead of the next owner's.  MPIX_Redop_finalize frees
// the caller's array and the pooled ones.
std::mutex g_pool_mu;
std::vector<DevState *> *g_pool = new std::vector<DevState *>();  // never destroyed
struct DevHolder {
    DevState *arr = nullptr;
    ~DevHolder()
    {
        if (arr) {
            std::lock_guard<std::mutex> l(g_pool_mu);
            g_pool->push_back(arr);
        }
    }
};
thread_local DevHolder t_dev;

int set_err(int e)
{
    t_last_error = e;
    return e;
}

int hip_err(hipError_t e)
{
    if (e == hipSuccess)
        return MPIX_REDOP_SUCCESS;
    if (getenv("MPIX_REDOP_VERBOSE"))
        fprintf(stderr, "mpix_redop: HIP error %d (%s)\n", (int) e, hipGetErrorString(e));
    return MPIX_REDOP_ERR_OTHER;
}

DevState *dev_state(int dev)
{
    if (dev < 0 || dev >= kMaxDev)
        return nullptr;
    if (!t_dev.arr) {
        std::lock_guard<std::mutex> l(g_pool_mu);
        if (!g_pool->empty()) {
            t_dev.arr = g_pool->back();
            g_pool->pop_back();
        } else {
            t_dev.arr = new DevState[kMaxDev];
        }
    }
    DevState &d = t_dev.arr[dev];
    if (!d.init) {
        for (int k = 0; k < 2; ++k)
            if (hipStreamCreateWithFlags(&d.s[k], hipStreamNonBlocking) != hipSuccess)
                return nullptr;
        if (hipEventCreateWithFlags(&d.done, hipEventDisableTiming) != hipSuccess)
            return nullptr;
        void *f = nullptr;
        if (hipHostMalloc(&f, 64, hipHostMallocCoherent) == hipSuccess) {
            d.flag = (volatile uint32_t *) f;
            *d.flag = 0;
            void *c = nullptr;
            if (hipMalloc(&c, 256) == hipSuccess) {
                // zeroed on the state's own stream and waited for: the
                // null-stream hipMemset is not ordered before kernels on the
                // non-blocking streams that read this counter
                if (hipMemsetAsync(c, 0, 256, d.s[0]) == hipSuccess &&
                    hipStreamSynchronize(d.s[0]) == hipSuccess)
                    d.flag_ctr = (uint32_t *) c;
                else
                    (void) hipFree(c);
            }
        }
        d.init = true;
    }
    return &d;
}

// The environment knobs, read once; no HIP call (CPU-only entry points --
// the support predicates, the knob getters and setters -- come through here).
void env()
{
    std::call_once(g_env_once, read_env);
}

// The default store policy, settled at the first launch that needs it: XCDs
// 3 and 7 write through when every visible device has 8 XCDs (SPX), else
// none.  While g_wt_xcd is kWtAuto (no MPIX_REDOP_WT_XCD, no explicit mask
// from MPIX_Redop_set_store_policy, or -1 set there) the launches use it.
std::atomic<int> g_wt_default{kWtAuto}, g_wt_sync_default{kWtAuto};
int wt_default(bool sync = false)
{
    std::call_once(g_wt_once, [] {
        int ndev = 0;
        bool spx = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
        for (int d = 0; spx && d < ndev; ++d) {
            int x = 0;
            spx = hipDeviceGetAttribute(&x, hipDeviceAttributeNumberOfXccs, d) == hipSuccess &&
                  x == 8;
        }
        (void) hipGetLastError();
        g_wt_default = spx ? 0x88 : 0;
        g_wt_sync_default = spx ? 0x22 : 0;
    });
    return sync ? g_wt_sync_default.load() : g_wt_default.load();
}

// Launch geometry and store policy of a kernel about to be enqueued (sync:
// for the synchronous entry, g_wt_xcd_sync).
LaunchCfg launch_cfg(bool zero_copy = false, bool sync = false)
{
    env();
    int wt = g_wt_xcd.load();
    if (sync) {
        const int ws = g_wt_xcd_sync.load();
        if (ws != kWtAuto)
            wt = ws;
        else if (wt == kWtAuto)
            wt = wt_default(true);
    }
    if (wt == kWtAuto)
        wt = wt_default();
    LaunchCfg c{g_block.load(), g_max_grid.load(), g_wt_tail.load(), g_wt_every.load(),
                g_wt_phase.load(), wt};
    if (!zero_copy)
        return c;
    // ... of one whose operand(s) include page-locked host memory (g_zc_grid)
    int z = g_zc_grid.load();
    if (z == kZcAuto)
        z = kZcLanes / (c.block > 0 ? c.block : 64);
    if (zero_copy && z > 0 && (c.max_grid <= 0 || c.max_grid > z))
        c.max_grid = z;
    return c;
}

Params params() { return Params{g_ftrue.load(), g_ffalse.load()}; }

// Spin until the pinned completion word holds `seq`.  The stream is queried
// every 4096 spins once 20 ms have passed (a query inside a short spin costs
// latency): an idle stream means the work and the word's store are done; a
// stream in an error state (a faulted kernel) ends the wait with that error
// instead of spinning forever.
int spin_on_flag(DevState *d, hipStream_t s, uint32_t seq)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 1; __atomic_load_n(d->flag, __ATOMIC_ACQUIRE) != seq; ++spins) {
        if ((spins & 0xfff) != 0 ||
            std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20))
            continue;
        hipError_t q = hipStreamQuery(s);
        if (q == hipErrorNotReady)
            continue;
        if (q == hipSuccess)
            return MPIX_REDOP_SUCCESS;
        return hip_err(q);
    }
    return MPIX_REDOP_SUCCESS;
}

// Completion wait of the synchronous entry points.  MPI progress engines
// poll; a blocking hipStreamSynchronize costs wake-up latency per call, and an
// event query goes through the runtime's signal path, so by default the
// stream writes a sequence number into pinned host memory after the kernel and
// the caller spins on that word.
int wait_stream(DevState *d, hipStream_t s)
{
    int mode = g_sync.load();
    if (mode == 0)
        return hip_err(hipStreamSynchronize(s));
    hipError_t e;
    if ((mode == 2 || mode == 3) && d->flag) {
        uint32_t seq = ++d->seq;
        e = hipStreamWriteValue32(s, (void *) d->flag, seq, 0);
        if (e != hipSuccess)
            return hip_err(e);
        return spin_on_flag(d, s, seq);
    }
    e = hipEventRecord(d->done, s);
    if (e != hipSuccess)
        return hip_err(e);
    while ((e = hipEventQuery(d->done)) == hipErrorNotReady) {
    }
    return hip_err(e);
}

enum class Where { Device, Pinned, Pageable };

// Device / managed memory is used in place.  Pinned (page-locked, mapped)
// host memory is read and written by the kernel directly over PCIe
// ("zero-copy": one pass, both link directions busy at once) unless
// MPIX_REDOP_PINNED=stage; pageable host memory has to be staged.
Where classify(const void *p, int *dev, const void **devptr)
{
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    *devptr = p;
    if (e != hipSuccess) {
        (void) hipGetLastError();
        return Where::Pageable;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) {
        *dev = a.device;
        return Where::Device;
    }
    if (a.type == hipMemoryTypeHost && a.devicePointer) {
        // devicePointer maps the start of the allocation containing p
        *devptr = (const char *) a.devicePointer + ((const char *) p - (const char *) a.hostPointer);
        return Where::Pinned;
    }
    return Where::Pageable;
}

bool overlaps(const void *a, const void *b, uint64_t bytes)
{
    uintptr_t x = (uintptr_t) a, y = (uintptr_t) b;
    return x < y + bytes && y < x + bytes;
}

// Argument checks shared by every entry point: the binding-layer checks of
// MPI_Reduce_local (binding_c.py:2774-2783: op/datatype legality, buffer
// aliasing, no MPI_IN_PLACE) plus count < 0.  On success *it holds the
// internal type and *ext its extent.
int validate(const void *in, const void *io, MPIX_Aint count, uint32_t dt, uint32_t op,
             uint32_t *it, uint64_t *ext)
{
    if (count < 0)
        return MPIX_REDOP_ERR_COUNT;
    if (!is_builtin_op(op))
        return MPIX_REDOP_ERR_OP;
    *it = to_internal(dt);
    if (*it == kNull)
        return MPIX_REDOP_ERR_TYPE;
    *ext = extent_of(*it);
    if (*ext == 0)
        return MPIX_REDOP_ERR_TYPE;
    if (!internal_ok(op, *it))
        return MPIX_REDOP_ERR_OP;
    if (count == 0)
        return MPIX_REDOP_SUCCESS;
    // no buffer spans 2^56 bytes; beyond that count * extent could wrap
    if ((uint64_t) count > ((uint64_t) 1 << 56) / *ext)
        return MPIX_REDOP_ERR_COUNT;
    if (!in || !io || in == (const void *) -1 || io == (const void *) -1)
        return MPIX_REDOP_ERR_BUFFER;
    if (overlaps(in, io, (uint64_t) count * *ext))
        return MPIX_REDOP_ERR_BUFFER;
    return MPIX_REDOP_SUCCESS;
}

// Enqueue on a stream; both buffers device-accessible, arguments validated.
// done/seq (synchronous callers): on success with *signalled set, seq will be
// stored to *done once the result is complete (Params::done; ctr: its
// workgroup counter, NULL = one workgroup only).
int enqueue(const void *in, void *io, uint64_t count, uint32_t it, uint64_t ext, uint32_t op,
            hipStream_t s, uint32_t *done = nullptr, uint32_t *ctr = nullptr, uint32_t seq = 0,
            bool *signalled = nullptr, bool zero_copy = false, bool sync = false)
{
    if (signalled)
        *signalled = false;
    uint32_t opi = op & 0xf;
    if (opi == 14)      // MPI_NO_OP
        return MPIX_REDOP_SUCCESS;
    if (opi == 13)      // MPI_REPLACE = MPIR_Localcopy (op_fns.c:445-457)
        return replace_rows(io, ext, in, ext, count, it, ext, s);
    if (opi == 15)      // MPIX_EQUAL, MPI_BYTE only (opequal.c:22-23)
        return ((it & 0xffffff00u) == U8 && count >= 8)
            ? hip_err(mpix::launch_equal(in, io, count, s)) : MPIX_REDOP_ERR_TYPE;
    const Entry *e = gpu_entry(opi, it);
    if (!e)
        return MPIX_REDOP_ERR_TYPE;
    Params prm = params();
    prm.done = done;
    prm.done_ctr = ctr;
    prm.done_seq = seq;
    int rc = hip_err(e->contig(in, io, count, prm, launch_cfg(zero_copy, sync), s));
    if (signalled)
        *signalled = done && rc == MPIX_REDOP_SUCCESS;
    return rc;
}

// Synchronous combine of device-accessible operands on the library stream.
// With the default flag wait, the contiguous launcher signals completion
// itself (a kernel of at most kSignalMaxGrid workgroups stores the word,
// saving the end-of-kernel and stream-packet round trip:
// profiles/r01_sync_latency.txt); other ops and the other wait modes go
// through wait_stream.
int run_sync(DevState *d, const void *in, void *io, uint64_t count, uint32_t it, uint64_t ext,
             uint32_t op, bool zero_copy = false)
{
    launch_cfg();       // environment read before g_sync is consulted
    // timed call (MPIX_Redop_sync_timing): the pair brackets the launch on
    // the state's stream, nothing else changes
    const int ti = d->t_used < d->t_cap ? d->t_used++ : -1;
    if (ti >= 0) {
        int rc = hip_err(hipEventRecord(d->tev[2 * ti], d->s[0]));
        if (rc)
            return rc;
    }
    struct Stop {
        DevState *d;
        int ti;
        ~Stop()
        {
            if (ti >= 0)
                (void) hipEventRecord(d->tev[2 * ti + 1], d->s[0]);
        }
    };
    if (g_sync.load() == 2 && d->flag) {
        const uint32_t seq = ++d->seq;
        bool signalled = false;
        int rc;
        {
            Stop stop{d, ti};
            rc = enqueue(in, io, count, it, ext, op, d->s[0], (uint32_t *) d->flag, d->flag_ctr,
                         seq, &signalled, zero_copy, true);
        }
        if (signalled)      // the kernel stores the word itself
            return spin_on_flag(d, d->s[0], seq);
        int rc2 = wait_stream(d, d->s[0]);
        return rc ? rc : rc2;
    }
    int rc;
    {
        Stop stop{d, ti};
        rc = enqueue(in, io, count, it, ext, op, d->s[0], nullptr, nullptr, 0, nullptr, zero_copy,
                     true);
    }
    int rc2 = wait_stream(d, d->s[0]);
    return rc ? rc : rc2;
}

// Host-resident operand(s): stream them through device scratch in chunks,
// alternating two streams so chunk k+1's copies overlap chunk k's kernel.
// in_peer >= 0: `in` is device memory of that device, which `dev` cannot reach
// (no peer access): it is streamed the same way with hipMemcpyPeerAsync.
int staged(const void *in, void *io, uint64_t count, uint32_t it, uint64_t ext, uint32_t op,
           bool in_host, bool io_host, int dev, int in_peer = -1)
{
    if (in_peer >= 0)
        in_host = true;
    DevState *d = dev_state(dev);
    if (!d)
        return MPIX_REDOP_ERR_OTHER;
    launch_cfg();
    uint64_t chunk_elems = g_stage_chunk / ext;
    if (chunk_elems == 0)
        chunk_elems = 1;
    if (chunk_elems > count)
        chunk_elems = count;
    size_t slot_bytes = (size_t) (chunk_elems * ext + 255) & ~(size_t) 255;
    size_t need = 4 * slot_bytes;
    if (d->scratch_bytes < need) {
        if (d->scratch)
            (void) hipFree(d->scratch);
        d->scratch = nullptr;
        d->scratch_bytes = 0;
        if (hipMalloc(&d->scratch, need) != hipSuccess)
            return MPIX_REDOP_ERR_OTHER;
        d->scratch_bytes = need;
    }
    int rc = MPIX_REDOP_SUCCESS;
    for (uint64_t off = 0, k = 0; off < count && rc == MPIX_REDOP_SUCCESS; off += chunk_elems, ++k) {
        uint64_t n = (count - off < chunk_elems) ? count - off : chunk_elems;
        hipStream_t s = d->s[k & 1];
        char *slot = (char *) d->scratch + (k & 1) * 2 * slot_bytes;
        const char *src_in = (const char *) in + off * ext;
        char *dst_io = (char *) io + off * ext;
        const void *kin = src_in;
        void *kio = dst_io;
        if (in_peer >= 0) {
            rc = hip_err(hipMemcpyPeerAsync(slot, dev, src_in, in_peer, n * ext, s));
            kin = slot;
        } else if (in_host) {
            rc = hip_err(hipMemcpyAsync(slot, src_in, n * ext, hipMemcpyHostToDevice, s));
            kin = slot;
        }
        if (rc == MPIX_REDOP_SUCCESS && io_host) {
            rc = hip_err(hipMemcpyAsync(slot + slot_bytes, dst_io, n * ext,
                                        hipMemcpyHostToDevice, s));
            kio = slot + slot_bytes;
        }
        if (rc == MPIX_REDOP_SUCCESS)
            rc = enqueue(kin, kio, n, it, ext, op, s);
        if (rc == MPIX_REDOP_SUCCESS && io_host)
            rc = hip_err(hipMemcpyAsync(dst_io, kio, n * ext, hipMemcpyDeviceToHost, s));
    }
    int rc2 = wait_stream(d, d->s[0]);
    int rc3 = wait_stream(d, d->s[1]);
    return rc ? rc : (rc2 ? rc2 : rc3);
}

// MPIX_EQUAL with host-resident operand(s) too large for the bounce buffer:
// whole-buffer copies into device scratch, ONE k_equal launch, and the 8-byte
// is_equal header back (k_equal writes nothing else).  When the scratch
// cannot be had nothing has been touched and MPI_ERR_TYPE sends the caller to
// its own op table.
int equal_whole(const void *in, void *io, uint64_t n, bool in_host, bool io_host, int dev,
                int in_peer = -1)
{
    DevState *d = dev_state(dev);
    if (!d)
        return MPIX_REDOP_ERR_OTHER;
    const size_t half = ((size_t) n + 255) & ~(size_t) 255;
    if (d->scratch_bytes < 2 * half) {
        if (d->scratch) {
            (void) hipStreamSynchronize(d->s[0]);
            (void) hipStreamSynchronize(d->s[1]);
            (void) hipFree(d->scratch);
        }
        d->scratch = nullptr;
        d->scratch_bytes = 0;
        if (hipMalloc(&d->scratch, 2 * half) != hipSuccess) {
            (void) hipGetLastError();
            return MPIX_REDOP_ERR_TYPE;
        }
        d->scratch_bytes = 2 * half;
    }
    hipStream_t s = d->s[0];
    const void *kin = in;
    void *kio = io;
    int rc = MPIX_REDOP_SUCCESS;
    if (in_peer >= 0) {
        rc = hip_err(hipMemcpyPeerAsync(d->scratch, dev, in, in_peer, n, s));
        kin = d->scratch;
    } else if (in_host) {
        rc = hip_err(hipMemcpyAsync(d->scratch, in, n, hipMemcpyHostToDevice, s));
        kin = d->scratch;
    }
    if (rc == MPIX_REDOP_SUCCESS && io_host) {
        kio = (char *) d->scratch + half;
        rc = hip_err(hipMemcpyAsync(kio, io, n, hipMemcpyHostToDevice, s));
    }
    if (rc == MPIX_REDOP_SUCCESS)
        rc = hip_err(mpix::launch_equal(kin, kio, n, s));
    if (rc == MPIX_REDOP_SUCCESS && io_host)
        rc = hip_err(hipMemcpyAsync(io, kio, 8, hipMemcpyDeviceToHost, s));
    int rc2 = wait_stream(d, s);
    return rc ? rc : rc2;
}

// Small pageable operand(s): memcpy into the pinned bounce buffer, one
// zero-copy kernel over it, memcpy the result back (a staged 1-element call
// costs ~42 us in three pageable hipMemcpy calls).  Returns -1 when the bounce buffer cannot be had (caller stages).
int bounced(const void *in, void *io, uint64_t count, uint32_t it, uint64_t ext, uint32_t op,
            bool in_host, bool io_host, int dev)
{
    DevState *d = dev_state(dev);
    if (!d)
        return MPIX_REDOP_ERR_OTHER;
    size_t bytes = (size_t) (count * ext);
    if (!d->bounce) {
        void *h = nullptr, *hd = nullptr;
        size_t half = (g_bounce_bytes + 255) & ~(size_t) 255;
        if (hipHostMalloc(&h, 2 * half, hipHostMallocDefault) != hipSuccess)
            return -1;
        if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) {
            (void) hipHostFree(h);
            return -1;
        }
        d->bounce = (char *) h;
        d->bounce_dev = (char *) hd;
        d->bounce_half = half;
    }
    if (bytes > d->bounce_half)
        return -1;
    const void *kin = in;
    void *kio = io;
    if (in_host) {
        memcpy(d->bounce, in, bytes);
        kin = d->bounce_dev;
    }
    if (io_host) {
        memcpy(d->bounce + d->bounce_half, io, bytes);
        kio = d->bounce_dev + d->bounce_half;
    }
    int rc = run_sync(d, kin, kio, count, it, ext, op, true);
    if (rc == MPIX_REDOP_SUCCESS && io_host)
        memcpy(io, d->bounce + d->bounce_half, bytes);
    return rc;
}

// Host workers for one pageable call: the configured count, at most one per
// CPU this process may run on (more would only take turns on the same cores).
int worker_count(int nthreads)
{
    int w = nthreads < 1 ? 1 : nthreads;
    cpu_set_t mine;
    if (sched_getaffinity(0, sizeof mine, &mine) == 0) {
        const int cpus = CPU_COUNT(&mine);
        if (cpus >= 1 && w > cpus)
            w = cpus;
    }
    return w;
}

// Large pageable operand(s): W host workers take chunks k = w, w + W, ...; per
// chunk a worker memcpys the pageable operand(s) into its pinned slot, runs one
// zero-copy kernel over the slot's device mapping on its own stream (a pinned
// or device operand is used in place), waits for it and memcpys the result
// back.  The workers' host copies overlap each other's PCIe transfers, where
// hipMemcpyAsync from pageable memory serialises through the runtime's own
// bounce.  Each element is combined exactly once, by the same kernel, so the
// bits equal every other path's.  Returns -1 when the slots cannot be had
// (caller stages).
// Copy into a pinned buffer the GPU is about to read over PCIe.  With plain
// stores the lines sit dirty in the CPU caches and every PCIe read of them is
// a snoop hit; non-temporal stores send them to DRAM (glibc's memcpy switches
// to those only above its own, L3-sized threshold, above our chunk size).
// MPIX_REDOP_PAGEABLE_NT=0 uses memcpy.
std::atomic<int> g_pipe_nt{-1};     // -1: not decided yet
__attribute__((target("avx2"))) static void copy_nt_avx2(char *dst, const char *src, size_t n)
{
    size_t head = (32 - ((uintptr_t) dst & 31)) & 31;
    if (head > n)
        head = n;
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *) (src + i));
        __m256i b = _mm256_loadu_si256((const __m256i *) (src + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *) (src + i + 64));
        __m256i d = _mm256_loadu_si256((const __m256i *) (src + i + 96));
        _mm256_stream_si256((__m256i *) (dst + i), a);
        _mm256_stream_si256((__m256i *) (dst + i + 32), b);
        _mm256_stream_si256((__m256i *) (dst + i + 64), c);
        _mm256_stream_si256((__m256i *) (dst + i + 96), d);
    }
    _mm_sfence();
    memcpy(dst + i, src + i, n - i);
}

void copy_to_pinned(char *dst, const char *src, size_t n)
{
    int nt = g_pipe_nt.load(std::memory_order_relaxed);
    if (nt < 0) {
        const char *e = getenv("MPIX_REDOP_PAGEABLE_NT");
        nt = (e ? atoi(e) != 0 : true) && __builtin_cpu_supports("avx2");
        g_pipe_nt.store(nt);
    }
    if (nt)
        copy_nt_avx2(dst, src, n);
    else
        memcpy(dst, src, n);
}

struct PipeTrace {
    int64_t *ns;        // 5 per chunk, or nullptr
    std::chrono::steady_clock::time_point t0;
};
inline void pipe_mark(PipeTrace *t, int, uint64_t k, int what)
{
    if (t->ns)
        t->ns[k * 5 + (uint64_t) what] = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                             std::chrono::steady_clock::now() - t->t0).count();
}

// CPUs of the GPU's NUMA node (sysfs local_cpulist of its PCI function),
// intersected with this process's affinity; or an explicit "a-b,c" list
std::vector<int> parse_cpulist(const char *txt)
{
    std::vector<int> out;
    for (const char *p = txt; *p;) {
        char *e;
        long a = strtol(p, &e, 10);
        if (e == p)
            break;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b && c < 4096; ++c)
            out.push_back((int) c);
        while (*p == ',' || *p == ' ' || *p == '\n')
            ++p;
    }
    return out;
}

std::vector<int> worker_cpus(int dev)
{
    std::vector<int> want;
    const std::string mode = g_pipe_affinity;
    if (mode == "gpu") {
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) == hipSuccess) {
            for (char *q = bus; *q; ++q)
                *q = (char) tolower(*q);
            std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
            if (FILE *f = fopen(path.c_str(), "r")) {
                char line[4096] = {0};
                if (fgets(line, sizeof line, f))
                    want = parse_cpulist(line);
                fclose(f);
            }
        }
        (void) hipGetLastError();
    } else if (mode != "none" && !mode.empty()) {
        want = parse_cpulist(mode.c_str());
    }
    cpu_set_t mine;
    std::vector<int> out;
    if (want.empty() || sched_getaffinity(0, sizeof mine, &mine) != 0)
        return out;
    for (int c : want)
        if (c < CPU_SETSIZE && CPU_ISSET(c, &mine))
            out.push_back(c);
    return out;
}

// Large pageable operand(s): W host workers take chunks k = w, w + W, ...; per
// chunk a worker memcpys the pageable operand(s) into a pinned buffer of its
// own, runs one zero-copy kernel over the buffer's device mapping on its own
// stream (a pinned or device operand is used in place) and memcpys the result
// back once that kernel is done.  Double-buffered (default), a worker copies
// chunk k + W into its second buffer while chunk k's kernel runs.  The
// workers' host copies overlap each other's PCIe transfers, where
// hipMemcpyAsync from pageable memory serialises through the runtime's own
// bounce.  Each element is combined exactly once, by the same kernel, so the
// bits equal every other path's.  Returns -1 when the buffers cannot be had
// (caller stages).
int pipelined(const void *in, void *io, uint64_t count, uint32_t it, uint64_t ext, uint32_t op,
              bool in_pg, bool io_pg, int dev, int nthreads)
{
    if (dev < 0 || dev >= kMaxDev)
        return -1;
    PipeSet &P = g_pipes[dev];
    std::unique_lock<std::mutex> busy(P.mu, std::try_to_lock);
    if (!busy.owns_lock())
        return -1;      // another thread is using the set: stage instead
    const size_t half = (g_pipe_chunk.load() + 255) & ~(size_t) 255;
    const int nbuf = g_pipe_db.load() ? 2 : 1;
    bool ready = P.half >= half && P.nbuf >= nbuf;
    for (int w = 0; ready && w < nthreads; ++w)
        ready = P.slot[w].host != nullptr;
    if (!ready) {
        // (re)allocate every worker's buffers at the current chunk size
        for (PipeSlot &sl : P.slot) {
            if (sl.s)
                (void) hipStreamSynchronize(sl.s);
            if (sl.host)
                (void) hipHostFree(sl.host);
            sl.host = sl.dev = nullptr;
        }
        P.half = 0;
        P.nbuf = 0;
        for (int w = 0; w < nthreads; ++w) {
            PipeSlot &sl = P.slot[w];
            if (!sl.s && hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess)
                return -1;
            for (hipEvent_t &e : sl.ev)
                if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                    return -1;
            void *h = nullptr, *hd = nullptr;
            if (hipHostMalloc(&h, 2 * half * (size_t) nbuf, hipHostMallocDefault) != hipSuccess)
                return -1;
            if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) {
                (void) hipHostFree(h);
                return -1;
            }
            sl.host = (char *) h;
            sl.dev = (char *) hd;
        }
        P.half = half;
        P.nbuf = nbuf;
    }
    if (!P.cpus_known) {
        P.cpus = worker_cpus(dev);
        P.cpus_known = true;
    }
    uint64_t chunk = half / ext;
    if (chunk == 0)
        return -1;
    const uint64_t nchunks = (count + chunk - 1) / chunk;
    const int W = (int) std::min<uint64_t>((uint64_t) worker_count(nthreads), nchunks);
    std::atomic<int> err{MPIX_REDOP_SUCCESS};
    // MPIX_REDOP_PIPE_TRACE=1: per chunk the host times (ns from the call's
    // start) of copy-in start / end, wait start / end, copy-out end, printed
    // as one JSON line to stderr (tools/pageable_probe.py reads them)
    static const bool trace_on = getenv("MPIX_REDOP_PIPE_TRACE") != nullptr;
    std::vector<int64_t> trace_buf(trace_on ? nchunks * 5 : 0, -1);
    PipeTrace trv{trace_on ? trace_buf.data() : nullptr, std::chrono::steady_clock::now()};
    PipeTrace *tr = &trv;
    auto fail = [&](int rc) {
        int z = MPIX_REDOP_SUCCESS;
        err.compare_exchange_strong(z, rc);
    };
    auto work = [&](int w) {
        PipeSlot &sl = P.slot[w];
        if (hipSetDevice(dev) != hipSuccess) {
            fail(MPIX_REDOP_ERR_OTHER);
            return;
        }
        char *hbuf[2] = {sl.host, sl.host + 2 * half};
        char *dbuf[2] = {sl.dev, sl.dev + 2 * half};
        // buffer b: copy chunk k's pageable operand(s) in, enqueue its kernel
        auto start = [&](uint64_t k, int b) -> int {
            const uint64_t off = k * chunk, n = std::min(chunk, count - off);
            const size_t bytes = (size_t) (n * ext);
            pipe_mark(tr, w, k, 0);
            if (in_pg)
                copy_to_pinned(hbuf[b], (const char *) in + off * ext, bytes);
            if (io_pg)
                copy_to_pinned(hbuf[b] + half, (char *) io + off * ext, bytes);
            pipe_mark(tr, w, k, 1);
            const void *kin = in_pg ? (const void *) dbuf[b] : (const char *) in + off * ext;
            void *kio = io_pg ? (void *) (dbuf[b] + half) : (char *) io + off * ext;
            int rc = enqueue(kin, kio, n, it, ext, op, sl.s, nullptr, nullptr, 0, nullptr, true);
            return rc ? rc : hip_err(hipEventRecord(sl.ev[b], sl.s));
        };
        // chunk k's kernel done: its result back to the pageable inout
        auto finish = [&](uint64_t k, int b) -> int {
            pipe_mark(tr, w, k, 2);
            int rc = hip_err(hipEventSynchronize(sl.ev[b]));
            pipe_mark(tr, w, k, 3);
            if (rc == MPIX_REDOP_SUCCESS && io_pg) {
                const uint64_t off = k * chunk, n = std::min(chunk, count - off);
                memcpy((char *) io + off * ext, hbuf[b] + half, (size_t) (n * ext));
            }
            pipe_mark(tr, w, k, 4);
            return rc;
        };
        uint64_t k = (uint64_t) w;
        int b = 0, rc = k < nchunks ? start(k, b) : MPIX_REDOP_SUCCESS;
        for (; k < nchunks && rc == MPIX_REDOP_SUCCESS && err.load() == MPIX_REDOP_SUCCESS;
             k += (uint64_t) W) {
            const uint64_t kn = k + (uint64_t) W;
            if (nbuf == 2) {
                if (kn < nchunks)
                    rc = start(kn, b ^ 1);          // overlaps chunk k's kernel
                int rc2 = finish(k, b);
                rc = rc ? rc : rc2;
                b ^= 1;
            } else {
                rc = finish(k, b);
                if (rc == MPIX_REDOP_SUCCESS && kn < nchunks)
                    rc = start(kn, b);
            }
        }
        // no kernel of this worker is left reading its buffers when the call
        // returns, also when another worker's failure ended the loop early
        (void) hipStreamSynchronize(sl.s);
        if (rc != MPIX_REDOP_SUCCESS)
            fail(rc);
    };
    std::vector<std::thread> pool;
    pool.reserve(W > 0 ? W - 1 : 0);
    for (int w = 1; w < W; ++w)
        pool.emplace_back([&, w]() {
            if (!P.cpus.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(P.cpus[(size_t) w % P.cpus.size()], &set);
                (void) pthread_setaffinity_np(pthread_self(), sizeof set, &set);
            }
            work(w);
        });
    work(0);        // the caller is worker 0 (its affinity is its own)
    for (std::thread &t : pool)
        t.join();
    if (trace_on) {
        fprintf(stderr, "{\"pipe_trace\": {\"W\": %d, \"chunk\": %zu, \"nbuf\": %d, \"ns\": [", W,
                half, nbuf);
        for (uint64_t i = 0; i < nchunks * 5; ++i)
            fprintf(stderr, "%s%lld", i ? "," : "", (long long) trace_buf[i]);
        fprintf(stderr, "]}}\n");
    }
    return err.load();
}

// Barrier of the wave workers (sense reversal).  A waiter spins with `pause`
// for up to kSpinNs, then sleeps on a futex on the generation word until the
// last worker arrives and wakes it.  Not a yield loop: a yielding waiter on a
// CPU shared with other runnable tasks can be left off it for a whole
// scheduler slice, and every step waits for the last worker to leave -- one
// such stall took a 256 MiB call from 12.6 to 21 ms
// (profiles/r04_pageable_swing.json, the slowest trace's step 7).  Not a long
// spin either: with fewer cores than workers, spinning waiters
// would keep the worker they wait for off the core.  The steps' own imbalance
// is well under the spin window, so a balanced wave never sleeps.
struct SpinBarrier {
    static constexpr int64_t kSpinNs = 200000;
    std::atomic<int> left;
    std::atomic<int> gen{0};
    std::atomic<int> sleepers{0};
    const int n;
    explicit SpinBarrier(int n_) : left(n_), n(n_) {}
    void wait()
    {
        const int g = gen.load();
        if (left.fetch_sub(1) == 1) {
            left.store(n);
            gen.fetch_add(1);           // seq_cst: ordered before the sleepers check
            if (sleepers.load() > 0)
                syscall(SYS_futex, reinterpret_cast<int *>(&gen), FUTEX_WAKE_PRIVATE, INT32_MAX,
                        nullptr, nullptr, 0);
            return;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spins = 1; gen.load(std::memory_order_acquire) == g; ++spins) {
            _mm_pause();
            if ((spins & 0xff) == 0 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(kSpinNs))
                break;
        }
        if (gen.load() != g)
            return;
        sleepers.fetch_add(1);          // seq_cst: the releaser sees it, or we see its gen
        while (gen.load() == g)
            syscall(SYS_futex, reinterpret_cast<int *>(&gen), FUTEX_WAIT_PRIVATE, g, nullptr,
                    nullptr, 0);
        sleepers.fetch_sub(1);
    }
};

// Wave mode (see g_pipe_wave).  Step s: the caller launches the kernel of
// chunk s - 1 (its copy-in finished in step s - 1); every worker copies its
// slice of chunk s in and, once chunk s - 2's kernel is done, its slice of
// chunk s - 2 out; then all meet.  Buffer s % 3 held chunk s - 3, whose
// copy-out ended in step s - 1.  Same kernel per element, same bits.
// Returns -1 when the buffers cannot be had (caller stages).
int waved(const void *in, void *io, uint64_t count, uint32_t it, uint64_t ext, uint32_t op,
          bool in_pg, bool io_pg, int dev, int nthreads)
{
    if (dev < 0 || dev >= kMaxDev)
        return -1;
    PipeSet &P = g_pipes[dev];
    std::unique_lock<std::mutex> busy(P.mu, std::try_to_lock);
    if (!busy.owns_lock())
        return -1;
    const size_t half = (g_pipe_chunk.load() + 255) & ~(size_t) 255;
    if (P.ring_half < half) {
        if (P.ring_s)
            (void) hipStreamSynchronize(P.ring_s);
        if (P.ring)
            (void) hipHostFree(P.ring);
        P.ring = P.ring_dev = nullptr;
        P.ring_half = 0;
        if (!P.ring_s && hipStreamCreateWithFlags(&P.ring_s, hipStreamNonBlocking) != hipSuccess)
            return -1;
        for (hipEvent_t &e : P.ring_ev)
            if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return -1;
        void *h = nullptr, *hd = nullptr;
        if (hipHostMalloc(&h, 3 * 2 * half, hipHostMallocDefault) != hipSuccess)
            return -1;
        if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) {
            (void) hipHostFree(h);
            return -1;
        }
        P.ring = (char *) h;
        P.ring_dev = (char *) hd;
        P.ring_half = half;
    }
    if (!P.cpus_known) {
        P.cpus = worker_cpus(dev);
        P.cpus_known = true;
    }
    const uint64_t chunk = half / ext;
    if (chunk == 0)
        return -1;
    // chunk sizes ramp up (chunk/8, /4, /2) so the first kernel starts after a
    // short copy-in, and down again at the end so the last copy-out is short;
    // full chunks in between.  Offsets and counts in elements.
    std::vector<std::pair<uint64_t, uint64_t>> chunks;
    {
        uint64_t off = 0;
        for (int r = 3; r >= 1 && off < count; --r) {
            const uint64_t c = std::max<uint64_t>(chunk >> r, 1);
            const uint64_t m = std::min(c, count - off);
            chunks.emplace_back(off, m);
            off += m;
        }
        const uint64_t tail_split = chunk;      // the last full chunk's worth goes in halves
        while (count - off > chunk + tail_split) {
            chunks.emplace_back(off, chunk);
            off += chunk;
        }
        for (int r = 1; off < count; r = r < 3 ? r + 1 : 3) {
            const uint64_t c = std::max<uint64_t>(chunk >> r, 1);
            const uint64_t m = (count - off <= c || r == 3) ? std::min(count - off, chunk) : c;
            chunks.emplace_back(off, m);
            off += m;
        }
    }
    const int64_t n = (int64_t) chunks.size();
    const int W = worker_count(nthreads);
    SpinBarrier bar(W);
    // MPIX_REDOP_PIPE_TRACE=1: per step and worker the host times (ns from the
    // call's start) at which the kernel launch (worker 0), the copy-in, the
    // wait for the kernel of chunk st - 2, its copy-out and the step's barrier
    // ended, and the CPU each worker started on -- one JSON line to stderr
    // (tools/pageable_swing.py reads it)
    static const bool trace_on = getenv("MPIX_REDOP_PIPE_TRACE") != nullptr;
    std::vector<int64_t> trace((size_t) (trace_on ? (n + 2) * W * 5 : 0), -1);
    std::vector<int> trace_cpu((size_t) (trace_on ? W : 0), -1);
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](int64_t st, int w, int what) {
        if (trace_on)
            trace[((size_t) st * (size_t) W + (size_t) w) * 5 + (size_t) what] =
                std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now() - t0).count();
    };
    std::atomic<int> err{MPIX_REDOP_SUCCESS};
    auto fail = [&](int rc) {
        int z = MPIX_REDOP_SUCCESS;
        err.compare_exchange_strong(z, rc);
    };
    auto span = [&](int64_t k, uint64_t *off, uint64_t *cnt) {
        *off = chunks[(size_t) k].first;
        *cnt = chunks[(size_t) k].second;
    };
    // worker w's slice of a chunk of `bytes`: 4 KiB-aligned parts
    auto slice = [&](int w, size_t bytes, size_t *lo, size_t *len) {
        size_t per = ((bytes + (size_t) W - 1) / (size_t) W + 4095) & ~(size_t) 4095;
        *lo = std::min(bytes, per * (size_t) w);
        *len = std::min(bytes - *lo, per);
    };
    auto work = [&](int w) {
        if (trace_on)
            trace_cpu[(size_t) w] = sched_getcpu();
        if (hipSetDevice(dev) != hipSuccess) {
            fail(MPIX_REDOP_ERR_OTHER);
        }
        for (int64_t st = 0; st <= n + 1; ++st) {
            if (w == 0 && st >= 1 && st - 1 < n && err.load() == MPIX_REDOP_SUCCESS) {
                uint64_t off, cnt;
                span(st - 1, &off, &cnt);
                const int b = (int) ((st - 1) % 3);
                char *d = P.ring_dev + (size_t) b * 2 * half;
                const void *kin = in_pg ? (const void *) d : (const char *) in + off * ext;
                void *kio = io_pg ? (void *) (d + half) : (char *) io + off * ext;
                // one stream for all chunks: kernels of consecutive chunks on
                // three streams, overlapping each other's ramp, measured 25 %
                // slower (57.5 vs 46.1 ms per 1 GiB; zero-copy kernels
                // running together get in each other's way).  The kernel
                // writes the page-locked buffer itself: a zero-copy kernel
                // that only reads host memory pays less at its end (~0.03 vs
                // ~0.12 ms, profiles/r03_zero_copy_split.json), but returning
                // the result from HBM with a copy engine while the next kernel
                // reads took 56 ms per GiB against 44.6
                // (profiles/r03_pageable_split_rejected.jsonl): the copy
                // engine and the CUs' PCIe reads share the link badly, as the
                // SDMA-only duplex pattern does (56 ms, bench.py pcie)
                int rc = enqueue(kin, kio, cnt, it, ext, op, P.ring_s, nullptr, nullptr, 0, nullptr,
                                 true);
                if (rc == MPIX_REDOP_SUCCESS)
                    rc = hip_err(hipEventRecord(P.ring_ev[b], P.ring_s));
                if (rc)
                    fail(rc);
                mark(st, w, 0);
            }
            if (st < n && err.load() == MPIX_REDOP_SUCCESS) {       // copy chunk st in
                uint64_t off, cnt;
                span(st, &off, &cnt);
                char *h = P.ring + (size_t) (st % 3) * 2 * half;
                size_t lo, len;
                slice(w, (size_t) (cnt * ext), &lo, &len);
                if (len && in_pg)
                    copy_to_pinned(h + lo, (const char *) in + off * ext + lo, len);
                if (len && io_pg)
                    copy_to_pinned(h + half + lo, (const char *) io + off * ext + lo, len);
                mark(st, w, 1);
            }
            if (st >= 2 && st - 2 < n && err.load() == MPIX_REDOP_SUCCESS) {   // chunk st-2 out
                const int b = (int) ((st - 2) % 3);
                int rc = hip_err(hipEventSynchronize(P.ring_ev[b]));
                mark(st, w, 2);
                if (rc)
                    fail(rc);
                else if (io_pg) {
                    uint64_t off, cnt;
                    span(st - 2, &off, &cnt);
                    size_t lo, len;
                    slice(w, (size_t) (cnt * ext), &lo, &len);
                    if (len)
                        memcpy((char *) io + off * ext + lo, P.ring + (size_t) b * 2 * half + half + lo,
                               len);
                }
                mark(st, w, 3);
            }
            bar.wait();
            mark(st, w, 4);
        }
    };
    std::vector<std::thread> pool;
    pool.reserve((size_t) W - 1);
    for (int w = 1; w < W; ++w)
        pool.emplace_back([&, w]() {
            if (!P.cpus.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(P.cpus[(size_t) w % P.cpus.size()], &set);
                (void) pthread_setaffinity_np(pthread_self(), sizeof set, &set);
            }
            work(w);
        });
    work(0);
    for (std::thread &t : pool)
        t.join();
    (void) hipStreamSynchronize(P.ring_s);      // nothing left reading the buffers
    if (trace_on) {
        fprintf(stderr, "{\"wave_trace\": {\"W\": %d, \"ext\": %llu, \"chunks\": [", W,
                (unsigned long long) ext);
        for (int64_t k = 0; k < n; ++k)
            fprintf(stderr, "%s%llu", k ? "," : "", (unsigned long long) chunks[(size_t) k].second);
        fprintf(stderr, "], \"cpus\": [");
        for (int w = 0; w < W; ++w)
            fprintf(stderr, "%s%d", w ? "," : "", trace_cpu[(size_t) w]);
        fprintf(stderr, "], \"ns\": [");
        for (size_t i = 0; i < trace.size(); ++i)
            fprintf(stderr, "%s%lld", i ? "," : "", (long long) trace[i]);
        fprintf(stderr, "]}}\n");
    }
    return err.load();
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev)
            (void) hipSetDevice(dev);
        else
            prev = -1;
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void) hipSetDevice(prev);
    }
};

// ------------------------------------------- split combiners' fixup words
// One buffer per (device, stream) for the words k_contig32 writes for a split
// combiner (redop_kernels.h is_split): stream order serialises its users on
// one stream, and no two streams share one.
struct FixupBuf {
    int dev;
    uintptr_t stream;
    void *ptr;
    size_t bytes;
};
std::mutex g_fixup_mu;
std::vector<FixupBuf> g_fixup;

void free_fixup_buffers()
{
    std::lock_guard<std::mutex> l(g_fixup_mu);
    for (FixupBuf &f : g_fixup) {
        DeviceGuard g(f.dev);
        (void) hipStreamSynchronize((hipStream_t) f.stream);
        (void) hipFree(f.ptr);
    }
    g_fixup.clear();
    (void) hipGetLastError();
}

// ------------------------------------------- peer access between devices
// A kernel on device `dev` may dereference another device's hipMalloc memory
// only once peer access dev -> owner is enabled.  The reference's HIP backend
// enables it for every device pair at init (yaksuri_hip_init_hooks.c:164-181:
// hipDeviceCanAccessPeer, then hipDeviceEnablePeerAccess, "already enabled"
// tolerated); here each pair is settled at its first use, once per process.
// State per ordered pair: 0 unknown, 1 direct access, 2 impossible (callers
// then copy with hipMemcpyPeerAsync or decline).  MPIX_REDOP_PEER=stage treats
// every pair as impossible (the staging path, testable on any 2-GPU box).
std::atomic<int8_t> g_peer[kMaxDev][kMaxDev];
std::mutex g_peer_mu;

enum PeerState : int8_t { kPeerUnknown = 0, kPeerDirect = 1, kPeerNone = 2, kPeerUnsure = 3 };

// kPeerDirect: kernels on `dev` may read `owner`'s memory; kPeerNone: the
// runtime says they may not (or MPIX_REDOP_PEER=stage); kPeerUnsure: the pair
// cannot even be asked (an owner index this process does not see, e.g. memory
// mapped from another process's GPU under a restricted HIP_VISIBLE_DEVICES) --
// used as it is, as the IPC mapping that produced it allows
PeerState peer_state(int dev, int owner)
{
    if (dev == owner)
        return kPeerDirect;
    int ndev = 0;
    if (dev < 0 || owner < 0 || dev >= kMaxDev || owner >= kMaxDev ||
        hipGetDeviceCount(&ndev) != hipSuccess || dev >= ndev || owner >= ndev) {
        (void) hipGetLastError();
        return kPeerUnsure;
    }
    int8_t st = g_peer[dev][owner].load(std::memory_order_acquire);
    if (st)
        return (PeerState) st;
    std::lock_guard<std::mutex> l(g_peer_mu);
    st = g_peer[dev][owner].load(std::memory_order_acquire);
    if (st)
        return (PeerState) st;
    const char *force = getenv("MPIX_REDOP_PEER");
    PeerState r;
    int can = 0;
    if (force && strcmp(force, "stage") == 0) {
        r = kPeerNone;
    } else if (hipDeviceCanAccessPeer(&can, dev, owner) != hipSuccess) {
        r = kPeerUnsure;
    } else if (!can) {
        r = kPeerNone;
    } else {
        DeviceGuard g(dev);
        hipError_t e = hipDeviceEnablePeerAccess(owner, 0);
        r = (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) ? kPeerDirect : kPeerNone;
    }
    (void) hipGetLastError();       // "already enabled" is sticky otherwise
    g_peer[dev][owner].store((int8_t) r, std::memory_order_release);
    return r;
}

bool peer_access(int dev, int owner) { return peer_state(dev, owner) == kPeerDirect; }

// The device a stream's kernels run on (the null stream: the current one).
int stream_device(hipStream_t s)
{
    int dev = 0;
    if (s) {
        hipDevice_t d;
        if (hipStreamGetDevice(s, &d) == hipSuccess)
            return (int) d;
        (void) hipGetLastError();
    }
    (void) hipGetDevice(&dev);
    return dev;
}

// The stream-ordered entry points take pointers a kernel on `s` can
// dereference: a pageable host pointer would fault the GPU and is refused with
// MPI_ERR_BUFFER; pinned host memory is translated to its device mapping; and
// another device's memory is reachable only with peer access (enabled here at
// first use), else refused too.  `launch` caches the stream's device (-2 = not
// looked up yet).
bool reachable(const void *p, hipStream_t s, int *launch, const void **devptr,
               bool *pinned = nullptr)
{
    int owner = -1;
    const Where w = classify(p, &owner, devptr);
    if (w == Where::Pageable)
        return false;
    if (w != Where::Device) {
        if (pinned)
            *pinned = true;     // page-locked host memory, read through its mapping
        return true;
    }
    if (*launch == -2)
        *launch = stream_device(s);
    return peer_state(*launch, owner) != kPeerNone;
}

// ------------------------------------------- derived targets as runs
// One uop call of typerep_op_fallback: `n` elements at extent stride from
// byte offset `off` of inout (may be negative: lb < 0), combined with the
// next n elements of the packed source.
struct Run {
    int64_t off, n;
};

// Enqueue a list of runs on `s`.  Runs are split by their offset modulo the
// extent so each launch indexes inout in whole elements from one base
// (inout + residue); the source offset table keeps the packed source in the
// original run order.  Residues must keep the 4-byte (2-byte for 2-byte
// types) alignment the element loads need.
int enqueue_runs(const void *inbuf, void *inoutbuf, const std::vector<Run> &runs, uint32_t dt,
                 uint32_t op, hipStream_t s)
{
    uint32_t it;
    uint64_t ext;
    int rc = validate(inbuf, inoutbuf, 0, dt, op, &it, &ext);
    if (rc != MPIX_REDOP_SUCCESS)
        return rc;
    int64_t total = 0;
    for (const Run &r : runs)
        total += r.n;
    if (total == 0)
        return MPIX_REDOP_SUCCESS;
    if (!inbuf || !inoutbuf || inbuf == (const void *) -1 || inoutbuf == (void *) -1)
        return MPIX_REDOP_ERR_BUFFER;
    {
        const void *pin, *pio;
        int launch = -2;
        if (!reachable(inbuf, s, &launch, &pin) || !reachable(inoutbuf, s, &launch, &pio))
            return MPIX_REDOP_ERR_BUFFER;
        inbuf = pin;
        inoutbuf = (void *) pio;
    }
    const int64_t e = (int64_t) ext, align = e < 4 ? e : 4;
    for (const Run &r : runs)
        if ((((r.off % e) + e) % e) % align)
            return MPIX_REDOP_ERR_ARG;
    uint32_t opi = op & 0xf;
    if (opi == 14)
        return MPIX_REDOP_SUCCESS;
    if (opi == 13) {    // REPLACE: one typemap copy per run
        int64_t src = 0;
        for (size_t k = 0; k < runs.size() && rc == MPIX_REDOP_SUCCESS; ++k) {
            rc = replace_rows((char *) inoutbuf + runs[k].off, ext,
                              (const char *) inbuf + src * e, ext, (uint64_t) runs[k].n, it, ext, s);
            src += runs[k].n;
        }
        return rc;
    }
    const Entry *en = gpu_entry(opi, it);
    if (!en)
        return MPIX_REDOP_ERR_TYPE;
    // group by residue; per group the table is [seg_off n][prefix n+1][src_off n]
    std::vector<int64_t> resid;
    std::vector<std::vector<size_t>> groups;
    for (size_t k = 0; k < runs.size(); ++k) {
        if (runs[k].n == 0)
            continue;
        int64_t r = ((runs[k].off % e) + e) % e;
        size_t g = 0;
        while (g < resid.size() && resid[g] != r)
            ++g;
        if (g == resid.size()) {
            resid.push_back(r);
            groups.emplace_back();
        }
        groups[g].push_back(k);
    }
    std::vector<int64_t> src_of(runs.size());
    {
        int64_t src = 0;
        for (size_t k = 0; k < runs.size(); ++k) {
            src_of[k] = src;
            src += runs[k].n;
        }
    }
    size_t need = 0;
    for (const auto &g : groups)
        need += 3 * g.size() + 1;
    std::vector<int64_t> tab(need);
    std::vector<size_t> base(groups.size());
    std::vector<int64_t> gtotal(groups.size());
    size_t at = 0;
    for (size_t g = 0; g < groups.size(); ++g) {
        const size_t n = groups[g].size();
        base[g] = at;
        int64_t pre = 0;
        for (size_t q = 0; q < n; ++q) {
            const Run &r = runs[groups[g][q]];
            tab[at + q] = (r.off - resid[g]) / e;
            tab[at + n + q] = pre;
            tab[at + 2 * n + 1 + q] = src_of[groups[g][q]];
            pre += r.n;
        }
        tab[at + 2 * n] = pre;
        gtotal[g] = pre;
        at += 3 * n + 1;
    }
    int dev = 0;
    (void) hipGetDevice(&dev);
    DevState *d = dev_state(dev);
    if (!d)
        return MPIX_REDOP_ERR_OTHER;
    DevState::IovSlot &sl = d->iov[d->iov_next++ & 1];
    if (!sl.done && hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess)
        return MPIX_REDOP_ERR_OTHER;
    // the slot's previous table may still be read by kernels queued on any
    // stream (this thread may have used another one then): wait for them
    rc = hip_err(hipEventSynchronize(sl.done));
    if (rc != MPIX_REDOP_SUCCESS)
        return rc;
    if (sl.cap < need) {
        if (sl.tab)
            (void) hipFree(sl.tab);
        if (sl.host)
            (void) hipHostFree(sl.host);
        sl.tab = nullptr;
        sl.host = nullptr;
        sl.cap = 0;
        if (hipMalloc((void **) &sl.tab, need * sizeof(int64_t)) != hipSuccess)
            return MPIX_REDOP_ERR_OTHER;
        if (hipHostMalloc((void **) &sl.host, need * sizeof(int64_t), hipHostMallocDefault) !=
            hipSuccess)
            return MPIX_REDOP_ERR_OTHER;
        sl.cap = need;
    }
    // the table goes through the pinned copy, so the upload is a true async
    // copy on s (no wait on the caller's stream); both copies are free for
    // reuse once sl.done, recorded after the launches below, has fired
    memcpy(sl.host, tab.data(), need * sizeof(int64_t));
    rc = hip_err(hipMemcpyAsync(sl.tab, sl.host, need * sizeof(int64_t), hipMemcpyHostToDevice, s));
    for (size_t g = 0; g < groups.size() && rc == MPIX_REDOP_SUCCESS; ++g) {
        const int64_t n = (int64_t) groups[g].size();
        const int64_t *t = sl.tab + base[g];
        rc = hip_err(en->iov(inbuf, (char *) inoutbuf + resid[g], t, t + n, t + 2 * n + 1, n,
                             (uint64_t) gtotal[g], params(), launch_cfg(), s));
    }
    int rc2 = hip_err(hipEventRecord(sl.done, s));
    return rc ? rc : rc2;
}

}  // namespace

namespace mpix {
uint64_t *fixup_buffer(hipStream_t s, size_t bytes)
{
    int dev = 0;
    if (hipStreamGetDevice(s, &dev) != hipSuccess)
        return nullptr;
    std::lock_guard<std::mutex> l(g_fixup_mu);
    FixupBuf *f = nullptr;
    for (FixupBuf &e : g_fixup)
        if (e.dev == dev && e.stream == (uintptr_t) s)
            f = &e;
    if (!f) {
        g_fixup.push_back(FixupBuf{dev, (uintptr_t) s, nullptr, 0});
        f = &g_fixup.back();
    }
    if (f->bytes < bytes) {
        DeviceGuard g(dev);
        if (f->ptr) {       // enqueued work on this stream may still read the old one
            if (hipStreamSynchronize(s) != hipSuccess)
                return nullptr;
            (void) hipFree(f->ptr);
            f->ptr = nullptr;
            f->bytes = 0;
        }
        size_t want = bytes < ((size_t) 64 << 10) ? (size_t) 64 << 10 : bytes;
        if (hipMalloc(&f->ptr, want) != hipSuccess) {
            (void) hipGetLastError();
            f->ptr = nullptr;
            return nullptr;
        }
        f->bytes = want;
    }
    return static_cast<uint64_t *>(f->ptr);
}
}  // namespace mpix

extern "C" {

int MPIX_Redop_init(void)
{
    launch_cfg();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return set_err(MPIX_REDOP_ERR_OTHER);
    return set_err(dev_state(dev) ? MPIX_REDOP_SUCCESS : MPIX_REDOP_ERR_OTHER);
}

static void free_states(DevState *arr)
{
    for (int i = 0; i < kMaxDev; ++i) {
        DevState &d = arr[i];
        if (!d.init)
            continue;
        DeviceGuard g(i);
        for (int k = 0; k < 2; ++k)
            if (d.s[k])
                (void) hipStreamDestroy(d.s[k]);
        if (d.done)
            (void) hipEventDestroy(d.done);
        if (d.flag)
            (void) hipHostFree((void *) d.flag);
        if (d.flag_ctr)
            (void) hipFree(d.flag_ctr);
        if (d.scratch)
            (void) hipFree(d.scratch);
        for (DevState::IovSlot &sl : d.iov) {
            if (sl.done) {
                (void) hipEventSynchronize(sl.done);
                (void) hipEventDestroy(sl.done);
            }
            if (sl.tab)
                (void) hipFree(sl.tab);
            if (sl.host)
                (void) hipHostFree(sl.host);
        }
        if (d.bounce)
            (void) hipHostFree(d.bounce);
        for (hipEvent_t e : d.tev)
            (void) hipEventDestroy(e);
        d = DevState();
    }
    delete[] arr;
}

int MPIX_Redop_finalize(void)
{
    free_fixup_buffers();
    std::vector<DevState *> pooled;
    {
        std::lock_guard<std::mutex> l(g_pool_mu);
        pooled.swap(*g_pool);
    }
    if (t_dev.arr)
        pooled.push_back(t_dev.arr);
    t_dev.arr = nullptr;
    for (DevState *arr : pooled)
        free_states(arr);
    for (int i = 0; i < kMaxDev; ++i) {     // the process-wide pageable worker slots
        PipeSet &P = g_pipes[i];
        std::lock_guard<std::mutex> l(P.mu);
        if (!P.slot[0].s && !P.slot[0].host && !P.ring && !P.ring_s)
            continue;
        DeviceGuard g(i);
        for (PipeSlot &sl : P.slot) {
            if (sl.s) {
                (void) hipStreamSynchronize(sl.s);
                (void) hipStreamDestroy(sl.s);
            }
            for (hipEvent_t e : sl.ev)
                if (e)
                    (void) hipEventDestroy(e);
            if (sl.host)
                (void) hipHostFree(sl.host);
            sl = PipeSlot();
        }
        P.half = 0;
        P.nbuf = 0;
        if (P.ring_s) {
            (void) hipStreamSynchronize(P.ring_s);
            (void) hipStreamDestroy(P.ring_s);
        }
        for (hipEvent_t &e : P.ring_ev)
            if (e) {
                (void) hipEventDestroy(e);
                e = nullptr;
            }
        if (P.ring)
            (void) hipHostFree(P.ring);
        P.ring = P.ring_dev = nullptr;
        P.ring_half = 0;
        P.ring_s = nullptr;
    }
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Reduce_local_async(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                            MPIX_Datatype datatype, MPIX_Op op, void *stream)
{
    uint32_t it;
    uint64_t ext;
    int rc = validate(inbuf, inoutbuf, count, (uint32_t) datatype, (uint32_t) op, &it, &ext);
    if (rc != MPIX_REDOP_SUCCESS || count == 0)
        return set_err(rc);
    const void *pin, *pio;
    int launch = -2;
    bool zc = false;
    if (!reachable(inbuf, (hipStream_t) stream, &launch, &pin, &zc) ||
        !reachable(inoutbuf, (hipStream_t) stream, &launch, &pio, &zc))
        return set_err(MPIX_REDOP_ERR_BUFFER);
    return set_err(enqueue(pin, (void *) pio, (uint64_t) count, it, ext, (uint32_t) op,
                           (hipStream_t) stream, nullptr, nullptr, 0, nullptr, zc));
}

// Several ready chunks in one launch (include/mpix_redop.h).  Checks first,
// all before any device work: the arguments, then that no triple's target
// overlaps another triple's target or source (the batch runs them in no
// particular order), then that the stream's device can reach every operand.
static_assert(mpix::kMaxBatchSegs == MPIX_BATCH_MAX, "one batch limit");

int MPIX_Reduce_local_batch_async(const void *const *inbufs, void *const *inoutbufs,
                                  const MPIX_Aint *counts, int k, MPIX_Datatype datatype,
                                  MPIX_Op op, void *stream)
{
    if (k < 1 || k > MPIX_BATCH_MAX || !inbufs || !inoutbufs || !counts)
        return set_err(MPIX_REDOP_ERR_ARG);
    uint32_t it = 0;
    uint64_t ext = 0;
    for (int i = 0; i < k; ++i) {
        int rc = validate(inbufs[i], inoutbufs[i], counts[i], (uint32_t) datatype, (uint32_t) op,
                          &it, &ext);
        if (rc != MPIX_REDOP_SUCCESS)
            return set_err(rc);
    }
    for (int i = 0; i < k; ++i) {
        if (!counts[i])
            continue;
        const uint64_t bi = (uint64_t) counts[i] * ext;
        for (int j = 0; j < k; ++j) {
            if (j == i || !counts[j])
                continue;
            const uint64_t bj = (uint64_t) counts[j] * ext;
            const uintptr_t ti = (uintptr_t) inoutbufs[i], tj = (uintptr_t) inoutbufs[j],
                            sj = (uintptr_t) inbufs[j];
            if ((ti < tj + bj && tj < ti + bi) || (ti < sj + bj && sj < ti + bi))
                return set_err(MPIX_REDOP_ERR_BUFFER);
        }
    }
    const uint32_t opi = (uint32_t) op & 0xf;
    const Entry *e = (opi >= 13) ? nullptr : gpu_entry(opi, it);
    if (opi < 13 && !e)
        return set_err(MPIX_REDOP_ERR_TYPE);
    const void *pin[MPIX_BATCH_MAX];
    void *pio[MPIX_BATCH_MAX];
    uint64_t cnt[MPIX_BATCH_MAX];
    bool zc[MPIX_BATCH_MAX];
    int m = 0, launch = -2;
    for (int i = 0; i < k; ++i) {
        if (!counts[i])
            continue;
        const void *a, *b;
        bool pinned = false;
        if (!reachable(inbufs[i], (hipStream_t) stream, &launch, &a, &pinned) ||
            !reachable(inoutbufs[i], (hipStream_t) stream, &launch, &b, &pinned))
            return set_err(MPIX_REDOP_ERR_BUFFER);
        pin[m] = a;
        pio[m] = (void *) b;
        zc[m] = pinned;
        cnt[m++] = (uint64_t) counts[i];
    }
    if (!m)
        return set_err(MPIX_REDOP_SUCCESS);
    // REPLACE / NO_OP / EQUAL, and every triple with a page-locked host
    // operand: a call each -- a kernel reading host memory over PCIe runs the
    // capped, looping zero-copy grid (g_zc_grid), which the
    // batch kernels' one-tile-per-block layout cannot.  The triples are
    // independent (checked above), so their order does not matter.
    int nd = 0;
    for (int i = 0; i < m; ++i) {
        if (!e || zc[i]) {
            int rc = enqueue(pin[i], pio[i], cnt[i], it, ext, (uint32_t) op, (hipStream_t) stream,
                             nullptr, nullptr, 0, nullptr, zc[i]);
            if (rc != MPIX_REDOP_SUCCESS)
                return set_err(rc);
            continue;
        }
        pin[nd] = pin[i];
        pio[nd] = pio[i];
        cnt[nd++] = cnt[i];
    }
    if (!nd)
        return set_err(MPIX_REDOP_SUCCESS);
    return set_err(hip_err(e->batch(pin, pio, cnt, nd, params(), launch_cfg(), (hipStream_t) stream)));
}

int MPIX_Reduce_local(const void *inbuf, void *inoutbuf, MPIX_Aint count, MPIX_Datatype datatype,
                      MPIX_Op op)
{
    uint32_t it;
    uint64_t ext;
    int rc = validate(inbuf, inoutbuf, count, (uint32_t) datatype, (uint32_t) op, &it, &ext);
    if (rc != MPIX_REDOP_SUCCESS || count == 0)
        return set_err(rc);
    uint32_t opi = (uint32_t) op & 0xf;
    if (opi == 15 ? ((it & 0xffffff00u) != U8 || count < 8)
                  : (opi != 13 && opi != 14 && !gpu_entry(opi, it)))
        return set_err(MPIX_REDOP_ERR_TYPE);
    launch_cfg();
    int din = -1, dio = -1, cur = 0;
    (void) hipGetDevice(&cur);
    const void *pin, *pio;
    Where win = classify(inbuf, &din, &pin);
    Where wio = classify(inoutbuf, &dio, &pio);
    bool zc = g_zero_copy.load();
    bool in_stage = win == Where::Pageable || (win == Where::Pinned && !zc);
    bool io_stage = wio == Where::Pageable || (wio == Where::Pinned && !zc);
    int dev = wio == Where::Device ? dio : (win == Where::Device ? din : cur);
    DeviceGuard guard(dev);
    if (win == Where::Device && wio == Where::Device && din != dio &&
        peer_state(dio, din) == kPeerNone)
        // operands on two devices without peer access: the kernel runs where
        // inout lives and `in` is copied over in chunks (hipMemcpyPeerAsync);
        // MPIX_EQUAL's one header covers the whole message: copied whole
        return set_err(opi == 15
                           ? equal_whole(pin, (void *) pio, (uint64_t) count, false, false, dev, din)
                           : staged(pin, (void *) pio, (uint64_t) count, it, ext, (uint32_t) op,
                                    false, false, dev, din));
    bool pageable = win == Where::Pageable || wio == Where::Pageable;
    if (pageable && (uint64_t) count * ext <= g_bounce_bytes) {
        // only pageable operands bounce; pinned ones are used through their mapping
        rc = bounced(win == Where::Pageable ? inbuf : pin,
                     wio == Where::Pageable ? inoutbuf : (void *) pio, (uint64_t) count, it, ext,
                     (uint32_t) op, win == Where::Pageable, wio == Where::Pageable, dev);
        if (rc >= 0)
            return set_err(rc);
    }
    if (opi == 15 && (in_stage || io_stage))
        // MPIX_EQUAL is one comparison over the whole buffer behind one
        // 8-byte header (opequal.c:20-35; MPIR_Reduce_equal: "we can't split
        // the message"), so it is never chunked
        return set_err(equal_whole(in_stage ? inbuf : pin, io_stage ? inoutbuf : (void *) pio,
                                   (uint64_t) count, in_stage, io_stage, dev));
    const int pipe_threads = g_pipe_threads.load();
    const bool wave = g_pipe_wave.load() != 0;
    if (pageable && zc && pipe_threads > 0 &&
        (uint64_t) count * ext >= (wave ? 2 : 2 * (uint64_t) pipe_threads) * g_pipe_chunk.load()) {
        // pageable operands through the workers' pinned slots; a pinned
        // operand is used through its device mapping
        rc = (wave ? waved : pipelined)(win == Where::Pageable ? inbuf : pin,
                                        wio == Where::Pageable ? inoutbuf : (void *) pio,
                                        (uint64_t) count, it, ext, (uint32_t) op,
                                        win == Where::Pageable, wio == Where::Pageable, dev,
                                        pipe_threads);
        if (rc >= 0)
            return set_err(rc);
    }
    if (in_stage || io_stage)
        return set_err(staged(in_stage ? inbuf : pin, io_stage ? inoutbuf : (void *) pio,
                              (uint64_t) count, it, ext, (uint32_t) op, in_stage, io_stage, dev));
    DevState *d = dev_state(dev);
    if (!d)
        return set_err(MPIX_REDOP_ERR_OTHER);
    return set_err(run_sync(d, pin, (void *) pio, (uint64_t) count, it, ext, (uint32_t) op,
                            win == Where::Pinned || wio == Where::Pinned));
}

int MPIX_Reduce_local_vector_async(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                                   MPIX_Aint blocklen, MPIX_Aint stride,
                                   MPIX_Datatype basic_type, MPIX_Op op, void *stream)
{
    if (count < 0 || blocklen < 0)
        return set_err(MPIX_REDOP_ERR_COUNT);
    if (stride < blocklen)
        return set_err(MPIX_REDOP_ERR_ARG);     // overlapping target runs
    uint32_t it;
    uint64_t ext;
    int rc = validate(inbuf, inoutbuf, 0, (uint32_t) basic_type, (uint32_t) op, &it, &ext);
    if (rc != MPIX_REDOP_SUCCESS)
        return set_err(rc);
    uint64_t n = (uint64_t) count * (uint64_t) blocklen;
    if (n == 0)
        return set_err(MPIX_REDOP_SUCCESS);
    if (!inbuf || !inoutbuf || inbuf == (const void *) -1 || inoutbuf == (void *) -1)
        return set_err(MPIX_REDOP_ERR_BUFFER);
    uint64_t span = ((uint64_t) (count - 1) * (uint64_t) stride + (uint64_t) blocklen) * ext;
    uintptr_t x = (uintptr_t) inbuf, y = (uintptr_t) inoutbuf;
    if (x < y + span && y < x + n * ext)
        return set_err(MPIX_REDOP_ERR_BUFFER);
    {
        const void *pin, *pio;
        int launch = -2;
        if (!reachable(inbuf, (hipStream_t) stream, &launch, &pin) ||
            !reachable(inoutbuf, (hipStream_t) stream, &launch, &pio))
            return set_err(MPIX_REDOP_ERR_BUFFER);
        inbuf = pin;
        inoutbuf = (void *) pio;
    }
    uint32_t opi = (uint32_t) op & 0xf;
    if (opi == 14)
        return set_err(MPIX_REDOP_SUCCESS);
    if (opi == 13) {
        PairMap pm;
        if (!padded_pair(it, &pm)) {
            rc = hip_err(hipMemcpy2DAsync(inoutbuf, (size_t) stride * ext, inbuf,
                                          (size_t) blocklen * ext, (size_t) blocklen * ext,
                                          (size_t) count, hipMemcpyDeviceToDevice,
                                          (hipStream_t) stream));
        } else if (blocklen <= count) {     // column k of every block
            for (MPIX_Aint k = 0; k < blocklen && rc == MPIX_REDOP_SUCCESS; ++k)
                rc = replace_rows((char *) inoutbuf + k * ext, (size_t) stride * ext,
                                  (const char *) inbuf + k * ext, (size_t) blocklen * ext,
                                  (uint64_t) count, it, ext, (hipStream_t) stream);
        } else {                            // block by block
            for (MPIX_Aint b = 0; b < count && rc == MPIX_REDOP_SUCCESS; ++b)
                rc = replace_rows((char *) inoutbuf + b * stride * ext, ext,
                                  (const char *) inbuf + b * blocklen * ext, ext,
                                  (uint64_t) blocklen, it, ext, (hipStream_t) stream);
        }
        return set_err(rc);
    }
    const Entry *e = gpu_entry(opi, it);
    if (!e)
        return set_err(MPIX_REDOP_ERR_TYPE);
    return set_err(hip_err(e->vector(inbuf, inoutbuf, (uint64_t) count, (uint64_t) blocklen,
                                     (uint64_t) stride, params(), launch_cfg(),
                                     (hipStream_t) stream)));
}

int MPIX_Reduce_local_vector(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                             MPIX_Aint blocklen, MPIX_Aint stride, MPIX_Datatype basic_type,
                             MPIX_Op op)
{
    int dev = 0;
    const void *dp;
    if (classify(inoutbuf, &dev, &dp) != Where::Device)
        return set_err(MPIX_REDOP_ERR_BUFFER);
    DeviceGuard guard(dev);
    DevState *d = dev_state(dev);
    if (!d)
        return set_err(MPIX_REDOP_ERR_OTHER);
    int rc = MPIX_Reduce_local_vector_async(inbuf, inoutbuf, count, blocklen, stride, basic_type,
                                            op, d->s[0]);
    int rc2 = wait_stream(d, d->s[0]);
    return set_err(rc ? rc : rc2);
}

int MPIX_Reduce_local_iov_async(const void *inbuf, void *inoutbuf, MPIX_Aint nseg,
                                const MPIX_Aint *seg_offsets, const MPIX_Aint *seg_counts,
                                MPIX_Datatype basic_type, MPIX_Op op, void *stream)
{
    if (nseg < 0)
        return set_err(MPIX_REDOP_ERR_COUNT);
    if (nseg > 0 && (!seg_offsets || !seg_counts))
        return set_err(MPIX_REDOP_ERR_BUFFER);
    std::vector<Run> runs;
    runs.reserve((size_t) nseg);
    for (MPIX_Aint s = 0; s < nseg; ++s) {
        if (seg_counts[s] < 0)
            return set_err(MPIX_REDOP_ERR_COUNT);
        runs.push_back(Run{seg_offsets[s], seg_counts[s]});
    }
    return set_err(enqueue_runs(inbuf, inoutbuf, runs, (uint32_t) basic_type, (uint32_t) op,
                                (hipStream_t) stream));
}

int MPIX_Reduce_local_iovec_async(const void *inbuf, void *inoutbuf, MPIX_Aint nseg,
                                  const MPIX_Aint *iov_offsets, const MPIX_Aint *iov_lens,
                                  MPIX_Datatype basic_type, MPIX_Op op, void *stream)
{
    if (nseg < 0)
        return set_err(MPIX_REDOP_ERR_COUNT);
    if (nseg > 0 && (!iov_offsets || !iov_lens))
        return set_err(MPIX_REDOP_ERR_BUFFER);
    uint32_t it = to_internal((uint32_t) basic_type);
    uint64_t ext = extent_of(it), size = size_of(it);
    if (it == kNull || ext == 0)
        return set_err(MPIX_REDOP_ERR_TYPE);
    // typerep_op.c:115-149: segments are gathered until they hold one
    // element's data (pairtypes split by their padding); each call covers
    // curr_len / size elements laid out at extent stride from target_ptr,
    // and a partial element left at the end of a segment starts the next one
    const bool pairtype = size < ext;
    std::vector<Run> runs;
    runs.reserve((size_t) nseg);
    MPIX_Aint curr = 0, target = 0;
    for (MPIX_Aint i = 0; i < nseg; ++i) {
        if (iov_lens[i] < 0)
            return set_err(MPIX_REDOP_ERR_COUNT);
        if (pairtype) {
            if (curr == 0)
                target = iov_offsets[i];
            curr += iov_lens[i];
            if (curr < (MPIX_Aint) size)
                continue;
        } else {
            target = iov_offsets[i];
            curr = iov_lens[i];
        }
        MPIX_Aint n = curr / (MPIX_Aint) size;
        MPIX_Aint data = n * (MPIX_Aint) size;
        runs.push_back(Run{target, n});
        if (pairtype) {
            curr -= data;
            if (curr > 0)
                target = iov_offsets[i] + (iov_lens[i] - curr);
        } else if (curr != data) {
            return set_err(MPIX_REDOP_ERR_ARG);   // the reference's MPIR_Assert (:147)
        }
    }
    return set_err(enqueue_runs(inbuf, inoutbuf, runs, (uint32_t) basic_type, (uint32_t) op,
                                (hipStream_t) stream));
}

int MPIX_Reduce_local_multi_async(const void *const *inbufs, int ninputs, void *inoutbuf,
                                  MPIX_Aint count, MPIX_Datatype datatype, MPIX_Op op,
                                  void *stream)
{
    if (ninputs < 1 || ninputs > mpix::kMaxMultiInputs || !inbufs)
        return set_err(MPIX_REDOP_ERR_ARG);
    uint32_t it;
    uint64_t ext;
    for (int q = 0; q < ninputs; ++q) {
        int rc = validate(inbufs[q], inoutbuf, count, (uint32_t) datatype, (uint32_t) op, &it,
                          &ext);
        if (rc != MPIX_REDOP_SUCCESS)
            return set_err(rc);
    }
    if (count == 0)
        return set_err(MPIX_REDOP_SUCCESS);
    const void *dins[mpix::kMaxMultiInputs];
    const void *pio;
    int launch = -2;
    if (!reachable(inoutbuf, (hipStream_t) stream, &launch, &pio))
        return set_err(MPIX_REDOP_ERR_BUFFER);
    for (int q = 0; q < ninputs; ++q)
        if (!reachable(inbufs[q], (hipStream_t) stream, &launch, &dins[q]))
            return set_err(MPIX_REDOP_ERR_BUFFER);
    inbufs = dins;
    inoutbuf = (void *) pio;
    uint32_t opi = (uint32_t) op & 0xf;
    if (opi == 14)
        return set_err(MPIX_REDOP_SUCCESS);
    if (opi == 13)      // REPLACE k times = copy of the last input
        return set_err(replace_rows(inoutbuf, ext, inbufs[ninputs - 1], ext, (uint64_t) count, it,
                                    ext, (hipStream_t) stream));
    const Entry *e = gpu_entry(opi, it);
    if (!e)
        return set_err(MPIX_REDOP_ERR_TYPE);
    return set_err(hip_err(e->multi(inbufs, ninputs, inoutbuf, (uint64_t) count, params(),
                                    launch_cfg(), (hipStream_t) stream)));
}

int MPIX_Reduce_local_tree_async(const void *const *inbufs, int ninputs, void *outbuf,
                                 MPIX_Aint count, MPIX_Datatype datatype, MPIX_Op op, void *stream)
{
    if (ninputs < 2 || ninputs > mpix::kMaxMultiInputs || (ninputs & (ninputs - 1)) || !inbufs ||
        !inbufs[0])
        return set_err(MPIX_REDOP_ERR_ARG);
    uint32_t it;
    uint64_t ext;
    // outbuf may be one of the slots itself (each lane reads all its slots'
    // elements before it writes that element); any partial overlap is
    // refused.  Slots 1..k-1 may be NULL: absent (the partner passes through).
    for (int q = 0; q < ninputs; ++q) {
        if (!inbufs[q])
            continue;
        const bool same = inbufs[q] == (const void *) outbuf;
        int rc = validate(same ? (const void *) ((const char *) outbuf + 1) : inbufs[q], outbuf,
                          same ? 0 : count, (uint32_t) datatype, (uint32_t) op, &it, &ext);
        if (rc == MPIX_REDOP_SUCCESS && same && count > 0 &&
            (uint64_t) count > ((uint64_t) 1 << 56) / ext)
            rc = MPIX_REDOP_ERR_COUNT;
        if (rc == MPIX_REDOP_SUCCESS && same && count > 0 &&
            (!outbuf || outbuf == (void *) -1))
            rc = MPIX_REDOP_ERR_BUFFER;
        if (rc != MPIX_REDOP_SUCCESS)
            return set_err(rc);
    }
    if (count == 0)
        return set_err(MPIX_REDOP_SUCCESS);
    uint32_t opi = (uint32_t) op & 0xf;
    if (opi == 15)
        return set_err(MPIX_REDOP_ERR_OP);      // EQUAL is never split or folded
    const void *dins[mpix::kMaxMultiInputs];
    const void *pout;
    int launch = -2;
    if (!reachable(outbuf, (hipStream_t) stream, &launch, &pout))
        return set_err(MPIX_REDOP_ERR_BUFFER);
    int last = 0;
    for (int q = 0; q < ninputs; ++q) {
        dins[q] = nullptr;
        if (inbufs[q] && !reachable(inbufs[q], (hipStream_t) stream, &launch, &dins[q]))
            return set_err(MPIX_REDOP_ERR_BUFFER);
        if (inbufs[q])
            last = q;
    }
    if (opi == 13 || opi == 14) {   // REPLACE folds to the last present slot, NO_OP to the first
        const void *src = dins[opi == 13 ? last : 0];
        if (src == pout)
            return set_err(MPIX_REDOP_SUCCESS);
        return set_err(replace_rows((void *) pout, ext, src, ext, (uint64_t) count, it, ext,
                                    (hipStream_t) stream));
    }
    const Entry *e = gpu_entry(opi, it);
    if (!e || !e->tree)
        return set_err(MPIX_REDOP_ERR_TYPE);
    return set_err(hip_err(e->tree(dins, ninputs, (void *) pout, (uint64_t) count, params(),
                                   launch_cfg(), (hipStream_t) stream)));
}

int MPIX_Copy_multi_async(const void *const *srcs, void *const *dsts, const MPIX_Aint *bytes,
                          int n, void *stream)
{
    if (n < 0 || n > mpix::kMaxMultiInputs || (n && (!srcs || !dsts || !bytes)))
        return set_err(MPIX_REDOP_ERR_ARG);
    const void *ds[mpix::kMaxMultiInputs];
    void *dd[mpix::kMaxMultiInputs];
    uint64_t nb[mpix::kMaxMultiInputs];
    int m = 0, launch = -2;
    for (int q = 0; q < n; ++q) {
        if (bytes[q] < 0)
            return set_err(MPIX_REDOP_ERR_COUNT);
        if (bytes[q] == 0)
            continue;
        if (!srcs[q] || !dsts[q] || overlaps(srcs[q], dsts[q], (uint64_t) bytes[q]))
            return set_err(MPIX_REDOP_ERR_BUFFER);
        const void *pd;
        if (!reachable(srcs[q], (hipStream_t) stream, &launch, &ds[m]) ||
            !reachable(dsts[q], (hipStream_t) stream, &launch, &pd))
            return set_err(MPIX_REDOP_ERR_BUFFER);
        dd[m] = (void *) pd;
        nb[m++] = (uint64_t) bytes[q];
    }
    if (!m)
        return set_err(MPIX_REDOP_SUCCESS);
    launch_cfg();
    return set_err(hip_err(mpix::launch_copy_multi(ds, dd, nb, m, (hipStream_t) stream,
                                                   (unsigned) launch_cfg().wt_xcd)));
}

int MPIX_Ipc_export(const void *devptr, void *handle_out, MPIX_Aint *offset_out)
{
    if (!devptr || !handle_out || !offset_out)
        return set_err(MPIX_REDOP_ERR_ARG);
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t) devptr);
    if (e != hipSuccess)
        return set_err(hip_err(e));
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, (void *) base);
    if (e != hipSuccess)
        return set_err(hip_err(e));
    memcpy(handle_out, &h, sizeof(h));
    *offset_out = (MPIX_Aint) ((const char *) devptr - (const char *) base);
    return set_err(MPIX_REDOP_SUCCESS);
}

int MPIX_Ipc_open(const void *handle, void **base_out)
{
    if (!handle || !base_out)
        return set_err(MPIX_REDOP_ERR_ARG);
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    return set_err(hip_err(hipIpcOpenMemHandle(base_out, h, hipIpcMemLazyEnablePeerAccess)));
}

int MPIX_Ipc_close(void *base)
{
    return set_err(hip_err(hipIpcCloseMemHandle(base)));
}

int MPIX_Redop_peer_access(int device, int peer_device)
{
    return peer_access(device, peer_device) ? 1 : 0;
}

// the (op, type) half of the predicate: a kernel exists (knob-independent)
static int has_gpu_path(uint32_t op, uint32_t it)
{
    if (it == kNull || extent_of(it) == 0 || !internal_ok(op, it))
        return 0;
    uint32_t opi = op & 0xf;
    if (opi == 13 || opi == 14)
        return 1;
    if (opi == 15)
        return (it & 0xffffff00u) == U8;
    return gpu_entry(opi, it) ? 1 : 0;
}

int MPIX_Redop_has_gpu_path(MPIX_Op op, MPIX_Datatype datatype)
{
    return has_gpu_path((uint32_t) op, to_internal((uint32_t) datatype));
}

// MPIR_Typerep_reduce_is_supported (typerep_yaksa_pack.c:227-271): the enable
// knob, the size threshold on the packed size for count > 0 (count 0, as
// reduce_local.c:68 passes it, only asks about the pair), then the pair
int MPIX_Redop_is_supported(MPIX_Op op, MPIX_Aint count, MPIX_Datatype datatype)
{
    env();
    if (!g_enable.load())
        return 0;
    uint32_t it = to_internal((uint32_t) datatype);
    if (count > 0) {
        const long long thr = g_threshold.load();
        const uint64_t sz = size_of(it);
        if (thr > 0 && sz && (uint64_t) count > (uint64_t) thr / sz)
            return 0;
    }
    return has_gpu_path((uint32_t) op, it);
}

// The same with the operands in view: both host-resident below the floor of
// their memory kind -> 0, MPICH keeps its op_fns.c loop for the chunk.  A
// device operand always goes to the GPU (the CPU could only reach it through
// two PCIe copies).
int MPIX_Redop_is_supported_buffers(MPIX_Op op, MPIX_Aint count, MPIX_Datatype datatype,
                                    const void *inbuf, const void *inoutbuf)
{
    if (!MPIX_Redop_is_supported(op, count, datatype))
        return 0;
    if (count <= 0 || !inbuf || !inoutbuf)
        return 1;
    int d0 = 0, d1 = 0;
    const void *p0, *p1;
    const Where w0 = classify(inbuf, &d0, &p0), w1 = classify(inoutbuf, &d1, &p1);
    if (w0 == Where::Device || w1 == Where::Device)
        return 1;
    const long long floor_bytes = (w0 == Where::Pageable || w1 == Where::Pageable)
                                      ? g_host_floor.load() : g_pinned_floor.load();
    const uint64_t bytes = (uint64_t) count * extent_of(to_internal((uint32_t) datatype));
    return (floor_bytes > 0 && bytes < (uint64_t) floor_bytes) ? 0 : 1;
}

int MPIX_Redop_set_support(int enable, MPIX_Aint threshold_bytes, MPIX_Aint host_floor_bytes,
                           MPIX_Aint pinned_floor_bytes)
{
    env();
    g_enable = enable != 0;
    g_threshold = (long long) threshold_bytes;
    g_host_floor = (long long) host_floor_bytes;
    g_pinned_floor = (long long) pinned_floor_bytes;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_get_support(int *enable, MPIX_Aint *threshold_bytes, MPIX_Aint *host_floor_bytes,
                           MPIX_Aint *pinned_floor_bytes)
{
    env();
    if (enable)
        *enable = g_enable.load() ? 1 : 0;
    if (threshold_bytes)
        *threshold_bytes = (MPIX_Aint) g_threshold.load();
    if (host_floor_bytes)
        *host_floor_bytes = (MPIX_Aint) g_host_floor.load();
    if (pinned_floor_bytes)
        *pinned_floor_bytes = (MPIX_Aint) g_pinned_floor.load();
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_op_dt_check(MPIX_Op op, MPIX_Datatype datatype)
{
    return binding_ok((uint32_t) op, (uint32_t) datatype) ? 1 : 0;
}

int MPIX_Redop_internal_op_dt_check(MPIX_Op op, MPIX_Datatype datatype)
{
    return internal_ok((uint32_t) op, (uint32_t) datatype) ? 1 : 0;
}

MPIX_Datatype MPIX_Datatype_internal(MPIX_Datatype datatype)
{
    return (MPIX_Datatype) to_internal((uint32_t) datatype);
}

MPIX_Aint MPIX_Datatype_extent(MPIX_Datatype datatype)
{
    return (MPIX_Aint) extent_of(to_internal((uint32_t) datatype));
}

MPIX_Aint MPIX_Datatype_size(MPIX_Datatype datatype)
{
    return (MPIX_Aint) size_of(to_internal((uint32_t) datatype));
}

int MPIX_Redop_set_fortran_booleans(int true_value, int false_value)
{
    g_ftrue = true_value;
    g_ffalse = false_value;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_set_launch(int block_threads, int max_grid)
{
    env();
    if (block_threads < 64 || block_threads > 1024 || block_threads % 64 || max_grid < 0)
        return MPIX_REDOP_ERR_ARG;
    g_block = block_threads;
    g_max_grid = max_grid;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_set_store_policy(int xcd_mask, int every, int phase, int tail_blocks)
{
    env();
    if (xcd_mask < kWtAuto || xcd_mask > 0xff || every < 0 || phase < 0 ||
        phase >= (every > 0 ? every : 1) || tail_blocks < 0)
        return MPIX_REDOP_ERR_ARG;
    g_wt_xcd = xcd_mask;
    g_wt_every = every;
    g_wt_phase = phase;
    g_wt_tail = tail_blocks;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_set_sync_store_policy(int xcd_mask)
{
    env();
    if (xcd_mask < kWtAuto || xcd_mask > 0xff)
        return MPIX_REDOP_ERR_ARG;
    g_wt_xcd_sync = xcd_mask;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_get_sync_store_policy(int *xcd_mask)
{
    env();
    if (!xcd_mask)
        return MPIX_REDOP_ERR_ARG;
    // as launch_cfg(…, sync = true) resolves it; -1 while the default is
    // not settled (no launch so far)
    const int ws = g_wt_xcd_sync.load(), x = g_wt_xcd.load();
    *xcd_mask = ws != kWtAuto ? ws : x != kWtAuto ? x : g_wt_sync_default.load();
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_sync_timing(int device, int ncalls)
{
    env();
    if (device < 0 || device >= kMaxDev || ncalls < 0 || ncalls > kSyncTimingMax)
        return set_err(MPIX_REDOP_ERR_ARG);
    DeviceGuard g(device);
    DevState *d = dev_state(device);
    if (!d)
        return set_err(MPIX_REDOP_ERR_OTHER);
    while (d->tev.size() < 2 * (size_t) ncalls) {
        hipEvent_t e = nullptr;
        int rc = hip_err(hipEventCreate(&e));
        if (rc)
            return set_err(rc);
        d->tev.push_back(e);
    }
    d->t_cap = ncalls;
    d->t_used = 0;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_sync_timing_read(int device, float *ms, int cap, int *got)
{
    env();
    if (device < 0 || device >= kMaxDev || !got || cap < 0 || (cap > 0 && !ms))
        return set_err(MPIX_REDOP_ERR_ARG);
    DeviceGuard g(device);
    DevState *d = dev_state(device);
    if (!d)
        return set_err(MPIX_REDOP_ERR_OTHER);
    const int n = d->t_used < cap ? d->t_used : cap;
    for (int i = 0; i < n; ++i) {
        int rc = hip_err(hipEventSynchronize(d->tev[2 * i + 1]));
        if (!rc)
            rc = hip_err(hipEventElapsedTime(&ms[i], d->tev[2 * i], d->tev[2 * i + 1]));
        if (rc)
            return set_err(rc);
    }
    *got = n;
    d->t_cap = d->t_used = 0;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_get_store_policy(int *xcd_mask, int *every, int *phase, int *tail_blocks)
{
    env();
    if (xcd_mask) {     // -1: the default, not settled yet (no launch so far)
        const int x = g_wt_xcd.load();
        *xcd_mask = x == kWtAuto ? g_wt_default.load() : x;
    }
    if (every)
        *every = g_wt_every.load();
    if (phase)
        *phase = g_wt_phase.load();
    if (tail_blocks)
        *tail_blocks = g_wt_tail.load();
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_set_pageable(int threads, MPIX_Aint chunk_bytes)
{
    env();
    if (threads < 0 || threads > 16 || chunk_bytes < 65536 || chunk_bytes > ((MPIX_Aint) 256 << 20))
        return MPIX_REDOP_ERR_ARG;
    g_pipe_threads = threads;
    g_pipe_chunk = (size_t) chunk_bytes;
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_get_pageable(int *threads, MPIX_Aint *chunk_bytes)
{
    env();
    if (threads)
        *threads = g_pipe_threads.load();
    if (chunk_bytes)
        *chunk_bytes = (MPIX_Aint) g_pipe_chunk.load();
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_get_launch(int *block_threads, int *unroll, int *max_grid)
{
    env();
    if (block_threads)
        *block_threads = g_block.load();
    if (unroll)
        *unroll = mpix::unroll();
    if (max_grid)
        *max_grid = g_max_grid.load();
    return MPIX_REDOP_SUCCESS;
}

int MPIX_Redop_last_error(void) { return t_last_error; }

const char *MPIX_Redop_error_string(int code)
{
    switch (code) {
        case MPIX_REDOP_SUCCESS: return "success";
        case MPIX_REDOP_ERR_BUFFER: return "invalid buffer (NULL, MPI_IN_PLACE or aliased)";
        case MPIX_REDOP_ERR_COUNT: return "invalid count";
        case MPIX_REDOP_ERR_TYPE: return "datatype unknown or not supported on the GPU path";
        case MPIX_REDOP_ERR_OP: return "operation not defined for this datatype";
        case MPIX_REDOP_ERR_ARG: return "invalid argument";
        case MPIX_REDOP_ERR_OTHER: return "HIP runtime error";
        default: return "internal error";
    }
}

const char *MPIX_Redop_build_info(void)
{
#define MPIX_STR2(x) #x
#define MPIX_STR(x) MPIX_STR2(x)
    return mpix_build_info();
}

// ------------------------------------------------ MPIR_op_function table
// A failed call is fatal, like the reference's MPIR_Assert(0) on a type its
// op function does not cover (op_fns.c:51-53), unless MPIX_REDOP_OPFN_ABORT=0:
// then the error class is only recorded for MPIX_Redop_last_error().
static void opfn_failed(const char *name, int rc, MPIX_Datatype type)
{
    if (!g_opfn_abort.load())
        return;
    fprintf(stderr, "MPIX_Op_table: %s on datatype 0x%08x failed: %s (MPI error class %d); "
                    "only pairs MPIX_Redop_is_supported() accepts may use the table\n",
            name, (unsigned) type, MPIX_Redop_error_string(rc), rc);
    fflush(stderr);
    abort();
}
#define MPIX_OPFN(name, handle)                                                           \
    void name(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type)           \
    {                                                                                     \
        env();          /* MPIX_REDOP_OPFN_ABORT, even if the call fails at once */      \
        int rc_ = MPIX_Reduce_local(invec, inoutvec, *len, *type, handle);               \
        if (rc_ != MPIX_REDOP_SUCCESS)                                                    \
            opfn_failed(#name, rc_, *type);                                               \
    }
MPIX_OPFN(MPIX_MAXF, MPIX_MAX)
MPIX_OPFN(MPIX_MINF, MPIX_MIN)
MPIX_OPFN(MPIX_SUM_fn, MPIX_SUM)
MPIX_OPFN(MPIX_PROD_fn, MPIX_PROD)
MPIX_OPFN(MPIX_LAND_fn, MPIX_LAND)
MPIX_OPFN(MPIX_BAND_fn, MPIX_BAND)
MPIX_OPFN(MPIX_LOR_fn, MPIX_LOR)
MPIX_OPFN(MPIX_BOR_fn, MPIX_BOR)
MPIX_OPFN(MPIX_LXOR_fn, MPIX_LXOR)
MPIX_OPFN(MPIX_BXOR_fn, MPIX_BXOR)
MPIX_OPFN(MPIX_MINLOC_fn, MPIX_MINLOC)
MPIX_OPFN(MPIX_MAXLOC_fn, MPIX_MAXLOC)
MPIX_OPFN(MPIX_REPLACE_fn, MPIX_REPLACE)
MPIX_OPFN(MPIX_NO_OP_fn, MPIX_NO_OP)
MPIX_OPFN(MPIX_EQUAL_fn, MPIX_EQUAL)
#undef MPIX_OPFN

// order of src/mpi/coll/op/oputil.c:10-27 / mpi.h.in:297-311
MPIX_op_function *const MPIX_Op_table[16] = {
    nullptr, MPIX_MAXF, MPIX_MINF, MPIX_SUM_fn, MPIX_PROD_fn, MPIX_LAND_fn, MPIX_BAND_fn,
    MPIX_LOR_fn, MPIX_BOR_fn, MPIX_LXOR_fn, MPIX_BXOR_fn, MPIX_MINLOC_fn, MPIX_MAXLOC_fn,
    MPIX_REPLACE_fn, MPIX_NO_OP_fn, MPIX_EQUAL_fn,
};

}  // extern "C"
