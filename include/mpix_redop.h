/*
 * mpix_redop.h -- C-ABI of the MI355X-native local reduction library
 * (libmpix_redop.so, built from mpich_amd/csrc/).
 *
 * This is the drop-in boundary for MPICH's local element-wise reduction:
 * every entry point below replaces one reference interface, cited as
 * reference-file:line (paths relative to the pmodels/mpich tree).
 *
 *   MPIX_Reduce_local        <- MPIR_Reduce_local
 *                               src/include/mpir_coll.h:62-63,
 *                               body src/mpi/coll/reduce_local/reduce_local.c:53-96
 *   MPIX_Reduce_local_async  <- same contract, enqueued on a caller HIP stream
 *                               (what the NBC engines need:
 *                               src/mpi/coll/transports/gentran/gentran_utils.c:157-167)
 *   MPIX_Redop_is_supported  <- MPIR_Typerep_reduce_is_supported
 *                               src/mpi/datatype/typerep/yaksa/typerep_yaksa_pack.c:218-271,
 *                               used by maint/gen_coll.py:546-547 for host staging
 *   MPIX_Op_table / MPIX_SUM.. <- MPIR_Op_table + MPIR_op_function
 *                               src/mpi/coll/op/oputil.c:10-27, src/include/mpir_op.h:206-209
 *   MPIX_Redop_op_dt_check   <- MPIR_op_dt_check  src/include/mpir_datatype.h:780-868
 *   MPIX_Redop_internal_op_dt_check <- MPIR_Internal_op_dt_check  mpir_datatype.h:870-933
 *   MPIX_Datatype_internal   <- MPIR_DATATYPE_REPLACE_BUILTIN  mpir_datatype.h:169-176
 *                               with the table of src/mpi/datatype/typeutil.c:29-109
 *   MPIX_Reduce_local_vector <- typerep_op_fallback on an MPI_Type_vector target
 *                               src/mpi/datatype/typerep/src/typerep_op.c:69-155
 *   MPIX_Redop_set_fortran_booleans <- MPIR_Abi_set_fortran_booleans_impl
 *                               src/mpi/datatype/typeutil.c:502-515
 *
 * Handles use MPICH's own 32-bit encoding (src/include/mpi.h.in:166-311 and
 * src/include/mpir_datatype.h:22-125), so an MPICH build can pass its
 * MPI_Datatype / MPI_Op values straight through.  Both the external builtin
 * handles (MPI_FLOAT = 0x4c00040a) and the internal ones MPIR_Reduce_local
 * receives (MPIR_FLOAT32|0x0a = 0x4c83040a) are accepted, as are the struct
 * pair types MPI_{FLOAT,DOUBLE,LONG,SHORT}_INT (0x8c00000k).
 *
 * No C++ or torch types appear here: plain pointers, sizes and int codes.
 */
#ifndef MPIX_REDOP_H_INCLUDED
#define MPIX_REDOP_H_INCLUDED

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int MPIX_Datatype;      /* same width/encoding as MPICH's MPI_Datatype */
typedef int MPIX_Op;            /* same width/encoding as MPICH's MPI_Op */
typedef intptr_t MPIX_Aint;     /* MPI_Aint on LP64 */

/* ---- return codes: MPI error classes (src/include/mpi.h.in:650-677) ---- */
#define MPIX_REDOP_SUCCESS     0
#define MPIX_REDOP_ERR_BUFFER  1        /* MPI_ERR_BUFFER: NULL / MPI_IN_PLACE / aliased */
#define MPIX_REDOP_ERR_COUNT   2        /* MPI_ERR_COUNT: negative count */
#define MPIX_REDOP_ERR_TYPE    3        /* MPI_ERR_TYPE: datatype unknown or not on GPU */
#define MPIX_REDOP_ERR_OP      9        /* MPI_ERR_OP: op undefined for this datatype */
#define MPIX_REDOP_ERR_ARG     12       /* MPI_ERR_ARG */
#define MPIX_REDOP_ERR_OTHER   15       /* MPI_ERR_OTHER: HIP runtime failure */
#define MPIX_REDOP_ERR_INTERN  16       /* MPI_ERR_INTERN */

/* ---- predefined ops (mpi.h.in:297-311); index = op & 0xf ---- */
#define MPIX_OP_NULL  ((MPIX_Op)0x18000000)
#define MPIX_MAX      ((MPIX_Op)0x58000001)
#define MPIX_MIN      ((MPIX_Op)0x58000002)
#define MPIX_SUM      ((MPIX_Op)0x58000003)
#define MPIX_PROD     ((MPIX_Op)0x58000004)
#define MPIX_LAND     ((MPIX_Op)0x58000005)
#define MPIX_BAND     ((MPIX_Op)0x58000006)
#define MPIX_LOR      ((MPIX_Op)0x58000007)
#define MPIX_BOR      ((MPIX_Op)0x58000008)
#define MPIX_LXOR     ((MPIX_Op)0x58000009)
#define MPIX_BXOR     ((MPIX_Op)0x5800000a)
#define MPIX_MINLOC   ((MPIX_Op)0x5800000b)
#define MPIX_MAXLOC   ((MPIX_Op)0x5800000c)
#define MPIX_REPLACE  ((MPIX_Op)0x5800000d)
#define MPIX_NO_OP    ((MPIX_Op)0x5800000e)
#define MPIX_EQUAL    ((MPIX_Op)0x5800000f)

/* ---- internal datatype encoding (mpir_datatype.h:22-125) ----
 * 0x4c | kind | size | builtin index.  Kinds: */
#define MPIX_TYPE_INTERNAL_MASK  0x800000
#define MPIX_TYPE_PAIR_MASK      0x400000
#define MPIX_TYPE_KIND_MASK      0x0f0000
#define MPIX_TYPE_FIXED          0x000000
#define MPIX_TYPE_SIGNED         0x010000
#define MPIX_TYPE_UNSIGNED       0x020000
#define MPIX_TYPE_FLOAT          0x030000
#define MPIX_TYPE_COMPLEX        0x040000
#define MPIX_TYPE_ALT_FLOAT      0x050000
#define MPIX_TYPE_ALT_COMPLEX    0x060000
#define MPIX_TYPE_FORTRAN_LOGICAL 0x070000

#define MPIX_INT8      ((MPIX_Datatype)0x4c810100)
#define MPIX_INT16     ((MPIX_Datatype)0x4c810200)
#define MPIX_INT32     ((MPIX_Datatype)0x4c810400)
#define MPIX_INT64     ((MPIX_Datatype)0x4c810800)
#define MPIX_INT128    ((MPIX_Datatype)0x4c811000)
#define MPIX_UINT8     ((MPIX_Datatype)0x4c820100)
#define MPIX_UINT16    ((MPIX_Datatype)0x4c820200)
#define MPIX_UINT32    ((MPIX_Datatype)0x4c820400)
#define MPIX_UINT64    ((MPIX_Datatype)0x4c820800)
#define MPIX_UINT128   ((MPIX_Datatype)0x4c821000)
#define MPIX_FLOAT16   ((MPIX_Datatype)0x4c830200)
#define MPIX_FLOAT32   ((MPIX_Datatype)0x4c830400)
#define MPIX_FLOAT64   ((MPIX_Datatype)0x4c830800)
#define MPIX_FLOAT128  ((MPIX_Datatype)0x4c831000)
#define MPIX_COMPLEX16 ((MPIX_Datatype)0x4c840400)  /* 2 x fp16 */
#define MPIX_COMPLEX32 ((MPIX_Datatype)0x4c840800)  /* float _Complex */
#define MPIX_COMPLEX64 ((MPIX_Datatype)0x4c841000)  /* double _Complex */
#define MPIX_COMPLEX128 ((MPIX_Datatype)0x4c842000) /* 2 x __float128 */
#define MPIX_BFLOAT16_INTERNAL ((MPIX_Datatype)0x4c850200)
#define MPIX_ALT_FLOAT128 ((MPIX_Datatype)0x4c851000)   /* x86-64 long double */
#define MPIX_ALT_COMPLEX128 ((MPIX_Datatype)0x4c862000) /* long double _Complex */
#define MPIX_FORTRAN_LOGICAL8   ((MPIX_Datatype)0x4c870100)
#define MPIX_FORTRAN_LOGICAL16  ((MPIX_Datatype)0x4c870200)
#define MPIX_FORTRAN_LOGICAL32  ((MPIX_Datatype)0x4c870400)
#define MPIX_FORTRAN_LOGICAL64  ((MPIX_Datatype)0x4c870800)
#define MPIX_FORTRAN_LOGICAL128 ((MPIX_Datatype)0x4c871000)
/* builtin pair types {T value; T loc} (mpir_datatype.h:111-125) */
#define MPIX_2INT8     ((MPIX_Datatype)0x4cc10200)
#define MPIX_2INT16    ((MPIX_Datatype)0x4cc10400)
#define MPIX_2INT32    ((MPIX_Datatype)0x4cc10800)
#define MPIX_2INT64    ((MPIX_Datatype)0x4cc11000)
#define MPIX_2UINT8    ((MPIX_Datatype)0x4cc20200)
#define MPIX_2UINT16   ((MPIX_Datatype)0x4cc20400)
#define MPIX_2UINT32   ((MPIX_Datatype)0x4cc20800)
#define MPIX_2UINT64   ((MPIX_Datatype)0x4cc21000)
#define MPIX_2FLOAT16  ((MPIX_Datatype)0x4cc30400)
#define MPIX_2FLOAT32  ((MPIX_Datatype)0x4cc30800)
#define MPIX_2FLOAT64  ((MPIX_Datatype)0x4cc31000)

/* ---- a few external builtin handles (mpi.h.in:166-264) ---- */
#define MPIX_MPI_CHAR          ((MPIX_Datatype)0x4c000101)
#define MPIX_MPI_INT           ((MPIX_Datatype)0x4c000405)
#define MPIX_MPI_LONG          ((MPIX_Datatype)0x4c000807)
#define MPIX_MPI_FLOAT         ((MPIX_Datatype)0x4c00040a)
#define MPIX_MPI_DOUBLE        ((MPIX_Datatype)0x4c00080b)
#define MPIX_MPI_BYTE          ((MPIX_Datatype)0x4c00010d)
#define MPIX_MPI_2INT          ((MPIX_Datatype)0x4c000816)
#define MPIX_MPI_C_FLOAT16     ((MPIX_Datatype)0x4c000246)
#define MPIX_MPI_BFLOAT16      ((MPIX_Datatype)0x4c00024c)
/* struct pair types, created by MPIR_Datatype_init_pairtypes (pairtypes.c:99-121) */
#define MPIX_MPI_FLOAT_INT       ((MPIX_Datatype)0x8c000000)
#define MPIX_MPI_DOUBLE_INT      ((MPIX_Datatype)0x8c000001)
#define MPIX_MPI_LONG_INT        ((MPIX_Datatype)0x8c000002)
#define MPIX_MPI_SHORT_INT       ((MPIX_Datatype)0x8c000003)
#define MPIX_MPI_LONG_DOUBLE_INT ((MPIX_Datatype)0x8c000004)

/* ---- library lifetime ----
 * init is optional (every entry point initialises lazily); finalize frees
 * the calling thread's streams and host-staging scratch, and those that
 * exited threads left in the reuse pool (a thread that exits without
 * finalizing hands its state to the next new thread). */
int MPIX_Redop_init(void);
int MPIX_Redop_finalize(void);

/* ---- the hot path ----
 * inoutbuf[i] = inoutbuf[i] OP inbuf[i] for i < count elements of
 * `datatype` (extent-strided, i.e. pair padding preserved).
 *
 * MPIX_Reduce_local: synchronous, like MPIR_Reduce_local.  Buffers may be
 * device memory (hipMalloc / managed) or host memory; host operands are
 * staged through device scratch with hipMemcpyAsync.  count == 0 is a
 * successful no-op (reduce_local.c:59-60).
 *
 * MPIX_Reduce_local_async: both buffers must be device-accessible; the
 * kernel is enqueued on `stream` (a hipStream_t, NULL = legacy default
 * stream) and the call returns without waiting. */
int MPIX_Reduce_local(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                      MPIX_Datatype datatype, MPIX_Op op);
int MPIX_Reduce_local_async(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                            MPIX_Datatype datatype, MPIX_Op op, void *stream);

/* Derived (vector) target, packed source -- typerep_op.c:115-150 with the
 * target an MPI_Type_vector(count, blocklen, stride, basic_type):
 *   for b < count, j < blocklen:
 *     inout[b*stride + j] = inout[b*stride + j] OP in[b*blocklen + j]
 * (stride and blocklen in elements; gaps in the target are never written).
 * Device buffers only; the sync form waits on its stream. */
int MPIX_Reduce_local_vector_async(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                                   MPIX_Aint blocklen, MPIX_Aint stride,
                                   MPIX_Datatype basic_type, MPIX_Op op, void *stream);
int MPIX_Reduce_local_vector(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                             MPIX_Aint blocklen, MPIX_Aint stride,
                             MPIX_Datatype basic_type, MPIX_Op op);

/* General derived target given as its flattened iov, packed source --
 * typerep_op_fallback (typerep_op.c:100-150) with the target's iov already
 * resolved to element runs: for s < nseg, in order, seg_counts[s] elements
 * (extent stride) at byte offset seg_offsets[s] of inoutbuf are combined
 * with the next seg_counts[s] elements of inbuf.  Offsets may be negative
 * (lb < 0) and need only the 4-byte alignment of the element loads (2 for
 * 2-byte types); runs must not overlap (MPI accumulate targets).  The
 * tables are host arrays, read before the call returns (the run table is
 * uploaded through pinned memory, asynchronously on `stream`; two table
 * slots are used in turn, so a call waits only for the kernels of the iov
 * call before the previous one, whose slot it takes over).
 * Device buffers. */
int MPIX_Reduce_local_iov_async(const void *inbuf, void *inoutbuf, MPIX_Aint nseg,
                                const MPIX_Aint *seg_offsets, const MPIX_Aint *seg_counts,
                                MPIX_Datatype basic_type, MPIX_Op op, void *stream);

/* The same fallback over the raw iov, as MPIR_Typerep_to_iov_offset gives
 * it (typerep_op.c:100-110): segment i is iov_lens[i] BYTES at byte offset
 * iov_offsets[i] of inoutbuf.  For a basic type each segment must hold
 * whole elements (the reference asserts, :147; here MPI_ERR_ARG).  For a
 * pair type whose size is below its extent (DOUBLE_INT, LONG_INT,
 * SHORT_INT: the padding splits each element into {value, int} segments)
 * segments are gathered until they hold curr_len >= size bytes, then
 * curr_len / size elements are combined at extent stride from the first
 * gathered segment, and a partial element left at a segment's end starts
 * the next run -- typerep_op.c:117-148 exactly. */
int MPIX_Reduce_local_iovec_async(const void *inbuf, void *inoutbuf, MPIX_Aint nseg,
                                  const MPIX_Aint *iov_offsets, const MPIX_Aint *iov_lens,
                                  MPIX_Datatype basic_type, MPIX_Op op, void *stream);

/* Multi-input form: equivalent to `ninputs` MPIX_Reduce_local calls
 *   for k = 0 .. ninputs-1:  inoutbuf = inoutbuf OP inbufs[k]
 * in that order (same association, same bits) but done in one pass over
 * memory.  Used by reduce-scatter schedules whose received blocks arrive
 * together (pairwise, reduce_scatter_block_intra_pairwise.c:86-100).
 * 1 <= ninputs <= 16; device-accessible buffers; stream-ordered. */
int MPIX_Reduce_local_multi_async(const void *const *inbufs, int ninputs, void *inoutbuf,
                                  MPIX_Aint count, MPIX_Datatype datatype, MPIX_Op op,
                                  void *stream);

/* Tree form: outbuf = the pairwise tree fold of ninputs = 2^L slots
 * (2 <= ninputs <= 16), level by level m = 1, 2, 4, ...:
 *   slot s (bit m of s clear) = slot s OP slot s+m   (slot s is inout)
 * and outbuf = slot 0.  inbufs[0] must be given; a NULL slot s > 0 is absent:
 * at its level the partner passes through unchanged (the first level of the
 * reference's fold of a non-power-of-two world, where only the paired ranks
 * combine).  Holding the block of rank r ^ bitrev(s) in slot s,
 * this is the association recursive halving gives rank r's block
 * (reduce_scatter_block_intra_recursive_halving.c:164-229, P a power of
 * two), so a schedule that can read every peer's block computes the
 * reference's bits in one pass.  outbuf may be one of the slots exactly (in
 * place); no partial overlap.  REPLACE yields the last present slot, NO_OP
 * the first; MPIX_EQUAL is refused (MPI_ERR_OP).  Device-accessible buffers;
 * stream-ordered. */
int MPIX_Reduce_local_tree_async(const void *const *inbufs, int ninputs, void *outbuf,
                                 MPIX_Aint count, MPIX_Datatype datatype, MPIX_Op op,
                                 void *stream);

/* n <= 16 independent copies dsts[q] <- srcs[q] (bytes[q] each) in ONE
 * stream-ordered launch, all running at once -- the allgather step of a pull
 * schedule, whose P-1 sources sit behind P-1 different xGMI links.
 * Device-accessible, non-overlapping pairs; zero-byte entries are skipped. */
int MPIX_Copy_multi_async(const void *const *srcs, void *const *dsts, const MPIX_Aint *bytes,
                          int n, void *stream);

/* ---- peer memory for the fused pull + combine ----
 * The reference maps peer GPU buffers with hipIpc* in its shm/ipc path
 * (src/mpl/src/gpu/mpl_gpu_hip.c:174-204).  Here a rank exports the
 * allocation holding `devptr` (handle: MPIX_IPC_HANDLE_BYTES opaque bytes,
 * plus the byte offset of devptr inside it); peers open it and pass the
 * mapped addresses straight to MPIX_Reduce_local_multi_async, so the combine
 * kernel reads the peers' blocks over xGMI with no intermediate copy. */
#define MPIX_IPC_HANDLE_BYTES 64
int MPIX_Ipc_export(const void *devptr, void *handle_out, MPIX_Aint *offset_out);
int MPIX_Ipc_open(const void *handle, void **base_out);
int MPIX_Ipc_close(void *base);

/* ---- operands on two devices ----
 * 1 if kernels on `device` can dereference memory of `peer_device` (same
 * device, or peer access enabled -- by this call at the pair's first use,
 * once per process), else 0.  Replaces the all-pairs loop of the reference's
 * HIP init hook (yaksa/src/backend/hip/hooks/yaksuri_hip_init_hooks.c:164-181:
 * hipDeviceCanAccessPeer, hipDeviceEnablePeerAccess, "already enabled"
 * tolerated).  Every entry point settles its pairs itself: MPIX_Reduce_local
 * runs on inout's device and, without peer access, copies `in` over with
 * hipMemcpyPeerAsync; the stream-ordered entry points return MPI_ERR_BUFFER
 * for an operand the stream's device cannot reach.  Env MPIX_REDOP_PEER=stage
 * treats every pair of distinct devices as unreachable. */
int MPIX_Redop_peer_access(int device, int peer_device);

/* 1 if (op, datatype) goes to the GPU path, else 0 -- the contract of
 * MPIR_Typerep_reduce_is_supported (typerep_yaksa_pack.c:227-271), which
 * reduce_local.c:68 (count 0) and maint/gen_coll.py:546-547 (count of the
 * collective) consult.  0 when the path is disabled (env MPIX_REDOP_ENABLE=0,
 * as MPIR_CVAR_ENABLE_YAKSA_REDUCTION), when count > 0 and the packed size
 * count * size exceeds the threshold (env MPIX_REDOP_THRESHOLD bytes, default
 * -1 = no limit, as MPIR_CVAR_YAKSA_REDUCTION_THRESHOLD), or when no kernel
 * covers the pair.  When 0, a caller keeps its own CPU op table. */
int MPIX_Redop_is_supported(MPIX_Op op, MPIX_Aint count, MPIX_Datatype datatype);

/* 1 if a GPU kernel covers (op, datatype), whatever the knobs above say (the
 * collectives of libmpix_coll decline a pair only when this is 0, so
 * MPIX_REDOP_ENABLE=0 never turns them off). */
int MPIX_Redop_has_gpu_path(MPIX_Op op, MPIX_Datatype datatype);

/* The same predicate with the operands in view, for reduce_local.c's branch:
 * additionally 0 when BOTH buffers are host-resident and one operand holds
 * fewer bytes than the host floor of its memory kind (pageable: env
 * MPIX_REDOP_HOST_FLOOR, page-locked: MPIX_REDOP_PINNED_FLOOR), below which one
 * core's op_fns.c loop beats the round trip over PCIe (crossover measured by
 * bench.py, `host_crossover`).  A device-resident operand always answers as
 * MPIX_Redop_is_supported does. */
int MPIX_Redop_is_supported_buffers(MPIX_Op op, MPIX_Aint count, MPIX_Datatype datatype,
                                    const void *inbuf, const void *inoutbuf);

/* The predicate's knobs at run time (the env variables above set them at
 * first use): enable 0/1, threshold (<= 0: none), the two host floors
 * (<= 0: no floor). */
int MPIX_Redop_set_support(int enable, MPIX_Aint threshold_bytes, MPIX_Aint host_floor_bytes,
                           MPIX_Aint pinned_floor_bytes);
int MPIX_Redop_get_support(int *enable, MPIX_Aint *threshold_bytes, MPIX_Aint *host_floor_bytes,
                           MPIX_Aint *pinned_floor_bytes);

/* Binding-level and internal legality of (op, datatype): 1 legal, 0 not. */
int MPIX_Redop_op_dt_check(MPIX_Op op, MPIX_Datatype datatype);
int MPIX_Redop_internal_op_dt_check(MPIX_Op op, MPIX_Datatype datatype);

/* External builtin -> internal type (identity for internal / pair handles,
 * MPIX_DATATYPE_NULL (0x0c000000) for unknown builtins). */
MPIX_Datatype MPIX_Datatype_internal(MPIX_Datatype datatype);
/* Extent in bytes of one element (pair types include padding); 0 if unknown. */
MPIX_Aint MPIX_Datatype_extent(MPIX_Datatype datatype);
/* Size in bytes of one element's data (MPIR_Datatype_get_size_macro):
 * the extent, except for the padded pairs DOUBLE_INT / LONG_INT (12),
 * SHORT_INT (6) and LONG_DOUBLE_INT (20); 0 if unknown. */
MPIX_Aint MPIX_Datatype_size(MPIX_Datatype datatype);

/* Fortran .TRUE./.FALSE. used by LAND/LOR/LXOR on Fortran logicals
 * (mpii_fortlogical.h:15,28; defaults 1 / 0 as typeutil.c:502-510). */
int MPIX_Redop_set_fortran_booleans(int true_value, int false_value);

/* ---- per-op function table, MPIR_op_function signature (mpir_op.h:206) ----
 * Synchronous; same pointer rules as MPIX_Reduce_local.  Only pairs that
 * MPIX_Redop_is_supported() accepts may be passed: the op functions return
 * void like the reference's, and a call that fails (a pair no kernel covers,
 * e.g. MPI_MAX on MPIX_BFLOAT16, or a HIP error) prints the reason and abort()s, as
 * the reference's MPIR_Assert(0) does (op_fns.c:51-53).  With env
 * MPIX_REDOP_OPFN_ABORT=0 the failure is only recorded and can be read with
 * MPIX_Redop_last_error(). */
typedef void MPIX_op_function(void *invec, void *inoutvec, MPIX_Aint *len,
                              MPIX_Datatype *type);
extern MPIX_op_function *const MPIX_Op_table[16];
void MPIX_MAXF(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_MINF(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_SUM_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_PROD_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_LAND_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_BAND_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_LOR_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_BOR_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_LXOR_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_BXOR_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_MINLOC_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_MAXLOC_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_REPLACE_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
void MPIX_NO_OP_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);
/* MPIX_EQUAL (opequal.c:20-35): MPI_BYTE, 8-byte is_equal header + payload */
void MPIX_EQUAL_fn(void *invec, void *inoutvec, MPIX_Aint *len, MPIX_Datatype *type);

int MPIX_Redop_last_error(void);
const char *MPIX_Redop_error_string(int code);

/* ---- several ready chunks in one launch (stream-ordered) ----
 * k independent combines inoutbufs[i][j] = OP(inoutbufs[i][j], inbufs[i][j]),
 * j < counts[i], i < k, of one datatype and op, issued as ONE kernel launch on
 * `stream`: the same bits as k MPIX_Reduce_local_async calls (each segment is
 * split into head / packets / tail exactly as a call of its own would be) at
 * the host cost of one launch (HIP's issue is ~2.5 us per launch,
 * profiles/r04_call_floor.json).  For the engines that find several vertices
 * ready at once -- gentran_utils.c:157-167 calls MPIR_Reduce_local per ready
 * reduce vertex, mpidu_sched.c:309-316 per reduce entry of a schedule round.
 * 1 <= k <= MPIX_BATCH_MAX, else MPI_ERR_ARG; no triple's target range may
 * overlap another triple's target or source range (MPI_ERR_BUFFER: the
 * segments run in no particular order); zero counts are skipped; every
 * operand must be reachable from the stream's device, as for
 * MPIX_Reduce_local_async.  All checks happen before any device work.
 * MPI_REPLACE / MPI_NO_OP / MPIX_EQUAL, operands that are not element-aligned
 * (for the 32-byte pair and complex types: not 16-byte aligned) and triples
 * with a page-locked host operand (read over PCIe by the capped, looping
 * zero-copy grid) are issued one launch per triple. */
#define MPIX_BATCH_MAX 64
int MPIX_Reduce_local_batch_async(const void *const *inbufs, void *const *inoutbufs,
                                  const MPIX_Aint *counts, int k, MPIX_Datatype datatype,
                                  MPIX_Op op, void *stream);

/* ---- launch geometry (performance knob, not semantics) ----
 * threads per block and a cap on the grid (0 = one tile per block, no
 * grid-stride loop).  The packets-per-thread unroll is a compile-time
 * constant (MPIX_REDOP_UNROLL).  Env MPIX_REDOP_BLOCK / MPIX_REDOP_MAXGRID
 * override the defaults at first use.  Kernels that read page-locked host
 * memory over PCIe (zero-copy) run at most 16384 threads' worth of looping
 * blocks (256 at the default 64 threads) unless max_grid is smaller, so loads
 * and stores share the link both ways; env MPIX_REDOP_ZC_GRID sets that cap
 * in blocks (0: none).  Defaults: 64-thread blocks, one 16-byte packet per
 * lane per operand. */
int MPIX_Redop_set_launch(int block_threads, int max_grid);
int MPIX_Redop_get_launch(int *block_threads, int *unroll, int *max_grid);

/* ---- store policy of the contiguous kernel (performance knob, not semantics) ----
 * Blocks of a contiguous launch that run on an XCD whose bit is set in
 * xcd_mask (HW_REG_XCC_ID, bits 0-7), blocks b with b % every == phase
 * (every > 0), and the last tail_blocks blocks store their result
 * write-through (the line leaves the XCD's L2 at once) instead of
 * non-temporally (the line stays in L2, dirty, until evicted or written back
 * at the end of the kernel).  Same bits either way.  Default (xcd_mask -1):
 * 0x88 (two XCDs of eight write through: 8-9 % faster at 1 GiB) when every
 * visible device has 8 XCDs, else 0, settled at the first kernel launch --
 * get_store_policy reports -1 until then, the settled mask after; set -1 to
 * return to it.  every = tail_blocks = 0.  Env MPIX_REDOP_WT_XCD /
 * MPIX_REDOP_WT_EVERY / MPIX_REDOP_WT_PHASE / MPIX_REDOP_WT_TAIL override
 * the defaults at first use.  Neither call, nor any support predicate or
 * other knob, makes a HIP call. */
int MPIX_Redop_set_store_policy(int xcd_mask, int every, int phase, int tail_blocks);
int MPIX_Redop_get_store_policy(int *xcd_mask, int *every, int *phase, int *tail_blocks);

/* The synchronous entry's own XCD mask (MPIX_Reduce_local on device or
 * page-locked operands: the MPIR_Reduce_local drop-in, whose kernels start
 * from an idle GPU call after call).  Default (-1): the mask set with
 * MPIX_Redop_set_store_policy / MPIX_REDOP_WT_XCD if any, else 0x22 on
 * 8-XCD devices (XCDs 1 and 5: the faster synchronous call,
 * profiles/r05_sync_xcd_masks.json), 0 otherwise; env MPIX_REDOP_WT_XCD_SYNC
 * at first use.  get reports the mask the next synchronous launch uses (-1
 * while the default is unsettled).  No HIP call. */
int MPIX_Redop_set_sync_store_policy(int xcd_mask);
int MPIX_Redop_get_sync_store_policy(int *xcd_mask);

/* Kernel timing of the synchronous entry, for measurement (bench.py's
 * roofline figure): the calling thread's next ncalls synchronous calls on
 * `device` (MPIX_Reduce_local on device or page-locked operands) record a HIP
 * event pair around their launch on the library's stream -- the combine as the
 * call runs it, nothing else changed.  ncalls = 0 stops; at most 65536.
 * _read waits for the recorded pairs, stores up to cap durations (ms, call
 * order) in ms[], their number in *got, and stops the recording.  No
 * counterpart in MPICH (a tool interface, like the MPIX_Redop_set_* knobs). */
int MPIX_Redop_sync_timing(int device, int ncalls);
int MPIX_Redop_sync_timing_read(int device, float *ms, int cap, int *got);

/* ---- large pageable host operands (performance knob) ----
 * threads > 0: pageable operands of at least 2 * chunk_bytes go through that many
 * host threads (the caller is one of them).  Default form, "wave": the
 * threads copy one chunk at a time into a page-locked buffer together (each
 * a slice), and ONE zero-copy kernel combines that chunk while they copy the
 * next one in and the previous result out; three chunk buffers rotate, and
 * the chunk sizes ramp up and down at both ends (short pipeline fill).  Env
 * MPIX_REDOP_PAGEABLE_MODE=worker selects the round-2 form instead: each
 * thread copies, combines and copies back chunks of its own (operands of at
 * least 2 * threads * chunk_bytes; env MPIX_REDOP_PAGEABLE_DB=1 gives every
 * thread two buffers).  Smaller operands, and all of them with threads = 0,
 * are staged through device scratch with hipMemcpyAsync.  Same bits every
 * way.  Defaults 8 threads x 64 MiB (env MPIX_REDOP_PAGEABLE_THREADS /
 * MPIX_REDOP_PAGEABLE_CHUNK at first use); threads 0..16, chunk 64 KiB..256
 * MiB.  The buffers are one set per device for the whole process (wave: 3 x
 * 2 x chunk of page-locked memory, 384 MiB at the defaults; worker: threads
 * x 2 x chunk, twice that with two buffers), freed by MPIX_Redop_finalize; a
 * call that finds the set in use by another thread stages its operands
 * instead.  Copies into the page-locked buffers use non-temporal stores (env
 * MPIX_REDOP_PAGEABLE_NT=0: memcpy), and env MPIX_REDOP_PAGEABLE_AFFINITY=gpu
 * pins the threads to the CPUs of the GPU's NUMA node (or to an explicit
 * cpulist such as "64-127"; default none). */
int MPIX_Redop_set_pageable(int threads, MPIX_Aint chunk_bytes);
int MPIX_Redop_get_pageable(int *threads, MPIX_Aint *chunk_bytes);

/* Build identification: the gfx target the code object was compiled for. */
const char *MPIX_Redop_build_info(void);

#define MPIX_DATATYPE_NULL ((MPIX_Datatype)0x0c000000)

#ifdef __cplusplus
}
#endif
#endif /* MPIX_REDOP_H_INCLUDED */
