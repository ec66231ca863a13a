/*
 * mpix_coll.h -- C-ABI of the reduce-scatter / allreduce / reduce schedules that feed
 * the MI355X local reduction (libmpix_coll.so, built from mpich_amd/csrc/).
 *
 * These are host-side C restatements of MPICH's collective schedules whose
 * every combine step is MPIR_Reduce_local -- here MPIX_Reduce_local_async
 * (include/mpix_redop.h) on the HIP stream the collective is enqueued on --
 * and whose point-to-point steps go through a transport:
 *
 *   MPIX_Reduce_scatter_block  <- MPIR_Reduce_scatter_block_intra_recursive_halving
 *                                  src/mpi/coll/reduce_scatter_block/
 *                                  reduce_scatter_block_intra_recursive_halving.c:38-260
 *                                 and ..._intra_pairwise.c:42-104 (MPICH's large-message
 *                                  choice, maint/tuning/coll/mpir/generic.json:316-341)
 *   MPIX_Reduce_scatter        <- MPIR_Reduce_scatter_intra_recursive_halving /
 *                                 _intra_pairwise  src/mpi/coll/reduce_scatter/ (per-rank
 *                                  recvcounts; generic.json:277-291)
 *   MPIX_Allreduce             <- MPIR_Allreduce_intra_reduce_scatter_allgather
 *                                  src/mpi/coll/allreduce/
 *                                  allreduce_intra_reduce_scatter_allgather.c:41-277
 *                                 and MPIR_Allreduce_intra_recursive_doubling
 *                                  allreduce_intra_recursive_doubling.c:24-150
 *                                 and MPIR_Allreduce_intra_ring  allreduce_intra_ring.c:10-105
 *   MPIX_Reduce                <- MPIR_Reduce_intra_binomial  src/mpi/coll/reduce/
 *                                  reduce_intra_binomial.c:12-131
 *                                 and MPIR_Reduce_intra_reduce_scatter_gather
 *                                  reduce_intra_reduce_scatter_gather.c:40-330
 *   MPIX_Comm_create_ccl       <- MPIR_RCCLcomm_init  src/util/ccl/rccl.c:21-52
 *                                 (ncclCommInitRank with a unique id the caller
 *                                  broadcasts, as rccl.c:36 does with MPIR_Bcast)
 *   MPIX_Comm_free             <- MPIR_RCCLcomm_free  src/util/ccl/rccl.c:237
 *
 * Same pairing, same operand order (MPIR_Reduce_local(tmp_recvbuf,
 * tmp_results)), same association as the reference schedules, hence the same
 * bits.  Transports:
 *   - RCCL (one process per GPU; every exchange step is one
 *     ncclGroupStart / ncclSend+ncclRecv / ncclGroupEnd on the stream, over
 *     xGMI between MI355X GPUs);
 *   - local: the ranks are threads of ONE process (one device each, or all on
 *     one device), an exchange is a stream-ordered device-to-device copy with
 *     event hand-offs -- the shared-memory analogue, also how the schedules
 *     are tested with several ranks on a single GPU;
 *   - host-local: the same with host memory and host memcpy (schedule tests on
 *     a machine without a GPU; needs a combine installed with
 *     MPIX_Comm_set_combine, since the product has no CPU compute path);
 *   - custom: a caller-supplied exchange function.
 *
 * Blocking entry points wait for their stream before returning; the _async
 * forms only enqueue (local and custom transports may block the host inside an
 * exchange until the peer rank reaches the matching step).  Return values are
 * the MPI error classes of mpix_redop.h.
 */
#ifndef MPIX_COLL_H_INCLUDED
#define MPIX_COLL_H_INCLUDED

#include <stddef.h>

#include "mpix_redop.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct MPIX_Comm_s *MPIX_Comm;

/* one point-to-point operation of an exchange step */
typedef struct {
    int peer;           /* rank in the communicator */
    int is_recv;        /* 0 send, 1 receive */
    void *buf;
    size_t bytes;
} MPIX_P2p_op;

/* transport hook: post all `nops` operations as one group; stream-ordered on
 * `stream` (ignored by host transports).  0 on success. */
typedef int (*MPIX_Exchange_fn)(void *ctx, int rank, const MPIX_P2p_op *ops, int nops,
                                void *stream);
/* combine hook, MPIX_Reduce_local_async's signature */
typedef int (*MPIX_Combine_fn)(const void *inbuf, void *inoutbuf, MPIX_Aint count,
                               MPIX_Datatype datatype, MPIX_Op op, void *stream);

/* ---- communicators ---- */
#define MPIX_CCL_UNIQUE_ID_BYTES 128
int MPIX_Ccl_get_unique_id(void *id_out);
/* collective over `size` processes; call with the HIP device already set */
int MPIX_Comm_create_ccl(int rank, int size, const void *id, MPIX_Comm *comm);
/* `size` in-process ranks; devices[r] is rank r's HIP device, or devices ==
 * NULL for the host-memory transport.  comms[r] is rank r's handle; each rank
 * must be driven by its own thread. */
int MPIX_Comm_create_local(int size, const int *devices, MPIX_Comm *comms);
/* memory kinds of a custom communicator */
#define MPIX_XPORT_DEVICE  0    /* device buffers; fn gets them as they are, stream-ordered */
#define MPIX_XPORT_HOST    1    /* host buffers (schedule tests; needs MPIX_Comm_set_combine) */
#define MPIX_XPORT_STAGED  2    /* device buffers, host transport: the library synchronises the
                                   stream, copies the send data into pinned staging memory, calls
                                   fn with HOST pointers (stream NULL) and copies what arrived
                                   back to the device buffers on the stream -- the
                                   MPIR_Coll_host_buffer_alloc / swap_back pattern
                                   (coll_impl.c:305-381) for a transport that cannot touch GPU
                                   memory (e.g. sockets, gloo) */
int MPIX_Comm_create_custom(int rank, int size, MPIX_Exchange_fn fn, void *ctx, int memory_kind,
                            MPIX_Comm *comm);
/* replace the combine (NULL restores MPIX_Reduce_local_async) */
int MPIX_Comm_set_combine(MPIX_Comm comm, MPIX_Combine_fn fn);
int MPIX_Comm_rank(MPIX_Comm comm, int *rank);
int MPIX_Comm_size(MPIX_Comm comm, int *size);
/* frees the handle; for local communicators, after every rank has freed its
 * handle the shared mailbox goes too */
int MPIX_Comm_free(MPIX_Comm comm);

/* ---- MPI_Reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op) ----
 * sendbuf holds size*recvcount elements; recvbuf recvcount.  sendbuf NULL =
 * MPI_IN_PLACE: recvbuf holds the size*recvcount inputs and gets the result
 * in its first recvcount elements (red_scat_block.c:58-70).  workspace: NULL
 * (the communicator keeps a grow-only scratch) or at least
 * MPIX_Reduce_scatter_block_workspace() bytes of the buffers' memory kind. */
#define MPIX_RSB_AUTO               0   /* generic.json: recursive halving < 512 KiB, else pairwise */
#define MPIX_RSB_RECURSIVE_HALVING  1   /* on RCCL communicators with P = 2^k >= 4 and
                                           equal blocks, each step's combine is cut along
                                           the next step's split: the half sent next on the
                                           collective's stream, the half kept on a second
                                           stream under the next exchange (half-steps of
                                           >= 1 MiB; MPIX_Comm_set_rh_overlap, or env
                                           MPIX_COLL_RH_OVERLAP=N bytes at creation, sets
                                           it for any device communicator, 0 off); same
                                           bits */
#define MPIX_RSB_PAIRWISE           2   /* the P-1 exchanges in ONE group + one multi-input combine */
#define MPIX_RSB_PAIRWISE_SEQUENTIAL 3  /* the reference's loop: P-1 sendrecv + combine steps */
#define MPIX_RSB_PAIRWISE_PIPELINED 4   /* PAIRWISE cut into 2..8 chunks (>= 4 MiB of the
                                           largest block each; below 8 MiB it is PAIRWISE):
                                           chunk k's combine, on a second stream, overlaps
                                           chunk k+1's group; same bits as PAIRWISE */
#define MPIX_RSB_PULL               5   /* fused pull + combine: ONE
                                           multi-input kernel reads this rank's block of all P-1
                                           peers over xGMI, folding them in the pairwise order:
                                           no receive buffer, same bits as PAIRWISE.  Across
                                           processes each rank copies its input into a pull
                                           window -- library-owned device memory exported once
                                           with hipIpc (as the reference's GPU ipc path maps
                                           peers, mpl_gpu_hip.c:174-204), mapped once by every
                                           peer and verified by a nonce read back through the
                                           mapping; ranks of a local communicator read each
                                           other's buffers directly.  A barrier before (inputs
                                           ready) and after (peers done reading).  A host
                                           communicator, or windows that cannot be mapped and
                                           verified on every rank, run PAIRWISE (same bits) */
#define MPIX_RSB_RECURSIVE_HALVING_MULTIPATH 6  /* RECURSIVE_HALVING's schedule and association
                                           (same bits), each step's exchange routed over all
                                           xGMI links: with P a power of two >= 4 and equal
                                           blocks, a step's half is cut into P/2 parts, one sent
                                           to the partner directly and each other relayed
                                           through a distinct third rank (first hop on link
                                           r^a, second on link r^(a^m)), the relay hops
                                           pipelined in chunks; every directed link of every
                                           rank carries 1/(P/2) of the half.  Other shapes run
                                           RECURSIVE_HALVING */
#define MPIX_RSB_RECURSIVE_HALVING_PULL 7  /* RECURSIVE_HALVING's association (same bits)
                                           computed by the pull of MPIX_RSB_PULL: every rank
                                           maps its peers' send buffers and ONE tree kernel
                                           (MPIX_Reduce_local_tree_async) reads its block of
                                           all P ranks over xGMI (pull windows, as
                                           MPIX_RSB_PULL) and folds them level by level as the
                                           log2(P) halving steps would, writing recvbuf
                                           directly.  P <= 16 (P not a power of two: the
                                           reference's pair fold is the tree's first level)
                                           and a device communicator; otherwise
                                           RECURSIVE_HALVING */
#define MPIX_RSB_LAST               MPIX_RSB_RECURSIVE_HALVING_PULL
size_t MPIX_Reduce_scatter_block_workspace(MPIX_Aint recvcount, MPIX_Datatype datatype,
                                           MPIX_Comm comm, int algorithm);
int MPIX_Reduce_scatter_block(const void *sendbuf, void *recvbuf, MPIX_Aint recvcount,
                              MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                              void *workspace, size_t workspace_bytes);
int MPIX_Reduce_scatter_block_async(const void *sendbuf, void *recvbuf, MPIX_Aint recvcount,
                                    MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm,
                                    int algorithm, void *workspace, size_t workspace_bytes,
                                    void *stream);

/* ---- MPI_Reduce_scatter(sendbuf, recvbuf, recvcounts, datatype, op) ----
 * (src/mpi/coll/reduce_scatter/reduce_scatter_intra_{recursive_halving,
 * pairwise}.c): rank i's result block has recvcounts[i] elements (zeros
 * allowed; size entries, host array); sendbuf holds sum(recvcounts)
 * elements, NULL = MPI_IN_PLACE (recvbuf holds them and gets the result in
 * its first recvcounts[rank] elements).  Algorithms and the auto switch
 * (512 KiB of total message, generic.json:277-291) as for the _block form. */
size_t MPIX_Reduce_scatter_workspace(const MPIX_Aint *recvcounts, MPIX_Datatype datatype,
                                     MPIX_Comm comm, int algorithm);
int MPIX_Reduce_scatter(const void *sendbuf, void *recvbuf, const MPIX_Aint *recvcounts,
                        MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                        void *workspace, size_t workspace_bytes);
int MPIX_Reduce_scatter_async(const void *sendbuf, void *recvbuf, const MPIX_Aint *recvcounts,
                              MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                              void *workspace, size_t workspace_bytes, void *stream);

/* ---- MPI_Reduce(sendbuf, recvbuf, count, datatype, op, root) ----
 * (src/mpi/coll/reduce/reduce_intra_{binomial,reduce_scatter_gather}.c):
 * recvbuf is significant at the root only; the root's sendbuf NULL =
 * MPI_IN_PLACE.  Non-root ranks accumulate in the workspace (NULL: the
 * communicator's scratch; else >= MPIX_Reduce_workspace() bytes). */
#define MPIX_REDUCE_AUTO            0   /* generic.json:206-250: binomial up to 2 KiB or count < pof2 */
#define MPIX_REDUCE_BINOMIAL        1
#define MPIX_REDUCE_SCATTER_GATHER  2   /* Rabenseifner: reduce-scatter + binomial gather; count >= pof2 */
size_t MPIX_Reduce_workspace(MPIX_Aint count, MPIX_Datatype datatype, int root, MPIX_Comm comm);
int MPIX_Reduce(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                MPIX_Op op, int root, MPIX_Comm comm, int algorithm, void *workspace,
                size_t workspace_bytes);
int MPIX_Reduce_async(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                      MPIX_Op op, int root, MPIX_Comm comm, int algorithm, void *workspace,
                      size_t workspace_bytes, void *stream);

/* ---- MPI_Scan / MPI_Exscan(sendbuf, recvbuf, count, datatype, op) ----
 * (src/mpi/coll/scan/scan_intra_recursive_doubling.c:60-150,
 * src/mpi/coll/exscan/exscan_intra_recursive_doubling.c:60-160): sendbuf
 * NULL = MPI_IN_PLACE; Exscan leaves rank 0's recvbuf untouched.  workspace:
 * NULL or >= MPIX_Scan_workspace() bytes (partial scan + incoming buffer). */
size_t MPIX_Scan_workspace(MPIX_Aint count, MPIX_Datatype datatype, MPIX_Comm comm);
int MPIX_Scan(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
              MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes);
int MPIX_Scan_async(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                    MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes,
                    void *stream);
int MPIX_Exscan(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes);
int MPIX_Exscan_async(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                      MPIX_Op op, MPIX_Comm comm, void *workspace, size_t workspace_bytes,
                      void *stream);

/* ---- MPI_Allreduce(sendbuf, recvbuf, count, datatype, op) ----
 * sendbuf NULL = MPI_IN_PLACE (recvbuf holds the input). */
#define MPIX_ALLREDUCE_AUTO                 0   /* generic.json:99-135: recursive doubling up to
                                                   8 bytes or below pof2 elements, else
                                                   reduce-scatter+allgather */
#define MPIX_ALLREDUCE_RECURSIVE_DOUBLING   1
#define MPIX_ALLREDUCE_REDUCE_SCATTER_ALLGATHER 2  /* allgather as ONE group of direct exchanges */
#define MPIX_ALLREDUCE_RSAG_RD_ALLGATHER    3   /* the reference's log2(P) allgather steps */
#define MPIX_ALLREDUCE_RING                 4   /* allreduce_intra_ring.c: ring reduce-scatter
                                                   (P-1 steps) + allgather of the blocks */
#define MPIX_ALLREDUCE_RSAG_MULTIPATH       5   /* REDUCE_SCATTER_ALLGATHER with every
                                                   reduce-scatter step spread over all links
                                                   through relays (P a power of two >= 4,
                                                   count a multiple of P; else plain steps;
                                                   a step too small for the relay slots runs
                                                   plain, and a call none of whose steps
                                                   could use the relays counts as
                                                   REDUCE_SCATTER_ALLGATHER); same bits */
#define MPIX_ALLREDUCE_PULL                 6   /* REDUCE_SCATTER_ALLGATHER's association (same
                                                   bits) as two pulls (pull windows, as
                                                   MPIX_RSB_PULL): ONE tree kernel reads this
                                                   rank's block of every rank's input
                                                   (MPIX_Reduce_local_tree_async), then ONE copy
                                                   kernel reads every peer's finished block
                                                   (MPIX_Copy_multi_async); no workspace.  P <= 16
                                                   (P not a power of two: the reference's pair
                                                   fold first) on a device communicator, else
                                                   REDUCE_SCATTER_ALLGATHER */
#define MPIX_ALLREDUCE_LAST                 MPIX_ALLREDUCE_PULL
size_t MPIX_Allreduce_workspace(MPIX_Aint count, MPIX_Datatype datatype, MPIX_Comm comm);
int MPIX_Allreduce(const void *sendbuf, void *recvbuf, MPIX_Aint count, MPIX_Datatype datatype,
                   MPIX_Op op, MPIX_Comm comm, int algorithm, void *workspace,
                   size_t workspace_bytes);
int MPIX_Allreduce_async(const void *sendbuf, void *recvbuf, MPIX_Aint count,
                         MPIX_Datatype datatype, MPIX_Op op, MPIX_Comm comm, int algorithm,
                         void *workspace, size_t workspace_bytes, void *stream);

/* stream the blocking forms use: the communicator's own (NULL) by default */
int MPIX_Comm_set_stream(MPIX_Comm comm, void *stream);

/* Largest single message the transport is handed: a schedule's message above
 * `bytes` is posted as several consecutive messages to the same peer in the
 * same exchange group (both sides split identically, so the k-th send of a
 * pair matches its k-th receive in posting order, equal sizes).  Default 1 GiB
 * on RCCL communicators (no count reaches 2^31; 0 or more than 1 GiB is refused
 * there), 0 = never split on the others. */
int MPIX_Comm_set_max_message(MPIX_Comm comm, MPIX_Aint bytes);

/* Smallest half-step (bytes) whose combine MPIX_RSB_RECURSIVE_HALVING cuts
 * along the next step's split and runs under the next exchange (see
 * MPIX_RSB_RECURSIVE_HALVING): 0 = never, -1 = the value the communicator
 * was created with.  A communicator starts with env MPIX_COLL_RH_OVERLAP (read
 * once, at creation) or, without it, its kind's default (1 MiB on RCCL
 * communicators, off on the others).  Local, not collective: every rank of a communicator must
 * set the same value before the collective (the split changes only which
 * stream runs a combine, never the bits). */
int MPIX_Comm_set_rh_overlap(MPIX_Comm comm, MPIX_Aint min_bytes);
int MPIX_Comm_get_rh_overlap(MPIX_Comm comm, MPIX_Aint *min_bytes);

/* Stream-ordered barrier: one 1-byte message to and from every peer on the
 * transport (on RCCL the stream passes it only once every peer's stream has
 * reached its own barrier). */
int MPIX_Comm_barrier(MPIX_Comm comm);

/* Symmetric device memory for the pull schedules (as NCCL's registered user
 * buffers): every rank calls MPIX_Comm_alloc_shared together with the same
 * `bytes`; each gets `bytes` of device memory that is exported once, mapped
 * by every peer and verified through the mapping (the nonce check of the
 * pull windows).  A pull schedule (MPIX_RSB_PULL,
 * MPIX_RSB_RECURSIVE_HALVING_PULL, MPIX_ALLREDUCE_PULL) whose buffers lie in
 * such memory at the same offset on every rank reads the peers' copies in
 * place, without first copying its input into the pull window.  Collective;
 * MPI_ERR_OTHER on every rank if no verified mapping could be made.
 * MPIX_Comm_free_shared is collective too; the memory itself is released by
 * MPIX_Comm_free.
 *
 * Device memory a communicator keeps until MPIX_Comm_free (so that a freed
 * allocation's identity never comes back while a peer may still hold a
 * mapping of it -- DESIGN.md, "Why windows"): shared allocations after
 * MPIX_Comm_free_shared; pull windows that failed verification (at most 3
 * per growth, each header + message size); outgrown pull windows (growth
 * doubles, so at most the final window's size again).  A communicator whose
 * ranks are not all on one node (host name and boot id exchanged once,
 * before the first window) allocates no window at all and runs the pulls'
 * transport forms. */
int MPIX_Comm_alloc_shared(MPIX_Comm comm, size_t bytes, void **ptr);
int MPIX_Comm_free_shared(MPIX_Comm comm, void *ptr);

/* Per-step breakdown of the device schedules: with
 * timing on, every exchange and combine step of the next collectives records
 * a HIP event on the collective's stream; MPIX_Comm_step_times() (after the
 * stream has completed) returns the device time between consecutive marks
 * and the label of the step that ended at each (`labels` may be NULL; each
 * label at most 32 bytes with its NUL) and clears the record.  Device
 * communicators only. */
/* Which schedule actually ran -- an explicitly requested algorithm may not be
 * able to run (a pull whose windows failed verification on some rank, a
 * device pair without peer access, MULTIPATH on a shape it does not cover or
 * with every step too small for its relay slots), in which case the schedule with
 * the same bits runs instead; this is how a caller tells.  pulls_enabled: 1
 * while the pull schedules can run on this communicator (0 once it is known to
 * span nodes; before the first pull that is not yet known and counts as 1);
 * last_rs_algorithm / last_allreduce_algorithm: the MPIX_RSB_* /
 * MPIX_ALLREDUCE_* value of the schedule the last reduce-scatter / allreduce
 * ran (AUTO resolved; -1 before the first); window_retries: pull-window
 * verification attempts that failed so far; fallbacks: calls whose requested
 * schedule did not run.  Any pointer may be NULL.  Local, not collective. */
int MPIX_Comm_get_state(MPIX_Comm comm, int *pulls_enabled, int *last_rs_algorithm,
                        int *last_allreduce_algorithm, int *window_retries, int *fallbacks);

int MPIX_Comm_set_step_timing(MPIX_Comm comm, int enable);
int MPIX_Comm_step_times(MPIX_Comm comm, double *ms, char (*labels)[32], int max, int *n);

#ifdef __cplusplus
}
#endif
#endif /* MPIX_COLL_H_INCLUDED */
