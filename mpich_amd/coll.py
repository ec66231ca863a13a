"""MPI collectives on torch.distributed process groups, run by libmpix_coll.

This module holds no schedule of its own: every call goes to the C++ host
schedules of libmpix_coll.so (include/mpix_coll.h), which restate MPICH's
reduce-scatter / allreduce algorithms index for index and combine every
received chunk with the HIP kernels of libmpix_redop.so.  What it adds is the
communicator for a process group:

  * backend "nccl" (RCCL on ROCm) and device tensors: an RCCL communicator of
    its own (MPIX_Comm_create_ccl, bootstrapped over the group as
    MPIR_RCCLcomm_init does with MPIR_Bcast, rccl.c:21-52); every exchange
    step is one ncclGroupStart / ncclSend + ncclRecv / ncclGroupEnd over xGMI;
  * any other backend (gloo): a custom communicator whose exchange function
    posts the step's sends and receives as one torch.distributed
    batch_isend_irecv group -- on host tensors directly (MPIX_XPORT_HOST; the
    caller installs a combine, the product has no CPU compute path), on device
    tensors through the library's pinned staging (MPIX_XPORT_STAGED, the
    MPIR_Coll_host_buffer_alloc pattern), so the C++ schedules and the HIP
    combine run multi-process on any box.

Reference algorithms (all in src/mpi/coll/):
  recursive_halving   reduce_scatter_block/..._intra_recursive_halving.c:38-260
  pairwise(_sequential) reduce_scatter_block/..._intra_pairwise.c:42-104
  pull                the pairwise order, read from hipIpc-mapped peer buffers
                      by one fused kernel (mpl_gpu_hip.c:174-204)
  allreduce           allreduce/allreduce_intra_reduce_scatter_allgather.c:41-277,
                      allreduce/allreduce_intra_recursive_doubling.c:24-150
"""
import os

import torch
import torch.distributed as dist

from . import ccl
from . import redop

# largest single message handed to gloo, as on RCCL: libmpix_coll splits
# bigger ones into several same-peer messages of one group
# (MPIX_Comm_set_max_message) before the exchange function sees them
MAX_MSG_BYTES = 1 << 30

_comms = {}


def _gloo_exchange(group):
    """exchange function of a custom communicator: one batch_isend_irecv
    group per schedule step, over host memory"""
    g2l = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)

    def fn(rank, ops):
        import ctypes
        p2p = []
        for peer, is_recv, addr, nbytes in ops:
            t = torch.frombuffer((ctypes.c_char * nbytes).from_address(addr), dtype=torch.uint8)
            p2p.append(dist.P2POp(dist.irecv if is_recv else dist.isend, t, g2l(peer),
                                  group=group))
        for w in dist.batch_isend_irecv(p2p):
            w.wait()
        return 0
    return fn


def comm_for(group=None, device=True):
    """the libmpix_coll communicator of `group` for device (True) or host
    (False) buffers, created once per (group, kind)"""
    key = (group, bool(device))         # the group object itself: an id() could be reused
    c = _comms.get(key)
    if c is None:
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        if device and dist.get_backend(group) == 'nccl':
            c = ccl.comm_create_ccl_from_process_group(group)
        else:
            c = ccl.comm_create_custom(rank, size, _gloo_exchange(group),
                                       ccl.XPORT_STAGED if device else ccl.XPORT_HOST)
            c.set_max_message(MAX_MSG_BYTES)
        _comms[key] = c
    return c


def free_comms():
    """free every communicator this module created (before the process
    group is destroyed)"""
    for c in _comms.values():
        c.free()
    _comms.clear()


def _is_device(*bufs):
    for b in bufs:
        if isinstance(b, torch.Tensor):
            return b.is_cuda
    return True


def _order_after_torch(comm, dev):
    """order the blocking collective after the torch work that produced its
    inputs (torch semantics; an MPI caller synchronises its own streams
    first).  A side stream of torch's is handed to the communicator; torch's
    default stream is the legacy NULL stream, which the communicator's own
    non-blocking stream does not wait for (and a NULL handle means "own
    stream" to MPIX_Comm_set_stream), so that one is synchronised instead."""
    if not dev:
        return
    cs = torch.cuda.current_stream()
    if cs.cuda_stream:
        comm.set_stream(cs)
    else:
        cs.synchronize()
        comm.set_stream(None)


def reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, group=None,
                         algorithm='recursive_halving', combine=None, workspace=None, timer=None):
    """MPI_Reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, comm).

    sendbuf holds size*recvcount elements, recvbuf recvcount; sendbuf None is
    MPI_IN_PLACE (recvbuf holds the inputs, the result lands in its first
    block).  algorithm: recursive_halving | pairwise | pairwise_sequential |
    pairwise_pipelined | pull | recursive_halving_multipath |
    recursive_halving_pull | auto.  combine: C combine address for host
    buffers (no CPU compute path here).  timer: a list that receives the
    per-step breakdown [{'phase', 'ms'}] of this call (device buffers).
    Raises RedopError on an MPI error class."""
    dev = _is_device(recvbuf, sendbuf)
    if not dev and combine is None:
        raise ValueError('host buffers need a combine function: the product path is the HIP '
                         'kernel (device buffers)')
    c = comm_for(group, dev)
    c.set_combine(combine)
    _order_after_torch(c, dev)
    if timer is not None:
        c.set_step_timing(True)
    try:
        redop.check(ccl.reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, c,
                                             algorithm, workspace=workspace),
                    'MPIX_Reduce_scatter_block')
    finally:
        if timer is not None:
            c.set_step_timing(False)
            timer.extend(c.step_times() if dev else [])
    return recvbuf


def reduce_scatter(sendbuf, recvbuf, recvcounts, datatype, op, group=None, algorithm='auto',
                   combine=None, workspace=None):
    """MPI_Reduce_scatter with per-rank recvcounts (zeros allowed); sendbuf
    None is MPI_IN_PLACE.  Same schedules and rules as reduce_scatter_block."""
    dev = _is_device(recvbuf, sendbuf)
    if not dev and combine is None:
        raise ValueError('host buffers need a combine function')
    c = comm_for(group, dev)
    c.set_combine(combine)
    _order_after_torch(c, dev)
    redop.check(ccl.reduce_scatter(sendbuf, recvbuf, list(recvcounts), datatype, op, c, algorithm,
                                   workspace=workspace), 'MPIX_Reduce_scatter')
    return recvbuf


def reduce_scatter_block_pairwise(sendbuf, recvbuf, recvcount, datatype, op, group=None,
                                  concurrent=True, **kw):
    """the reference's pairwise exchange: all P-1 exchanges as one group
    (concurrent) or its sequential loop"""
    return reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, group=group,
                                algorithm='pairwise' if concurrent else 'pairwise_sequential', **kw)


def reduce_scatter_block_pull(sendbuf, recvbuf, recvcount, datatype, op, group=None, **kw):
    """fused pull + combine over hipIpc-mapped peer buffers (device tensors
    from the caching allocator, i.e. hipMalloc)"""
    return reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, group=group,
                                algorithm='pull', **kw)


ALGORITHMS = {'recursive_halving': reduce_scatter_block,
              'pairwise': reduce_scatter_block_pairwise,
              'pull': reduce_scatter_block_pull}


def reduce_scatter_block_auto(sendbuf, recvbuf, recvcount, datatype, op, group=None, **kw):
    """MPIR_CVAR_REDUCE_SCATTER_BLOCK_INTRA_ALGORITHM (cvars.txt:1712-1726):
    env value recursive_halving | pairwise, else `auto` (generic.json:316-341,
    decided in C: recursive halving below 512 KiB of total message)"""
    algo = os.environ.get('MPIR_CVAR_REDUCE_SCATTER_BLOCK_INTRA_ALGORITHM', 'auto')
    if algo not in ('recursive_halving', 'pairwise'):
        algo = 'auto'
    return reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, group=group,
                                algorithm=algo, **kw)


def allreduce(sendbuf, recvbuf, count, datatype, op, group=None, combine=None, workspace=None,
              allgather='direct', algorithm=None):
    """MPI_Allreduce by reduce-scatter + allgather (Rabenseifner).
    allgather 'direct' = one group of P-1 direct exchanges, 'recursive_doubling'
    = the reference's log2(P) steps (:191-226); same bits either way.
    algorithm overrides: auto | recursive_doubling | reduce_scatter_allgather |
    rsag_rd_allgather | ring | rsag_multipath (each reduce-scatter step over
    every link through relays; same bits).  sendbuf None = MPI_IN_PLACE."""
    if algorithm is None:
        if allgather not in ('direct', 'recursive_doubling'):
            raise ValueError('allgather must be direct or recursive_doubling')
        algorithm = 'reduce_scatter_allgather' if allgather == 'direct' else 'rsag_rd_allgather'
    dev = _is_device(recvbuf, sendbuf)
    if not dev and combine is None:
        raise ValueError('host buffers need a combine function')
    c = comm_for(group, dev)
    c.set_combine(combine)
    _order_after_torch(c, dev)
    redop.check(ccl.allreduce(sendbuf, recvbuf, count, datatype, op, c, algorithm,
                              workspace=workspace), 'MPIX_Allreduce')
    return recvbuf


def allreduce_recursive_doubling(sendbuf, recvbuf, count, datatype, op, group=None, **kw):
    return allreduce(sendbuf, recvbuf, count, datatype, op, group=group,
                     algorithm='recursive_doubling', **kw)


def allreduce_auto(sendbuf, recvbuf, count, datatype, op, group=None, **kw):
    """MPIR_CVAR_ALLREDUCE_INTRA_ALGORITHM or, by default, generic.json:99-135
    (decided in C)"""
    algo = os.environ.get('MPIR_CVAR_ALLREDUCE_INTRA_ALGORITHM', 'auto')
    if algo not in ('recursive_doubling', 'reduce_scatter_allgather'):
        algo = 'auto'
    return allreduce(sendbuf, recvbuf, count, datatype, op, group=group, algorithm=algo, **kw)
