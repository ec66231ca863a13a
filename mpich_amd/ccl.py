"""Host-side binding of libmpix_coll.so (include/mpix_coll.h): the
reduce-scatter / allreduce schedules of MPICH in C++ host code, combining
through the HIP kernels of libmpix_redop.so, over RCCL (one process per GPU)
or the in-process transports (ranks as threads of one process).

Mirrors the reference interface: MPI_Reduce_scatter_block(sendbuf, recvbuf,
recvcount, datatype, op, comm) and MPI_Allreduce(sendbuf, recvbuf, count,
datatype, op, comm) with MPI error classes as return values; `comm` is a
`Comm` created here.  Like redop.py this module computes nothing itself and
fails loudly if the library is missing.
"""
import ctypes
import os

import torch  # noqa: F401  (one HIP runtime per process: torch's)

from . import handles as H
from . import redop

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libmpix_coll.so')
UNIQUE_ID_BYTES = 128

RSB_AUTO, RSB_RECURSIVE_HALVING, RSB_PAIRWISE, RSB_PAIRWISE_SEQUENTIAL = 0, 1, 2, 3
RSB_PAIRWISE_PIPELINED, RSB_PULL, RSB_RECURSIVE_HALVING_MULTIPATH = 4, 5, 6
RSB_RECURSIVE_HALVING_PULL = 7
RSB_ALGORITHMS = {'auto': RSB_AUTO, 'recursive_halving': RSB_RECURSIVE_HALVING,
                  'pairwise': RSB_PAIRWISE, 'pairwise_sequential': RSB_PAIRWISE_SEQUENTIAL,
                  'pairwise_pipelined': RSB_PAIRWISE_PIPELINED, 'pull': RSB_PULL,
                  'recursive_halving_multipath': RSB_RECURSIVE_HALVING_MULTIPATH,
                  'recursive_halving_pull': RSB_RECURSIVE_HALVING_PULL}
XPORT_DEVICE, XPORT_HOST, XPORT_STAGED = 0, 1, 2
AR_AUTO, AR_RECURSIVE_DOUBLING, AR_RSAG, AR_RSAG_RD, AR_RING, AR_RSAG_MULTIPATH = 0, 1, 2, 3, 4, 5
AR_PULL = 6
AR_ALGORITHMS = {'auto': AR_AUTO, 'recursive_doubling': AR_RECURSIVE_DOUBLING,
                 'reduce_scatter_allgather': AR_RSAG, 'rsag_rd_allgather': AR_RSAG_RD,
                 'ring': AR_RING, 'rsag_multipath': AR_RSAG_MULTIPATH, 'pull': AR_PULL}

_lib = None

COMBINE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ssize_t,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p)


class P2pOp(ctypes.Structure):
    """MPIX_P2p_op"""
    _fields_ = [('peer', ctypes.c_int), ('is_recv', ctypes.c_int), ('buf', ctypes.c_void_p),
                ('bytes', ctypes.c_size_t)]


EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(P2pOp),
                               ctypes.c_int, ctypes.c_void_p)


def lib():
    global _lib
    if _lib is None:
        redop.lib()                     # libmpix_redop.so first (RTLD_GLOBAL)
        if not os.path.exists(LIB_PATH):
            raise ImportError('libmpix_coll.so is not built (%s); run `make -C mpich_amd/csrc`'
                              % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, aint, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_ssize_t, ctypes.c_size_t
        sig = {
            'MPIX_Ccl_get_unique_id': ([vp], i32),
            'MPIX_Comm_create_ccl': ([i32, i32, vp, ctypes.POINTER(vp)], i32),
            'MPIX_Comm_create_local': ([i32, ctypes.POINTER(i32), ctypes.POINTER(vp)], i32),
            'MPIX_Comm_create_custom': ([i32, i32, vp, vp, i32, ctypes.POINTER(vp)], i32),
            'MPIX_Comm_set_combine': ([vp, vp], i32),
            'MPIX_Comm_set_stream': ([vp, vp], i32),
            'MPIX_Comm_set_max_message': ([vp, ctypes.c_ssize_t], i32),
            'MPIX_Comm_set_rh_overlap': ([vp, ctypes.c_ssize_t], i32),
            'MPIX_Comm_get_rh_overlap': ([vp, ctypes.POINTER(ctypes.c_ssize_t)], i32),
            'MPIX_Comm_barrier': ([vp], i32),
            'MPIX_Comm_alloc_shared': ([vp, sz, ctypes.POINTER(vp)], i32),
            'MPIX_Comm_free_shared': ([vp, vp], i32),
            'MPIX_Comm_set_step_timing': ([vp, i32], i32),
            'MPIX_Comm_get_state': ([vp] + [ctypes.POINTER(i32)] * 5, i32),
            'MPIX_Comm_step_times': ([vp, ctypes.POINTER(ctypes.c_double), vp, i32,
                                      ctypes.POINTER(i32)], i32),
            'MPIX_Comm_rank': ([vp, ctypes.POINTER(i32)], i32),
            'MPIX_Comm_size': ([vp, ctypes.POINTER(i32)], i32),
            'MPIX_Comm_free': ([vp], i32),
            'MPIX_Reduce_scatter_block_workspace': ([aint, i32, vp, i32], sz),
            'MPIX_Reduce_scatter_block': ([vp, vp, aint, i32, i32, vp, i32, vp, sz], i32),
            'MPIX_Reduce_scatter_block_async': ([vp, vp, aint, i32, i32, vp, i32, vp, sz, vp],
                                                i32),
            'MPIX_Reduce_scatter_workspace': ([ctypes.POINTER(aint), i32, vp, i32], sz),
            'MPIX_Reduce_scatter': ([vp, vp, ctypes.POINTER(aint), i32, i32, vp, i32, vp, sz],
                                    i32),
            'MPIX_Reduce_scatter_async': ([vp, vp, ctypes.POINTER(aint), i32, i32, vp, i32, vp,
                                           sz, vp], i32),
            'MPIX_Reduce_workspace': ([aint, i32, i32, vp], sz),
            'MPIX_Reduce': ([vp, vp, aint, i32, i32, i32, vp, i32, vp, sz], i32),
            'MPIX_Reduce_async': ([vp, vp, aint, i32, i32, i32, vp, i32, vp, sz, vp], i32),
            'MPIX_Scan_workspace': ([aint, i32, vp], sz),
            'MPIX_Scan': ([vp, vp, aint, i32, i32, vp, vp, sz], i32),
            'MPIX_Scan_async': ([vp, vp, aint, i32, i32, vp, vp, sz, vp], i32),
            'MPIX_Exscan': ([vp, vp, aint, i32, i32, vp, vp, sz], i32),
            'MPIX_Exscan_async': ([vp, vp, aint, i32, i32, vp, vp, sz, vp], i32),
            'MPIX_Allreduce_workspace': ([aint, i32, vp], sz),
            'MPIX_Allreduce': ([vp, vp, aint, i32, i32, vp, i32, vp, sz], i32),
            'MPIX_Allreduce_async': ([vp, vp, aint, i32, i32, vp, i32, vp, sz, vp], i32),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def _addr(buf):
    return redop._addr(buf)


def _ws(workspace):
    """(address, bytes) of an optional workspace tensor / array"""
    if workspace is None:
        return None, 0
    nb = redop._nbytes(workspace)
    return _addr(workspace), (nb if nb is not None else 0)


def _fits(datatype, op, *pairs):
    """every (buffer, element count) pair: the tensor / array holds that many
    elements (redop._span_check; None buffers and raw pointers pass)"""
    for buf, n in pairs:
        if buf is not None:
            redop._span_check(int(n), datatype, op, buf)


class Comm:
    """One rank's handle of a libmpix_coll communicator."""

    def __init__(self, handle):
        self.h = ctypes.c_void_p(handle)
        r, s = ctypes.c_int(), ctypes.c_int()
        lib().MPIX_Comm_rank(self.h, ctypes.byref(r))
        lib().MPIX_Comm_size(self.h, ctypes.byref(s))
        self.rank, self.size = r.value, s.value
        self._keep = []

    def set_combine(self, fn):
        """install a combine function pointer (an int address, e.g. a C
        symbol of the test oracle) or None for the HIP kernel"""
        redop.check(lib().MPIX_Comm_set_combine(self.h, fn), 'MPIX_Comm_set_combine')

    def set_stream(self, stream):
        redop.check(lib().MPIX_Comm_set_stream(self.h, None if stream is None else
                                               redop._stream_ptr(stream)), 'MPIX_Comm_set_stream')

    def set_max_message(self, nbytes):
        """MPIX_Comm_set_max_message: messages above nbytes go as several
        same-peer messages in one exchange group (0: never split)"""
        redop.check(lib().MPIX_Comm_set_max_message(self.h, nbytes), 'MPIX_Comm_set_max_message')

    def set_rh_overlap(self, min_bytes):
        """MPIX_Comm_set_rh_overlap: smallest recursive-halving half-step whose
        combine runs under the next exchange (0 never, -1 the communicator
        kind's default: 1 MiB on RCCL, off elsewhere); same bits either way"""
        redop.check(lib().MPIX_Comm_set_rh_overlap(self.h, min_bytes), 'MPIX_Comm_set_rh_overlap')

    def rh_overlap(self):
        v = ctypes.c_ssize_t()
        redop.check(lib().MPIX_Comm_get_rh_overlap(self.h, ctypes.byref(v)),
                    'MPIX_Comm_get_rh_overlap')
        return v.value

    def barrier(self):
        redop.check(lib().MPIX_Comm_barrier(self.h), 'MPIX_Comm_barrier')

    def alloc_shared(self, nbytes):
        """collective MPIX_Comm_alloc_shared: the device address of `nbytes` of
        symmetric memory the pull schedules read in place"""
        p = ctypes.c_void_p()
        redop.check(lib().MPIX_Comm_alloc_shared(self.h, nbytes, ctypes.byref(p)),
                    'MPIX_Comm_alloc_shared')
        return p.value

    def shared_tensor(self, numel, dtype):
        """a torch tensor over fresh shared memory of `numel` elements
        (collective; the memory lives until free_shared / free)"""
        import torch
        esize = torch.empty((), dtype=dtype).element_size()
        ptr = self.alloc_shared(numel * esize)
        typestr = {torch.float32: '<f4', torch.float64: '<f8', torch.int32: '<i4',
                   torch.int64: '<i8', torch.uint8: '|u1'}[dtype]

        class _Dev:     # __cuda_array_interface__ v3: how torch adopts device memory
            __cuda_array_interface__ = {'shape': (numel,), 'typestr': typestr,
                                        'data': (ptr, False), 'version': 3}
        t = torch.as_tensor(_Dev(), device='cuda')
        assert t.data_ptr() == ptr
        return t

    def free_shared(self, ptr):
        """collective MPIX_Comm_free_shared (an address from alloc_shared or a
        shared_tensor's data_ptr())"""
        redop.check(lib().MPIX_Comm_free_shared(self.h, ptr), 'MPIX_Comm_free_shared')

    def set_step_timing(self, enable=True):
        redop.check(lib().MPIX_Comm_set_step_timing(self.h, 1 if enable else 0),
                    'MPIX_Comm_set_step_timing')

    def step_times(self, max_steps=64):
        """[{'phase': label, 'ms': t}] since timing was switched on (device
        communicators; waits for the recorded events)"""
        ms = (ctypes.c_double * max_steps)()
        labels = ctypes.create_string_buffer(32 * max_steps)
        n = ctypes.c_int()
        redop.check(lib().MPIX_Comm_step_times(self.h, ms, labels, max_steps, ctypes.byref(n)),
                    'MPIX_Comm_step_times')
        raw = labels.raw
        return [dict(phase=raw[32 * k:32 * (k + 1)].split(b'\0', 1)[0].decode(),
                     ms=round(ms[k], 4)) for k in range(n.value)]

    def state(self):
        """MPIX_Comm_get_state: which schedule the last collectives actually
        ran (names from RSB_ALGORITHMS / AR_ALGORITHMS, None before the
        first), whether the pulls can run, failed window verifications and
        calls whose requested schedule did not run"""
        v = [ctypes.c_int() for _ in range(5)]
        redop.check(lib().MPIX_Comm_get_state(self.h, *[ctypes.byref(x) for x in v]),
                    'MPIX_Comm_get_state')
        rs_names = {n: k for k, n in RSB_ALGORITHMS.items()}
        ar_names = {n: k for k, n in AR_ALGORITHMS.items()}
        return dict(pulls_enabled=bool(v[0].value), last_rs=rs_names.get(v[1].value),
                    last_allreduce=ar_names.get(v[2].value), window_retries=v[3].value,
                    fallbacks=v[4].value)

    def free(self):
        if self.h:
            rc = lib().MPIX_Comm_free(self.h)
            self.h = None
            return rc
        return 0


def get_unique_id():
    b = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    redop.check(lib().MPIX_Ccl_get_unique_id(b), 'MPIX_Ccl_get_unique_id')
    return b.raw


def comm_create_ccl(rank, size, unique_id):
    """RCCL communicator (MPIR_RCCLcomm_init, rccl.c:21-52): rank 0's
    get_unique_id() must reach every rank first (the reference bcasts it)."""
    h = ctypes.c_void_p()
    redop.check(lib().MPIX_Comm_create_ccl(rank, size, unique_id, ctypes.byref(h)),
                'MPIX_Comm_create_ccl')
    return Comm(h.value)


def comm_create_ccl_from_process_group(group=None):
    """convenience: bootstrap the RCCL communicator over an initialised
    torch.distributed process group (the role MPIR_Bcast plays in rccl.c:36)"""
    import torch.distributed as dist
    rank, size = dist.get_rank(group), dist.get_world_size(group)
    obj = [get_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group else 0,
                               group=group)
    return comm_create_ccl(rank, size, obj[0])


def comm_create_custom(rank, size, exchange, memory_kind=XPORT_DEVICE):
    """communicator over a caller transport: `exchange(rank, ops)` gets a list
    of (peer, is_recv, address, bytes) and moves them as one group (host
    addresses for XPORT_HOST / XPORT_STAGED); it returns 0 on success"""
    def tramp(ctx, r, ops, nops, stream):
        try:
            return int(exchange(r, [(ops[i].peer, ops[i].is_recv, ops[i].buf, ops[i].bytes)
                                    for i in range(nops)]) or 0)
        except Exception:           # never let an exception unwind through C
            import traceback
            traceback.print_exc()
            return 1
    cb = EXCHANGE_FN(tramp)
    h = ctypes.c_void_p()
    redop.check(lib().MPIX_Comm_create_custom(rank, size, ctypes.cast(cb, ctypes.c_void_p), None,
                                               memory_kind, ctypes.byref(h)),
                'MPIX_Comm_create_custom')
    c = Comm(h.value)
    c._keep.append(cb)
    return c


def comm_create_local(size, devices=None):
    """`size` in-process ranks (drive each from its own thread); devices=None
    is the host-memory transport (needs set_combine: no CPU compute path)."""
    hs = (ctypes.c_void_p * size)()
    devs = None if devices is None else (ctypes.c_int * size)(*devices)
    redop.check(lib().MPIX_Comm_create_local(size, devs, hs), 'MPIX_Comm_create_local')
    return [Comm(hs[r]) for r in range(size)]


def reduce_scatter_block(sendbuf, recvbuf, recvcount, datatype, op, comm, algorithm='auto',
                         workspace=None, stream=None, blocking=True):
    """MPI_Reduce_scatter_block; returns the MPI error class."""
    a = RSB_ALGORITHMS[algorithm] if isinstance(algorithm, str) else algorithm
    ws, wsb = _ws(workspace)
    total = recvcount * comm.size
    _fits(datatype, op, (sendbuf, total), (recvbuf, total if sendbuf is None else recvcount))
    if blocking:
        return lib().MPIX_Reduce_scatter_block(_addr(sendbuf), _addr(recvbuf), recvcount,
                                               H.as_c_int(datatype), H.as_c_int(op), comm.h, a,
                                               ws, wsb)
    return lib().MPIX_Reduce_scatter_block_async(_addr(sendbuf), _addr(recvbuf), recvcount,
                                                 H.as_c_int(datatype), H.as_c_int(op), comm.h, a,
                                                 ws, wsb, redop._stream_ptr(stream))


def reduce_scatter(sendbuf, recvbuf, recvcounts, datatype, op, comm, algorithm='auto',
                   workspace=None, stream=None, blocking=True):
    """MPI_Reduce_scatter with per-rank recvcounts (sendbuf None =
    MPI_IN_PLACE); returns the MPI error class."""
    a = RSB_ALGORITHMS[algorithm] if isinstance(algorithm, str) else algorithm
    ws, wsb = _ws(workspace)
    cnts = (ctypes.c_ssize_t * len(recvcounts))(*recvcounts)
    if len(recvcounts) == comm.size and all(c >= 0 for c in recvcounts):
        total = sum(recvcounts)
        _fits(datatype, op, (sendbuf, total),
              (recvbuf, total if sendbuf is None else recvcounts[comm.rank]))
    if blocking:
        return lib().MPIX_Reduce_scatter(_addr(sendbuf), _addr(recvbuf), cnts,
                                         H.as_c_int(datatype), H.as_c_int(op), comm.h, a, ws, wsb)
    return lib().MPIX_Reduce_scatter_async(_addr(sendbuf), _addr(recvbuf), cnts,
                                           H.as_c_int(datatype), H.as_c_int(op), comm.h, a, ws,
                                           wsb, redop._stream_ptr(stream))


REDUCE_ALGORITHMS = {'auto': 0, 'binomial': 1, 'reduce_scatter_gather': 2}


def reduce(sendbuf, recvbuf, count, datatype, op, root, comm, algorithm='auto', workspace=None,
           stream=None, blocking=True):
    """MPI_Reduce to `root` (the root's sendbuf None = MPI_IN_PLACE; recvbuf
    only significant at the root); returns the MPI error class."""
    a = REDUCE_ALGORITHMS[algorithm] if isinstance(algorithm, str) else algorithm
    ws, wsb = _ws(workspace)
    _fits(datatype, op, (sendbuf, count), (recvbuf if comm.rank == root else None, count))
    if blocking:
        return lib().MPIX_Reduce(_addr(sendbuf), _addr(recvbuf), count, H.as_c_int(datatype),
                                 H.as_c_int(op), root, comm.h, a, ws, wsb)
    return lib().MPIX_Reduce_async(_addr(sendbuf), _addr(recvbuf), count, H.as_c_int(datatype),
                                   H.as_c_int(op), root, comm.h, a, ws, wsb,
                                   redop._stream_ptr(stream))


def scan(sendbuf, recvbuf, count, datatype, op, comm, exclusive=False, workspace=None,
         stream=None, blocking=True):
    """MPI_Scan, or MPI_Exscan with exclusive=True (sendbuf None =
    MPI_IN_PLACE); returns the MPI error class."""
    ws, wsb = _ws(workspace)
    name = 'MPIX_Exscan' if exclusive else 'MPIX_Scan'
    _fits(datatype, op, (sendbuf, count), (recvbuf, count))
    if blocking:
        return getattr(lib(), name)(_addr(sendbuf), _addr(recvbuf), count, H.as_c_int(datatype),
                                    H.as_c_int(op), comm.h, ws, wsb)
    return getattr(lib(), name + '_async')(_addr(sendbuf), _addr(recvbuf), count,
                                           H.as_c_int(datatype), H.as_c_int(op), comm.h, ws, wsb,
                                           redop._stream_ptr(stream))


def rs_workspace_bytes(recvcounts, datatype, comm, algorithm='auto'):
    a = RSB_ALGORITHMS[algorithm] if isinstance(algorithm, str) else algorithm
    cnts = (ctypes.c_ssize_t * len(recvcounts))(*recvcounts)
    return lib().MPIX_Reduce_scatter_workspace(cnts, H.as_c_int(datatype), comm.h, a)


def allreduce(sendbuf, recvbuf, count, datatype, op, comm, algorithm='auto', workspace=None,
              stream=None, blocking=True):
    """MPI_Allreduce (sendbuf None = MPI_IN_PLACE); returns the MPI error class."""
    a = AR_ALGORITHMS[algorithm] if isinstance(algorithm, str) else algorithm
    ws, wsb = _ws(workspace)
    _fits(datatype, op, (sendbuf, count), (recvbuf, count))
    if blocking:
        return lib().MPIX_Allreduce(_addr(sendbuf), _addr(recvbuf), count, H.as_c_int(datatype),
                                    H.as_c_int(op), comm.h, a, ws, wsb)
    return lib().MPIX_Allreduce_async(_addr(sendbuf), _addr(recvbuf), count, H.as_c_int(datatype),
                                      H.as_c_int(op), comm.h, a, ws, wsb,
                                      redop._stream_ptr(stream))


def rsb_workspace_bytes(recvcount, datatype, comm, algorithm='auto'):
    a = RSB_ALGORITHMS[algorithm] if isinstance(algorithm, str) else algorithm
    return lib().MPIX_Reduce_scatter_block_workspace(recvcount, H.as_c_int(datatype), comm.h, a)


def allreduce_workspace_bytes(count, datatype, comm):
    return lib().MPIX_Allreduce_workspace(count, H.as_c_int(datatype), comm.h)
