"""ORACLE loader -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/liboracle_redop.so (the clean-room CPU
restatement in redop_oracle.c).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product package
mpich_amd/ never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'build', 'liboracle_redop.so')

_lib = None


def build(force=False):
    """Compile the oracle with gcc (oracle/Makefile)."""
    srcs = [os.path.join(HERE, f) for f in ('redop_oracle.c', 'host_bench.c')]
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(['make', '-s', '-C', HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, il = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
        L.oracle_reduce_local.argtypes = [vp, vp, il, i32, i32]
        L.oracle_reduce_local_mt.argtypes = [vp, vp, il, i32, i32, i32]
        L.oracle_reduce_local_vector.argtypes = [vp, vp, il, il, il, i32, i32]
        L.oracle_reduce_local_iov.argtypes = [vp, vp, il, ctypes.POINTER(il), ctypes.POINTER(il),
                                              i32, i32]
        L.oracle_reduce_local_iovec.argtypes = L.oracle_reduce_local_iov.argtypes
        L.oracle_size.argtypes = [i32]
        L.oracle_size.restype = il
        L.oracle_internal.argtypes = [i32]
        L.oracle_extent.argtypes = [i32]
        L.oracle_extent.restype = il
        L.oracle_op_dt_check.argtypes = [i32, i32]
        L.oracle_internal_op_dt_check.argtypes = [i32, i32]
        L.oracle_set_fortran_booleans.argtypes = [i32, i32]
        L.oracle_set_fortran_booleans.restype = None
        L.oracle_rsb_recursive_halving.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), il,
                                                   i32, i32, i32]
        L.oracle_rsb_pairwise.argtypes = L.oracle_rsb_recursive_halving.argtypes
        L.oracle_rs_recursive_halving.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                  ctypes.POINTER(il), i32, i32, i32]
        L.oracle_rs_pairwise.argtypes = L.oracle_rs_recursive_halving.argtypes
        L.oracle_reduce_binomial.argtypes = [ctypes.POINTER(vp), vp, il, i32, i32, i32, i32]
        L.oracle_reduce_rsg.argtypes = L.oracle_reduce_binomial.argtypes
        L.oracle_allreduce_rabenseifner.argtypes = L.oracle_rsb_recursive_halving.argtypes
        L.oracle_allreduce_recursive_doubling.argtypes = L.oracle_rsb_recursive_halving.argtypes
        L.oracle_allreduce_ring.argtypes = L.oracle_rsb_recursive_halving.argtypes
        L.oracle_scan.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), il, i32, i32, i32, i32]
        L.oracle_wtime.restype = ctypes.c_double
        dp, ip = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)
        L.oracle_bench_reduce.argtypes = [il, i32, i32, i32, ip, ctypes.c_double, dp, dp, ip, dp]
        L.oracle_bench_triad.argtypes = [il, i32, ip, ctypes.c_double, dp, dp, ip, dp]
        _lib = L
    return _lib


def _i32(h):
    """MPI handles above 0x7fffffff (pair types 0x8c......) as C int."""
    return ctypes.c_int(h - (1 << 32) if h >= (1 << 31) else h).value


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def reduce_local(inbuf, inoutbuf, count, datatype, op, nthreads=1):
    """inoutbuf = inoutbuf OP inbuf on numpy buffers; returns the MPI error class."""
    if nthreads > 1:
        return lib().oracle_reduce_local_mt(_ptr(inbuf), _ptr(inoutbuf), count, _i32(datatype),
                                            _i32(op), nthreads)
    return lib().oracle_reduce_local(_ptr(inbuf), _ptr(inoutbuf), count, _i32(datatype), _i32(op))


def reduce_local_vector(inbuf, inoutbuf, count, blocklen, stride, datatype, op):
    return lib().oracle_reduce_local_vector(_ptr(inbuf), _ptr(inoutbuf), count, blocklen, stride,
                                            _i32(datatype), _i32(op))


def reduce_local_iov(inbuf, inoutbuf, seg_offsets, seg_counts, datatype, op):
    n = len(seg_offsets)
    return lib().oracle_reduce_local_iov(_ptr(inbuf), _ptr(inoutbuf), n,
                                         (ctypes.c_long * n)(*seg_offsets),
                                         (ctypes.c_long * n)(*seg_counts), _i32(datatype),
                                         _i32(op))


def reduce_local_iovec(inbuf, inoutbuf, iov_offsets, iov_lens, datatype, op):
    """typerep_op_fallback over a raw iov (byte offsets, byte lengths)"""
    n = len(iov_offsets)
    return lib().oracle_reduce_local_iovec(_ptr(inbuf), _ptr(inoutbuf), n,
                                           (ctypes.c_long * n)(*iov_offsets),
                                           (ctypes.c_long * n)(*iov_lens), _i32(datatype),
                                           _i32(op))


def size(datatype):
    return lib().oracle_size(_i32(datatype))


def internal(datatype):
    return lib().oracle_internal(_i32(datatype)) & 0xffffffff


def extent(datatype):
    return lib().oracle_extent(_i32(datatype))


def op_dt_check(op, datatype):
    return bool(lib().oracle_op_dt_check(_i32(op), _i32(datatype)))


def internal_op_dt_check(op, datatype):
    return bool(lib().oracle_internal_op_dt_check(_i32(op), _i32(datatype)))


def set_fortran_booleans(t, f):
    lib().oracle_set_fortran_booleans(t, f)


def rsb_recursive_halving(sendbufs, recvcount, datatype, op, algorithm='recursive_halving'):
    """Simulate MPI_Reduce_scatter_block (recursive halving or pairwise) over
    P ranks in one process; returns the list of per-rank result arrays."""
    P = len(sendbufs)
    ext = extent(datatype)
    recvs = [np.zeros(recvcount * ext, np.uint8) for _ in range(P)]
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in sendbufs])
    rp = (ctypes.c_void_p * P)(*[r.ctypes.data for r in recvs])
    fn = lib().oracle_rsb_pairwise if algorithm == 'pairwise' else \
        lib().oracle_rsb_recursive_halving
    rc = fn(sp, rp, recvcount, _i32(datatype), _i32(op), P)
    if rc:
        raise RuntimeError('oracle rsb failed: %d' % rc)
    return recvs


def rs_schedule(sendbufs, recvcounts, datatype, op, algorithm='recursive_halving'):
    """Simulate MPI_Reduce_scatter (per-rank recvcounts) over P ranks in one
    process with the reference's recursive halving or pairwise schedule."""
    P = len(sendbufs)
    ext = extent(datatype)
    recvs = [np.zeros(max(1, c) * ext, np.uint8)[:c * ext] for c in recvcounts]
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in sendbufs])
    rp = (ctypes.c_void_p * P)(*[r.ctypes.data for r in recvs])
    cn = (ctypes.c_long * P)(*recvcounts)
    fn = lib().oracle_rs_pairwise if algorithm == 'pairwise' else \
        lib().oracle_rs_recursive_halving
    rc = fn(sp, rp, cn, _i32(datatype), _i32(op), P)
    if rc:
        raise RuntimeError('oracle reduce_scatter failed: %d' % rc)
    return recvs


def reduce_schedule(sendbufs, count, datatype, op, root, algorithm='binomial'):
    """Simulate MPI_Reduce to `root` over P ranks with the reference's
    binomial or reduce_scatter_gather schedule; returns the root's vector."""
    P = len(sendbufs)
    out = np.zeros(max(1, count * extent(datatype)), np.uint8)
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in sendbufs])
    fn = lib().oracle_reduce_rsg if algorithm == 'reduce_scatter_gather' else \
        lib().oracle_reduce_binomial
    rc = fn(sp, out.ctypes.data, count, _i32(datatype), _i32(op), root, P)
    if rc:
        raise RuntimeError('oracle reduce failed: %d' % rc)
    return out[:count * extent(datatype)]


def scan_schedule(sendbufs, recvbufs, count, datatype, op, exclusive=False):
    """Simulate MPI_Scan / MPI_Exscan (recursive doubling) over P ranks;
    recvbufs (uint8 arrays) are updated in place."""
    P = len(sendbufs)
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in sendbufs])
    rp = (ctypes.c_void_p * P)(*[r.ctypes.data for r in recvbufs])
    rc = lib().oracle_scan(sp, rp, count, _i32(datatype), _i32(op), P, int(exclusive))
    if rc:
        raise RuntimeError('oracle scan failed: %d' % rc)
    return recvbufs


def rsb_pairwise(sendbufs, recvcount, datatype, op):
    return rsb_recursive_halving(sendbufs, recvcount, datatype, op, algorithm='pairwise')


def allreduce_rabenseifner(sendbufs, count, datatype, op, algorithm='reduce_scatter_allgather'):
    """Simulate MPIR_Allreduce_intra_reduce_scatter_allgather (or, with
    algorithm='recursive_doubling', MPIR_Allreduce_intra_recursive_doubling)
    over P ranks."""
    P = len(sendbufs)
    ext = extent(datatype)
    recvs = [np.zeros(count * ext, np.uint8) for _ in range(P)]
    sp = (ctypes.c_void_p * P)(*[s.ctypes.data for s in sendbufs])
    rp = (ctypes.c_void_p * P)(*[r.ctypes.data for r in recvs])
    fn = {'recursive_doubling': lib().oracle_allreduce_recursive_doubling,
          'ring': lib().oracle_allreduce_ring}.get(algorithm, lib().oracle_allreduce_rabenseifner)
    rc = fn(sp, rp, count, _i32(datatype), _i32(op), P)
    if rc:
        raise RuntimeError('oracle allreduce failed: %d' % rc)
    return recvs


def wtime():
    return lib().oracle_wtime()


def combine_fn_address():
    """address of oracle_combine (MPIX_Combine_fn signature), for installing
    the oracle as the combine of a host-memory libmpix_coll communicator"""
    return ctypes.cast(lib().oracle_combine, ctypes.c_void_p).value


def _bench(fn, *args):
    best, med, passes, span = ctypes.c_double(), ctypes.c_double(), ctypes.c_int(), \
        ctypes.c_double()
    rc = fn(*args, ctypes.byref(best), ctypes.byref(med), ctypes.byref(passes), ctypes.byref(span))
    if rc:
        raise RuntimeError('host bench failed (%d)' % rc)
    return best.value, med.value, passes.value, span.value


def bench_reduce(count, datatype, op, cpus, seconds):
    """MPI_Reduce_local(datatype, op) on `count` elements split over one
    pinned thread per entry of `cpus` (each first-touches its own slice);
    (best, median) seconds per pass, the number of passes and the wall span
    of all passes (passes / span = sustained rate)"""
    arr = (ctypes.c_int * len(cpus))(*cpus)
    return _bench(lib().oracle_bench_reduce, count, _i32(datatype), _i32(op), len(cpus), arr,
                  float(seconds))


def bench_pair(count, datatype, op, cpus, seconds):
    """MPI_Reduce_local(datatype, op) and the host triad in the same passes
    (host_bench.c oracle_bench_pair): (reduce best, reduce median, passes,
    span, triad best, triad median, median per-pass reduce / triad time)"""
    L = lib()
    arr = (ctypes.c_int * len(cpus))(*cpus)
    best, med, passes, span = ctypes.c_double(), ctypes.c_double(), ctypes.c_int(), \
        ctypes.c_double()
    pair = (ctypes.c_double * 3)()
    rc = L.oracle_bench_pair(ctypes.c_long(count), _i32(datatype), _i32(op), len(cpus), arr,
                             ctypes.c_double(seconds), ctypes.byref(best), ctypes.byref(med),
                             ctypes.byref(passes), ctypes.byref(span), pair)
    if rc:
        raise RuntimeError('host bench failed (%d)' % rc)
    return best.value, med.value, passes.value, span.value, pair[0], pair[1], pair[2]


def bench_rsb_rank(recvcount, P, rank, cpu, reps, datatype, op):
    """one rank's host work in MPICH's recursive-halving reduce-scatter-block
    (copy in, the log2(P) combines, copy out) on one pinned core
    (host_bench.c oracle_bench_rsb_rank): dict of median seconds and the
    elements combined per call"""
    L = lib()
    out = (ctypes.c_double * 5)()
    rc = L.oracle_bench_rsb_rank(ctypes.c_long(recvcount), int(P), int(rank), int(cpu), int(reps),
                                 _i32(datatype), _i32(op), out)
    if rc:
        raise RuntimeError('host RSB bench failed (%d)' % rc)
    return dict(copy_in_s=out[0], combine_s=out[1], copy_out_s=out[2], total_s=out[3],
                combined_elements=int(out[4]))


def bench_triad(count, cpus, seconds):
    """host STREAM triad on `count` fp32 (12 bytes each) over pinned threads"""
    arr = (ctypes.c_int * len(cpus))(*cpus)
    return _bench(lib().oracle_bench_triad, count, len(cpus), arr, float(seconds))
