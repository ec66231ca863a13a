"""Host-side binding of libmpix_redop.so -- the MI355X local reduction.

Mirrors the reference interface for this path: MPI_Reduce_local /
MPIR_Reduce_local (src/mpi/coll/reduce_local/reduce_local.c:53-96) with the
same argument meaning (inbuf, inoutbuf, count, datatype, op) and MPI error
classes as return values, plus the stream-ordered and vector-target forms of
include/mpix_redop.h.  Buffers may be torch tensors, numpy arrays or raw
integer addresses.

This module never computes anything itself: every call goes to the HIP
library, and importing it fails loudly if the library was not built.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first: one runtime per process)

from . import handles as H

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libmpix_redop.so')

_lib = None


class RedopError(RuntimeError):
    def __init__(self, code, what=''):
        self.code = code
        super().__init__('%s: MPI error class %d (%s)' % (what or 'mpix_redop', code,
                                                         error_string(code) if _lib else '?'))


def lib():
    """The loaded C-ABI library (raises if the HIP build is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError('libmpix_redop.so is not built (%s); run '
                              '`python -c "import __graft_entry__ as g; g.build()"` '
                              'or `make -C mpich_amd/csrc`' % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        vp, i32, aint = ctypes.c_void_p, ctypes.c_int, ctypes.c_ssize_t
        sig = {
            'MPIX_Redop_init': ([], i32),
            'MPIX_Redop_finalize': ([], i32),
            'MPIX_Reduce_local': ([vp, vp, aint, i32, i32], i32),
            'MPIX_Reduce_local_async': ([vp, vp, aint, i32, i32, vp], i32),
            'MPIX_Reduce_local_vector': ([vp, vp, aint, aint, aint, i32, i32], i32),
            'MPIX_Reduce_local_vector_async': ([vp, vp, aint, aint, aint, i32, i32, vp], i32),
            'MPIX_Reduce_local_multi_async': ([ctypes.POINTER(vp), i32, vp, aint, i32, i32, vp],
                                              i32),
            'MPIX_Reduce_local_tree_async': ([ctypes.POINTER(vp), i32, vp, aint, i32, i32, vp],
                                             i32),
            'MPIX_Reduce_local_batch_async': ([ctypes.POINTER(vp), ctypes.POINTER(vp),
                                               ctypes.POINTER(aint), i32, i32, i32, vp], i32),
            'MPIX_Reduce_local_iov_async': ([vp, vp, aint, ctypes.POINTER(aint),
                                             ctypes.POINTER(aint), i32, i32, vp], i32),
            'MPIX_Reduce_local_iovec_async': ([vp, vp, aint, ctypes.POINTER(aint),
                                               ctypes.POINTER(aint), i32, i32, vp], i32),
            'MPIX_Redop_is_supported': ([i32, aint, i32], i32),
            'MPIX_Redop_is_supported_buffers': ([i32, aint, i32, vp, vp], i32),
            'MPIX_Redop_set_support': ([i32, aint, aint, aint], i32),
            'MPIX_Redop_get_support': ([ctypes.POINTER(i32)] + [ctypes.POINTER(aint)] * 3, i32),
            'MPIX_Ipc_export': ([vp, vp, ctypes.POINTER(aint)], i32),
            'MPIX_Ipc_open': ([vp, ctypes.POINTER(vp)], i32),
            'MPIX_Ipc_close': ([vp], i32),
            'MPIX_Redop_peer_access': ([i32, i32], i32),
            'MPIX_Redop_has_gpu_path': ([i32, i32], i32),
            'MPIX_Redop_op_dt_check': ([i32, i32], i32),
            'MPIX_Redop_internal_op_dt_check': ([i32, i32], i32),
            'MPIX_Datatype_internal': ([i32], i32),
            'MPIX_Datatype_extent': ([i32], aint),
            'MPIX_Datatype_size': ([i32], aint),
            'MPIX_Redop_set_fortran_booleans': ([i32, i32], i32),
            'MPIX_Redop_set_launch': ([i32, i32], i32),
            'MPIX_Redop_get_launch': ([ctypes.POINTER(i32)] * 3, i32),
            'MPIX_Redop_set_store_policy': ([i32, i32, i32, i32], i32),
            'MPIX_Redop_get_store_policy': ([ctypes.POINTER(i32)] * 4, i32),
            'MPIX_Redop_set_sync_store_policy': ([i32], i32),
            'MPIX_Redop_get_sync_store_policy': ([ctypes.POINTER(i32)], i32),
            'MPIX_Redop_sync_timing': ([i32, i32], i32),
            'MPIX_Redop_sync_timing_read': ([i32, ctypes.POINTER(ctypes.c_float), i32,
                                             ctypes.POINTER(i32)], i32),
            'MPIX_Redop_set_pageable': ([i32, aint], i32),
            'MPIX_Redop_get_pageable': ([ctypes.POINTER(i32), ctypes.POINTER(aint)], i32),
            'MPIX_Redop_last_error': ([], i32),
            'MPIX_Redop_error_string': ([i32], ctypes.c_char_p),
            'MPIX_Redop_build_info': ([], ctypes.c_char_p),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def _addr(buf):
    """base address of a buffer: a raw int pointer is passed through; a
    tensor or array must be contiguous (an MPI buffer is one span)"""
    if buf is None:
        return None
    if isinstance(buf, int):
        return buf
    if isinstance(buf, torch.Tensor):
        if not buf.is_contiguous():
            raise ValueError('non-contiguous tensor: an MPI buffer is one contiguous span')
        return buf.data_ptr()
    if hasattr(buf, 'ctypes'):          # numpy
        if not buf.flags['C_CONTIGUOUS']:
            raise ValueError('non-contiguous array: an MPI buffer is one contiguous span')
        return buf.ctypes.data
    raise TypeError('unsupported buffer type %r' % type(buf))


def _nbytes(buf):
    if isinstance(buf, torch.Tensor):
        return buf.numel() * buf.element_size()
    if hasattr(buf, 'nbytes'):
        return buf.nbytes
    return None                         # raw pointer: the caller vouches for the span


_extent_cache = {}


def _checked_extent(op, datatype):
    """extent of `datatype` when (op, datatype) is a supported pair, else 0.
    Both answers are fixed by the compiled op table (MPIX_Redop_is_supported
    ignores count), so they are looked up once per pair: the Python mirror's
    per-call cost is part of every synchronous call it times."""
    key = (op, datatype)
    ext = _extent_cache.get(key)
    if ext is None:
        cop, cdt = H.as_c_int(op), H.as_c_int(datatype)
        ext = 0
        # the pair itself, whatever the enable / threshold knobs say: the
        # span check guards every call the kernels would run
        legal = lib().MPIX_Redop_op_dt_check(cop, cdt) or \
            lib().MPIX_Redop_internal_op_dt_check(cop, cdt)
        if (op & 0xff) == 0x0f and (datatype_internal(datatype) & 0xffffff00) != 0x4c820100:
            legal = False                   # MPIX_EQUAL: MPI_BYTE only (opequal.c:22-23)
        if legal:
            ext = max(0, lib().MPIX_Datatype_extent(cdt))
        _extent_cache[key] = ext
    return ext


def _span_check(count, datatype, op, *bufs):
    """count elements of `datatype` must fit every tensor / array operand: a
    short buffer would be an out-of-bounds access on the device, not an MPI
    error the C call could report.  Calls the C side rejects anyway (bad
    count, type or op) go through, so they return their MPI error class."""
    if not isinstance(count, int) or count <= 0:
        return
    ext = _checked_extent(op, datatype)
    if ext <= 0:
        return                          # the C call reports MPI_ERR_OP / MPI_ERR_TYPE
    for b in bufs:
        nb = _nbytes(b)
        if nb is not None and nb < count * ext:
            raise ValueError('buffer of %d bytes is too small for %d elements of extent %d'
                             % (nb, count, ext))


def _bounds(buf):
    """[lo, hi) addresses a tensor / array may touch: its whole storage (a
    derived target may reach before the view's start, lb < 0); None for a
    raw pointer (the caller vouches for the span)"""
    if isinstance(buf, torch.Tensor):
        st = buf.untyped_storage()
        return st.data_ptr(), st.data_ptr() + st.nbytes()
    if hasattr(buf, 'ctypes'):
        root = buf
        while getattr(root, 'base', None) is not None and hasattr(root.base, 'ctypes'):
            root = root.base
        import numpy as np
        return np.byte_bounds(root)
    return None


def _range_check(buf, lo_off, hi_off, what):
    """bytes [addr+lo_off, addr+hi_off) of `buf` must lie inside its storage"""
    b = _bounds(buf)
    if b is None or hi_off <= lo_off:
        return
    a = _addr(buf)
    if a + lo_off < b[0] or a + hi_off > b[1]:
        raise ValueError('%s: bytes [%d, %d) of the buffer fall outside its storage (%d bytes)'
                         % (what, lo_off, hi_off, b[1] - b[0]))


def _stream_ptr(stream):
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def MPI_Reduce_local(inbuf, inoutbuf, count, datatype, op):
    """inoutbuf = inoutbuf OP inbuf, synchronous; returns an MPI error class.

    Device buffers must be ready (the caller orders its own streams, as an
    MPI caller does); host buffers are staged through the device."""
    _span_check(count, datatype, op, inbuf, inoutbuf)
    return lib().MPIX_Reduce_local(_addr(inbuf), _addr(inoutbuf), count, H.as_c_int(datatype),
                                   H.as_c_int(op))


def reduce_local_async(inbuf, inoutbuf, count, datatype, op, stream=None):
    """Enqueue the combine on `stream` (default: torch's current stream)."""
    _span_check(count, datatype, op, inbuf, inoutbuf)
    return lib().MPIX_Reduce_local_async(_addr(inbuf), _addr(inoutbuf), count,
                                         H.as_c_int(datatype), H.as_c_int(op),
                                         _stream_ptr(stream))


def reduce_local_vector(inbuf, inoutbuf, count, blocklen, stride, basic_type, op, stream=None,
                        sync=False):
    """Vector target / packed source (typerep_op.c:115-150)."""
    ext = _checked_extent(op, basic_type)
    if ext > 0 and isinstance(count, int) and isinstance(blocklen, int) and count > 0 \
            and blocklen > 0 and isinstance(stride, int) and stride >= blocklen:
        _range_check(inoutbuf, 0, ((count - 1) * stride + blocklen) * ext, 'vector target')
        _range_check(inbuf, 0, count * blocklen * ext, 'packed source')
    if sync:
        return lib().MPIX_Reduce_local_vector(_addr(inbuf), _addr(inoutbuf), count, blocklen,
                                              stride, H.as_c_int(basic_type), H.as_c_int(op))
    return lib().MPIX_Reduce_local_vector_async(_addr(inbuf), _addr(inoutbuf), count, blocklen,
                                                stride, H.as_c_int(basic_type), H.as_c_int(op),
                                                _stream_ptr(stream))


def reduce_local_iov_async(inbuf, inoutbuf, seg_offsets, seg_counts, basic_type, op,
                           stream=None):
    """derived target given as its flattened iov (byte offsets, element counts)"""
    n = len(seg_offsets)
    ext = _checked_extent(op, basic_type)
    if ext > 0 and n and all(c >= 0 for c in seg_counts):
        live = [(o, c) for o, c in zip(seg_offsets, seg_counts) if c > 0]
        if live:
            _range_check(inoutbuf, min(o for o, _ in live), max(o + c * ext for o, c in live),
                         'iov target')
            _range_check(inbuf, 0, sum(c for _, c in live) * ext, 'packed source')
    offs = (ctypes.c_ssize_t * n)(*seg_offsets)
    cnts = (ctypes.c_ssize_t * n)(*seg_counts)
    return lib().MPIX_Reduce_local_iov_async(_addr(inbuf), _addr(inoutbuf), n, offs, cnts,
                                             H.as_c_int(basic_type), H.as_c_int(op),
                                             _stream_ptr(stream))


def reduce_local_iovec_async(inbuf, inoutbuf, iov_offsets, iov_lens, basic_type, op,
                             stream=None):
    """derived target given as its raw iov (byte offsets, byte lengths):
    typerep_op_fallback incl. the pairtype gather (typerep_op.c:100-150)"""
    n = len(iov_offsets)
    ext = _checked_extent(op, basic_type)
    size = datatype_size(basic_type) if ext > 0 else 0
    if ext > 0 and size > 0 and n and all(x >= 0 for x in iov_lens):
        live = [(o, ln) for o, ln in zip(iov_offsets, iov_lens) if ln > 0]
        if live:
            _range_check(inoutbuf, min(o for o, _ in live), max(o + ln for o, ln in live),
                         'iov target')
            _range_check(inbuf, 0, (sum(ln for _, ln in live) // size) * ext, 'packed source')
    offs = (ctypes.c_ssize_t * n)(*iov_offsets)
    lens = (ctypes.c_ssize_t * n)(*iov_lens)
    return lib().MPIX_Reduce_local_iovec_async(_addr(inbuf), _addr(inoutbuf), n, offs, lens,
                                               H.as_c_int(basic_type), H.as_c_int(op),
                                               _stream_ptr(stream))


def reduce_local_multi_async(inbufs, inoutbuf, count, datatype, op, stream=None):
    """inoutbuf = (...((inoutbuf OP in[0]) OP in[1])...) OP in[k-1], one pass."""
    _span_check(count, datatype, op, inoutbuf, *inbufs)
    arr = (ctypes.c_void_p * len(inbufs))(*[_addr(b) for b in inbufs])
    return lib().MPIX_Reduce_local_multi_async(arr, len(inbufs), _addr(inoutbuf), count,
                                               H.as_c_int(datatype), H.as_c_int(op),
                                               _stream_ptr(stream))


def reduce_local_tree_async(inbufs, outbuf, count, datatype, op, stream=None):
    """outbuf = pairwise tree fold of the 2^L inbufs, levels m = 1, 2, 4, ...
    (slot s = slot s OP slot s+m); outbuf may be one of the inbufs exactly; a
    None slot (not slot 0) is absent: its partner passes through."""
    _span_check(count, datatype, op, outbuf, *[b for b in inbufs if b is not None])
    arr = (ctypes.c_void_p * len(inbufs))(*[None if b is None else _addr(b) for b in inbufs])
    return lib().MPIX_Reduce_local_tree_async(arr, len(inbufs), _addr(outbuf), count,
                                              H.as_c_int(datatype), H.as_c_int(op),
                                              _stream_ptr(stream))


BATCH_MAX = 64


def reduce_local_batch_async(inbufs, inoutbufs, counts, datatype, op, stream=None):
    """k independent combines inoutbufs[i] OP= inbufs[i] (counts[i] elements
    each) in one launch on `stream` -- the same bits as k reduce_local_async
    calls; no target may overlap another triple's source or target."""
    k = len(counts)
    if len(inbufs) != k or len(inoutbufs) != k:
        raise ValueError('inbufs, inoutbufs and counts must have one entry per triple')
    for b, o, c in zip(inbufs, inoutbufs, counts):
        _span_check(c, datatype, op, b, o)
    ins = (ctypes.c_void_p * max(k, 1))(*[_addr(b) for b in inbufs])
    ios = (ctypes.c_void_p * max(k, 1))(*[_addr(b) for b in inoutbufs])
    cnt = (ctypes.c_ssize_t * max(k, 1))(*counts)
    return lib().MPIX_Reduce_local_batch_async(ins, ios, cnt, k, H.as_c_int(datatype),
                                               H.as_c_int(op), _stream_ptr(stream))


IPC_HANDLE_BYTES = 64


def ipc_export(buf):
    """(handle bytes, byte offset of buf inside its allocation)"""
    h = ctypes.create_string_buffer(IPC_HANDLE_BYTES)
    off = ctypes.c_ssize_t()
    check(lib().MPIX_Ipc_export(_addr(buf), h, ctypes.byref(off)), 'MPIX_Ipc_export')
    return h.raw, off.value


def ipc_open(handle):
    """map a peer allocation; returns its base address in this process"""
    p = ctypes.c_void_p()
    check(lib().MPIX_Ipc_open(handle, ctypes.byref(p)), 'MPIX_Ipc_open')
    return p.value


def ipc_close(base):
    return lib().MPIX_Ipc_close(base)


def peer_access(device, peer_device):
    """True if kernels on `device` can read `peer_device`'s memory (peer access
    enabled at the pair's first use, yaksuri_hip_init_hooks.c:164-181)"""
    return bool(lib().MPIX_Redop_peer_access(device, peer_device))


def has_gpu_path(op, datatype):
    """a kernel covers (op, datatype), whatever the support knobs say"""
    return bool(lib().MPIX_Redop_has_gpu_path(H.as_c_int(op), H.as_c_int(datatype)))


def check(rc, what='MPI_Reduce_local'):
    if rc != H.MPI_SUCCESS:
        raise RedopError(rc, what)
    return rc


def is_supported(op, datatype, count=0):
    return bool(lib().MPIX_Redop_is_supported(H.as_c_int(op), count, H.as_c_int(datatype)))


def is_supported_buffers(op, datatype, count, inbuf, inoutbuf):
    """the pointer-aware predicate (host-resident operands below the floor of
    their memory kind stay with the caller's CPU loop)"""
    return bool(lib().MPIX_Redop_is_supported_buffers(H.as_c_int(op), count, H.as_c_int(datatype),
                                                      _addr(inbuf), _addr(inoutbuf)))


def set_support(enable=True, threshold_bytes=-1, host_floor_bytes=None, pinned_floor_bytes=None):
    """the predicate's knobs (None keeps the current floor); returns an MPI error class"""
    cur = get_support()
    return lib().MPIX_Redop_set_support(
        1 if enable else 0, threshold_bytes,
        cur['host_floor_bytes'] if host_floor_bytes is None else host_floor_bytes,
        cur['pinned_floor_bytes'] if pinned_floor_bytes is None else pinned_floor_bytes)


def get_support():
    e = ctypes.c_int()
    t, h, p = ctypes.c_ssize_t(), ctypes.c_ssize_t(), ctypes.c_ssize_t()
    check(lib().MPIX_Redop_get_support(ctypes.byref(e), ctypes.byref(t), ctypes.byref(h),
                                       ctypes.byref(p)))
    return dict(enable=bool(e.value), threshold_bytes=t.value, host_floor_bytes=h.value,
                pinned_floor_bytes=p.value)


def op_dt_check(op, datatype):
    return bool(lib().MPIX_Redop_op_dt_check(H.as_c_int(op), H.as_c_int(datatype)))


def internal_op_dt_check(op, datatype):
    return bool(lib().MPIX_Redop_internal_op_dt_check(H.as_c_int(op), H.as_c_int(datatype)))


def datatype_internal(datatype):
    return lib().MPIX_Datatype_internal(H.as_c_int(datatype)) & 0xffffffff


def datatype_extent(datatype):
    return lib().MPIX_Datatype_extent(H.as_c_int(datatype))


def datatype_size(datatype):
    return lib().MPIX_Datatype_size(H.as_c_int(datatype))


def set_fortran_booleans(true_value, false_value):
    return lib().MPIX_Redop_set_fortran_booleans(true_value, false_value)


def set_pageable(threads, chunk_bytes=16 << 20):
    """host workers (0 = hipMemcpyAsync staging) and chunk size for large
    pageable operands of the synchronous call; returns an MPI error class"""
    return lib().MPIX_Redop_set_pageable(threads, chunk_bytes)


def get_pageable():
    t, c = ctypes.c_int(), ctypes.c_ssize_t()
    check(lib().MPIX_Redop_get_pageable(ctypes.byref(t), ctypes.byref(c)))
    return dict(threads=t.value, chunk_bytes=c.value)


def set_launch(block_threads=256, max_grid=0):
    return lib().MPIX_Redop_set_launch(block_threads, max_grid)


def get_launch():
    b, u, g = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib().MPIX_Redop_get_launch(ctypes.byref(b), ctypes.byref(u), ctypes.byref(g))
    return dict(block=b.value, unroll=u.value, max_grid=g.value)


def set_store_policy(xcd_mask=0, every=0, phase=0, tail_blocks=0):
    """contiguous kernel: blocks on the XCDs of xcd_mask, blocks b with
    b % every == phase, and the last tail_blocks blocks store write-through
    (performance knob, same bits)"""
    return lib().MPIX_Redop_set_store_policy(xcd_mask, every, phase, tail_blocks)


def get_store_policy():
    x, e, p, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib().MPIX_Redop_get_store_policy(ctypes.byref(x), ctypes.byref(e), ctypes.byref(p),
                                            ctypes.byref(t)))
    return dict(xcd_mask=x.value, every=e.value, phase=p.value, tail_blocks=t.value)


def set_sync_store_policy(xcd_mask=-1):
    """the synchronous entry's own XCD mask (-1: the default)"""
    return lib().MPIX_Redop_set_sync_store_policy(xcd_mask)


def get_sync_store_policy():
    x = ctypes.c_int()
    check(lib().MPIX_Redop_get_sync_store_policy(ctypes.byref(x)))
    return x.value


def sync_timing(device, ncalls):
    """Record a HIP event pair around the launch of the calling thread's next
    `ncalls` synchronous calls on `device` (MPIX_Redop_sync_timing)."""
    check(lib().MPIX_Redop_sync_timing(int(device), int(ncalls)))


def sync_timing_read(device, cap=1 << 16):
    """The recorded kernel durations in ms, call order; stops the recording."""
    buf = (ctypes.c_float * cap)()
    got = ctypes.c_int()
    check(lib().MPIX_Redop_sync_timing_read(int(device), buf, cap, ctypes.byref(got)))
    return list(buf[:got.value])


def error_string(code):
    return lib().MPIX_Redop_error_string(code).decode()


def build_info():
    return lib().MPIX_Redop_build_info().decode()


def finalize():
    return lib().MPIX_Redop_finalize()
