"""CPU-side checks of the C-ABI boundary (no GPU compute calls):
libmpix_redop.so loads, exports every function/object include/mpix_redop.h
declares, and its handle tables / legality matrix / support predicate agree
with the oracle's independent restatement of the reference's tables."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'mpix_redop.h')
COLL_HEADER = os.path.join(ROOT, 'include', 'mpix_coll.h')


def declared_symbols(header=HEADER):
    src = open(header).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    funcs = set(re.findall(r'\b(MPIX_\w+)\s*\(', src))
    funcs -= {m for m in funcs if re.search(r'#define\s+' + m + r'\b', src)}
    funcs -= set(re.findall(r'typedef\s+\w+\s+(MPIX_\w+)\s*\(', src))
    objs = set(re.findall(r'extern\s+MPIX_op_function\s*\*\s*const\s+(MPIX_\w+)', src))
    return funcs | objs


@pytest.fixture(scope='module')
def R():
    from mpich_amd import redop
    return redop


def test_library_exports_every_declared_symbol(R):
    L = R.lib()
    syms = declared_symbols()
    assert len(syms) >= 30
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing


def test_coll_library_exports_every_declared_symbol(R):
    """libmpix_coll.so (include/mpix_coll.h) loads without a GPU and exports
    every function it declares"""
    from mpich_amd import ccl
    L = ccl.lib()
    syms = declared_symbols(COLL_HEADER)
    assert len(syms) >= 15
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing


def test_op_table_layout(R):
    L = R.lib()
    tab = (ctypes.c_void_p * 16).in_dll(L, 'MPIX_Op_table')
    # oputil.c:10-27 order: NULL, MAX, MIN, SUM, PROD, LAND, BAND, LOR, BOR,
    # LXOR, BXOR, MINLOC, MAXLOC, REPLACE, NO_OP, EQUAL
    names = [None, 'MPIX_MAXF', 'MPIX_MINF', 'MPIX_SUM_fn', 'MPIX_PROD_fn', 'MPIX_LAND_fn',
             'MPIX_BAND_fn', 'MPIX_LOR_fn', 'MPIX_BOR_fn', 'MPIX_LXOR_fn', 'MPIX_BXOR_fn',
             'MPIX_MINLOC_fn', 'MPIX_MAXLOC_fn', 'MPIX_REPLACE_fn', 'MPIX_NO_OP_fn',
             'MPIX_EQUAL_fn']
    for i, n in enumerate(names):
        if n is None:
            assert not tab[i]
        else:
            assert tab[i] == ctypes.cast(getattr(L, n), ctypes.c_void_p).value


def all_handles():
    from mpich_amd import handles as H
    ext = [v for k, v in vars(H).items() if k.startswith(('MPI_', 'MPIX_')) and isinstance(v, int)
           and (v >> 24) in (0x4c, 0x8c)]
    internal = [v for k, v in vars(H).items() if k.startswith('MPIR_')]
    return sorted(set(ext + internal + [0x4c0000ff, 0x4c000012, 0x8c000007]))


def test_tables_agree_with_oracle(R, oracle):
    from mpich_amd import handles as H
    for dt in all_handles():
        assert R.datatype_internal(dt) == oracle.internal(dt), hex(dt)
        assert R.datatype_extent(dt) == oracle.extent(dt), hex(dt)
        for op in H.OPS.values():
            assert R.op_dt_check(op, dt) == oracle.op_dt_check(op, dt), (hex(op), hex(dt))
            it = R.datatype_internal(dt)
            assert R.internal_op_dt_check(op, it) == oracle.internal_op_dt_check(op, it), \
                (hex(op), hex(dt))


def test_support_predicate(R):
    """MPIR_Typerep_reduce_is_supported mirror: every legal pair except the
    bf16 ops the reference itself asserts on (MPIR_BFLOAT16 is in no type
    group but SUM's helper, op_fns.c:459-493).  Round 4 covers the x87 long
    double and __float128 families: compare-and-select in integer arithmetic,
    SUM / PROD in software extended / quad arithmetic (redop_soft.h)."""
    from mpich_amd import handles as H
    n_supported = 0
    for dt in all_handles():
        for name, op in H.OPS.items():
            legal = R.internal_op_dt_check(op, R.datatype_internal(dt))
            sup = R.is_supported(op, dt)
            if sup:
                n_supported += 1
                assert legal
            elif legal and op not in (H.MPI_REPLACE, H.MPI_NO_OP):
                raw = R.datatype_internal(dt) & 0xffffff00
                assert raw == H.MPIR_BFLOAT16 and op != H.MPI_SUM, (name, hex(dt))
    assert n_supported > 300
    assert R.is_supported(H.MPI_SUM, H.MPI_FLOAT)
    assert R.is_supported(H.MPI_MAXLOC, H.MPI_SHORT_INT)
    assert not R.is_supported(H.MPI_MAX, H.MPIX_BFLOAT16)
    assert not R.is_supported(H.MPI_BAND, H.MPI_FLOAT)
    for op in (H.MPI_MAX, H.MPI_MIN, H.MPI_SUM, H.MPI_PROD):
        assert R.is_supported(op, H.MPI_LONG_DOUBLE) and R.is_supported(op, H.MPI_REAL16)
    for t in (H.MPI_COMPLEX32, H.MPI_C_LONG_DOUBLE_COMPLEX, H.MPI_CXX_LONG_DOUBLE_COMPLEX):
        assert R.is_supported(H.MPI_SUM, t) and R.is_supported(H.MPI_PROD, t)
    for op in (H.MPI_MAXLOC, H.MPI_MINLOC):
        assert R.is_supported(op, H.MPI_LONG_DOUBLE_INT)
        assert R.is_supported(op, H.MPIR_2FLOAT128)


def test_errors_without_gpu(R):
    """argument errors are detected before any device work
    (binding_c.py:2774-2783 checks; count==0 is a no-op, reduce_local.c:59-60)."""
    from mpich_amd import handles as H
    assert R.MPI_Reduce_local(0, 0, 0, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_SUCCESS
    assert R.MPI_Reduce_local(4096, 8192, -1, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_ERR_COUNT
    assert R.MPI_Reduce_local(4096, 4096, 10, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(4096, 4100, 10, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(2 ** 64 - 1, 8192, 10, H.MPI_INT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(0, 8192, 10, H.MPI_INT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(4096, 1 << 20, 10, H.MPI_FLOAT, H.MPI_BAND) == H.MPI_ERR_OP
    assert R.MPI_Reduce_local(4096, 1 << 20, 10, H.MPI_INT, H.MPI_MAXLOC) == H.MPI_ERR_OP
    assert R.MPI_Reduce_local(4096, 1 << 20, 10, H.MPI_PACKED, H.MPI_SUM) == H.MPI_ERR_OP
    assert R.MPI_Reduce_local(4096, 1 << 20, 10, 0x4c0000ff, H.MPI_SUM) == H.MPI_ERR_TYPE
    assert R.MPI_Reduce_local(4096, 1 << 20, 10, H.MPI_INT, H.MPI_OP_NULL) == H.MPI_ERR_OP
    assert R.MPI_Reduce_local(4096, 1 << 20, 10, H.MPIX_BFLOAT16, H.MPI_MAX) == H.MPI_ERR_TYPE
    # count * extent that would wrap 64 bits (no buffer spans 2^56 bytes)
    assert R.MPI_Reduce_local(4096, 1 << 20, 1 << 62, H.MPI_INT, H.MPI_SUM) == H.MPI_ERR_COUNT


def test_tree_entry_argument_errors(R):
    """MPIX_Reduce_local_tree_async: 2..16 operands, a power of two; the output
    may be slot 0 itself but overlap nothing else; MPIX_EQUAL is refused;
    host (non device-accessible) buffers are MPI_ERR_BUFFER -- all before any
    device work"""
    import ctypes
    from mpich_amd import handles as H
    L = R.lib()

    def call(ptrs, out, count=16, dt=H.MPI_FLOAT, op=H.MPI_SUM):
        arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
        return L.MPIX_Reduce_local_tree_async(arr, len(ptrs), out, count, dt, op, None)
    base = 1 << 20
    ins = [base + i * 4096 for i in range(8)]
    for k in (1, 3, 6, 32):
        assert call(ins[:k] if k <= 8 else ins * 4, 1 << 24) == H.MPI_ERR_ARG, k
    assert call(ins[:4], ins[1] + 8) == H.MPI_ERR_BUFFER           # overlaps slot 1
    assert call(ins[:4], 1 << 24, count=-1) == H.MPI_ERR_COUNT
    assert call(ins[:4], 1 << 24, op=H.MPI_BAND) == H.MPI_ERR_OP
    assert call(ins[:4], 1 << 24, dt=H.MPI_BYTE, op=H.MPIX_EQUAL) == H.MPI_ERR_OP
    assert call(ins[:4], 1 << 24, count=0) == H.MPI_SUCCESS
    import numpy as np
    a = [np.zeros(16, np.float32) for _ in range(4)]
    assert call([x.ctypes.data for x in a], a[0].ctypes.data) == H.MPI_ERR_BUFFER   # host


def test_copy_multi_argument_errors(R):
    """MPIX_Copy_multi_async: at most 16 segments, byte counts >= 0, no
    overlapping pair, host memory refused -- all before any device work"""
    import ctypes
    import numpy as np
    from mpich_amd import handles as H
    L = R.lib()
    vp = ctypes.c_void_p
    L.MPIX_Copy_multi_async.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                        ctypes.POINTER(ctypes.c_ssize_t), ctypes.c_int, vp]

    def call(triples):
        n = len(triples)
        return L.MPIX_Copy_multi_async((vp * max(n, 1))(*[t[0] for t in triples]),
                                       (vp * max(n, 1))(*[t[1] for t in triples]),
                                       (ctypes.c_ssize_t * max(n, 1))(*[t[2] for t in triples]),
                                       n, None)
    assert call([(1 << 20, 1 << 21, 64)] * 17) == H.MPI_ERR_ARG
    assert call([(1 << 20, 1 << 21, -1)]) == H.MPI_ERR_COUNT
    assert call([(1 << 20, (1 << 20) + 8, 64)]) == H.MPI_ERR_BUFFER
    assert call([(1 << 20, 1 << 21, 0)]) == H.MPI_SUCCESS
    assert call([]) == H.MPI_SUCCESS
    a, b = np.zeros(16, np.uint8), np.zeros(16, np.uint8)
    assert call([(a.ctypes.data, b.ctypes.data, 16)]) == H.MPI_ERR_BUFFER


def test_errors_reduce_local_errors_test(R):
    """test/mpi/errors/coll/reduce_local.c:38-58: MPI_IN_PLACE as either
    buffer and inbuf == inoutbuf are MPI_ERR_BUFFER (checked before any
    device work, so host pointers suffice here)"""
    import numpy as np
    from mpich_amd import handles as H
    size = 4
    buf = np.arange(size, dtype=np.int32)
    recv = np.full(size, -1, np.int32)
    in_place = 2 ** 64 - 1      # MPI_IN_PLACE == (void *) -1 (mpi.h.in)
    assert R.MPI_Reduce_local(in_place, recv, size, H.MPI_INT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(buf, in_place, size, H.MPI_INT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(recv, recv, size, H.MPI_INT, H.MPI_SUM) == H.MPI_ERR_BUFFER


def test_launch_knobs(R):
    cfg = R.get_launch()
    assert cfg['block'] % 64 == 0 and cfg['unroll'] >= 1
    assert R.set_launch(100, 0) == 12
    assert R.set_launch(cfg['block'], cfg['max_grid']) == 0
    assert 'gfx950' in R.build_info()


def test_python_mirror_rejects_bad_spans():
    """the Python mirror checks what the raw C-ABI cannot: a tensor / array
    operand must be one contiguous span holding count elements (a short or
    strided buffer would be an out-of-bounds device access, not an MPI error)"""
    import numpy as np
    from mpich_amd import handles as H
    from mpich_amd import redop
    a = np.zeros(64, np.float32)
    with pytest.raises(ValueError, match='non-contiguous'):
        redop.MPI_Reduce_local(a[::2], a[:32].copy(), 32, H.MPI_FLOAT, H.MPI_SUM)
    with pytest.raises(ValueError, match='too small'):
        redop.MPI_Reduce_local(a, np.zeros(16, np.float32), 32, H.MPI_FLOAT, H.MPI_SUM)
    with pytest.raises(ValueError, match='too small'):      # pairs: extent, not value size
        redop.reduce_local_async(np.zeros(4, np.int32), np.zeros(4, np.int32), 3, H.MPI_2INT,
                                 H.MPI_MAXLOC, stream=0)
    with pytest.raises(ValueError, match='too small'):
        redop.reduce_local_multi_async([a, a[:8].copy()], a, 32, H.MPI_FLOAT, H.MPI_SUM, stream=0)


def test_python_collective_wrappers_reject_short_buffers(oracle):
    """mpich_amd.ccl checks tensor / array spans the same way before the C
    call: sendbuf P*recvcount, recvbuf recvcount (all of it for MPI_IN_PLACE)"""
    import numpy as np
    from mpich_amd import ccl
    from mpich_amd import handles as H
    comms = ccl.comm_create_local(2)
    try:
        for c in comms:
            c.set_combine(oracle.combine_fn_address())
        c0 = comms[0]
        with pytest.raises(ValueError, match='too small'):
            ccl.reduce_scatter_block(np.zeros(10, np.float32), np.zeros(8, np.float32), 8,
                                     H.MPI_FLOAT, H.MPI_SUM, c0)
        with pytest.raises(ValueError, match='too small'):
            ccl.reduce_scatter_block(None, np.zeros(8, np.float32), 8, H.MPI_FLOAT, H.MPI_SUM, c0)
        with pytest.raises(ValueError, match='too small'):
            ccl.allreduce(np.zeros(8, np.float32), np.zeros(4, np.float32), 8, H.MPI_FLOAT,
                          H.MPI_SUM, c0)
        with pytest.raises(ValueError, match='non-contiguous'):
            ccl.scan(np.zeros(16, np.float32)[::2], np.zeros(8, np.float32), 8, H.MPI_FLOAT,
                     H.MPI_SUM, c0)
    finally:
        for c in comms:
            assert c.free() == 0
