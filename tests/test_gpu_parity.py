"""GPU parity: the HIP path through the C-ABI against the oracle and the
golden vectors.  Bit-exact for integer, logical, bitwise, MAX/MIN and
MAXLOC/MINLOC; bit-exact for FP SUM/PROD too (one IEEE op per element on
both sides) except that a NaN result only has to be a NaN (payload bits of
arithmetic NaNs are unpinned: x86 and gfx950 pick different default NaNs).

Sizes: MPIX_PARITY_BYTES per operand (default 4 MiB) for the random sweep;
the BASELINE configs' full sizes are covered by the *_full tests.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from tests import golden_util as gu

pytestmark = pytest.mark.gpu

SWEEP_BYTES = int(os.environ.get('MPIX_PARITY_BYTES', 4 << 20))


@pytest.fixture(scope='module')
def R():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


@pytest.fixture(scope='module')
def H():
    from mpich_amd import handles
    return handles


def dev(a):
    """numpy bytes -> device uint8 tensor (synchronised)"""
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()
    torch.cuda.synchronize()
    return t


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


# --------------------------------------------------------------- generators
def gen_int(rng, n, size, logical=False):
    a = rng.integers(0, 256, n * size, dtype=np.uint8)
    if logical:
        z = rng.random(n) < 0.3
        a.reshape(n, size)[z] = 0
    return a


def gen_float(rng, n, npt):
    x = rng.uniform(-1, 1, n).astype(npt)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan], npt)
    k = rng.random(n) < 0.01
    x[k] = sp[rng.integers(0, len(sp), k.sum())]
    if npt == np.float32:
        d = rng.random(n) < 0.003        # subnormals must not be flushed
        x[d] = (rng.uniform(-1, 1, d.sum()) * 1e-39).astype(np.float32)
    return x.view(np.uint8)


def gen_bf16(rng, n):
    f = rng.uniform(-4, 4, n).astype(np.float32)
    k = rng.random(n) < 0.01
    f[k] = np.array([np.inf, -np.inf, 0.0, -0.0], np.float32)[rng.integers(0, 4, k.sum())]
    b = (f.view(np.uint32) >> 16).astype(np.uint16)
    b ^= rng.integers(0, 2, n, dtype=np.uint16)      # odd low bits: ties-away cases
    b[((b & 0x7f80) == 0x7f80) & ((b & 0x7f) != 0)] = 0x3f80
    return b.view(np.uint8)


def gen_logical(rng, n, size):
    vals = np.array([0, 1, -1, 5, 0], np.int64)
    v = vals[rng.integers(0, len(vals), n)]
    return v.astype('<i%d' % size).view(np.uint8) if size <= 8 else \
        np.stack([v, np.where(v < 0, -1, 0)], 1).astype('<i8').view(np.uint8).reshape(-1)


def gen_pair(rng, n, vdt, ldt, ext, loff, floaty):
    buf = rng.integers(0, 256, n * ext, dtype=np.uint8).reshape(n, ext)   # random padding
    if floaty:
        v = rng.integers(0, 16, n).astype(vdt)
        v[rng.random(n) < 0.02] = np.nan
    else:
        v = rng.integers(0, 16, n).astype(vdt)
    lv = rng.integers(-1000, 1000, n).astype(ldt)
    buf[:, :np.dtype(vdt).itemsize] = v.view(np.uint8).reshape(n, -1)
    buf[:, loff:loff + np.dtype(ldt).itemsize] = lv.view(np.uint8).reshape(n, -1)
    return buf.reshape(-1)


def _sweep():
    from mpich_amd import handles as H
    I = ['MPI_MAX', 'MPI_MIN', 'MPI_SUM', 'MPI_PROD', 'MPI_LAND', 'MPI_BAND', 'MPI_LOR',
         'MPI_BOR', 'MPI_LXOR', 'MPI_BXOR']
    F = ['MPI_MAX', 'MPI_MIN', 'MPI_SUM', 'MPI_PROD']
    L = ['MPI_LAND', 'MPI_LOR', 'MPI_LXOR']
    LOC = ['MPI_MAXLOC', 'MPI_MINLOC']
    out = []
    for nm, size in (('MPI_INT8_T', 1), ('MPI_INT16_T', 2), ('MPI_INT32_T', 4), ('MPI_INT64_T', 8),
                     ('MPI_UINT8_T', 1), ('MPI_UINT16_T', 2), ('MPI_UINT32_T', 4),
                     ('MPI_UINT64_T', 8), ('MPI_INTEGER16', 16), ('MPIR_UINT128', 16)):
        for op in I:
            out.append((nm, op, 'int', size))
    for op in ('MPI_BAND', 'MPI_BOR', 'MPI_BXOR'):
        out.append(('MPI_BYTE', op, 'int', 1))
    for op in L:
        out.append(('MPI_C_BOOL', op, 'int', 1))
        for nm, size in (('MPI_LOGICAL1', 1), ('MPI_LOGICAL2', 2), ('MPI_LOGICAL4', 4),
                         ('MPI_LOGICAL8', 8), ('MPI_LOGICAL16', 16)):
            out.append((nm, op, 'flog', size))
    for nm, size in (('MPIX_C_FLOAT16', 2), ('MPI_FLOAT', 4), ('MPI_DOUBLE', 8)):
        for op in F:
            out.append((nm, op, 'fp', size))
    out.append(('MPIX_BFLOAT16', 'MPI_SUM', 'bf16', 2))
    for nm, size in (('MPI_COMPLEX4', 2), ('MPI_C_FLOAT_COMPLEX', 4), ('MPI_C_DOUBLE_COMPLEX', 8)):
        for op in ('MPI_SUM', 'MPI_PROD'):
            out.append((nm, op, 'cplx', size))
    pairs = [('MPI_2INT', '<i4', '<i4', 8, 4), ('MPI_2REAL', '<f4', '<f4', 8, 4),
             ('MPI_2DOUBLE_PRECISION', '<f8', '<f8', 16, 8), ('MPI_FLOAT_INT', '<f4', '<i4', 8, 4),
             ('MPI_DOUBLE_INT', '<f8', '<i4', 16, 8), ('MPI_LONG_INT', '<i8', '<i4', 16, 8),
             ('MPI_SHORT_INT', '<i2', '<i4', 8, 4), ('MPIR_2INT8', '<i1', '<i1', 2, 1),
             ('MPIR_2INT16', '<i2', '<i2', 4, 2), ('MPIR_2INT64', '<i8', '<i8', 16, 8),
             ('MPIR_2UINT8', '<u1', '<u1', 2, 1), ('MPIR_2UINT16', '<u2', '<u2', 4, 2),
             ('MPIR_2UINT32', '<u4', '<u4', 8, 4), ('MPIR_2UINT64', '<u8', '<u8', 16, 8),
             ('MPIR_2FLOAT16', '<f2', '<f2', 4, 2)]
    for p in pairs:
        for op in LOC:
            out.append((p[0], op, ('pair',) + p[1:], None))
    del H
    return out


SWEEP = _sweep()


def make_operand(rng, kind, size, n, dtname):
    if kind == 'int':
        return gen_int(rng, n, size, logical=True)
    if kind == 'flog':
        return gen_logical(rng, n, size)
    if kind == 'fp':
        return gen_float(rng, n, {2: np.float16, 4: np.float32, 8: np.float64}[size])
    if kind == 'bf16':
        return gen_bf16(rng, n)
    if kind == 'cplx':
        return gen_float(rng, 2 * n, {2: np.float16, 4: np.float32, 8: np.float64}[size])
    vdt, ldt, ext, loff = kind[1:]
    return gen_pair(rng, n, vdt, ldt, ext, loff, vdt.startswith('<f'))


def nan_mask(raw, kind, size):
    """per-element NaN flag of a result buffer for the nan-equivalent kinds"""
    if kind == 'fp':
        return np.isnan(raw.view({2: np.float16, 4: np.float32, 8: np.float64}[size]))
    if kind == 'cplx':
        f = np.isnan(raw.view({2: np.float16, 4: np.float32, 8: np.float64}[size]))
        return f.reshape(-1, 2).any(1)
    if kind == 'bf16':
        b = raw.view(np.uint16)
        return ((b & 0x7f80) == 0x7f80) & ((b & 0x7f) != 0)
    return None


def compare(got, exp, kind, size, op, ext):
    """number of mismatching elements under the module's parity rule"""
    g = got.reshape(-1, ext)
    e = exp.reshape(-1, ext)
    bad = (g != e).any(1)
    if op in ('MPI_SUM', 'MPI_PROD') and kind in ('fp', 'cplx', 'bf16'):
        gn = nan_mask(got, kind, size)
        en = nan_mask(exp, kind, size)
        if kind == 'cplx':
            # a NaN component must be NaN on both sides, the rest bit-exact
            comp = {2: np.float16, 4: np.float32, 8: np.float64}[size]
            gc, ec = got.view(comp).reshape(-1, 2), exp.view(comp).reshape(-1, 2)
            gcn, ecn = np.isnan(gc), np.isnan(ec)
            cmp_bits = (gc.view(np.uint8).reshape(len(gc), 2, size) !=
                        ec.view(np.uint8).reshape(len(ec), 2, size)).any(2)
            cbad = np.where(gcn | ecn, gcn != ecn, cmp_bits).any(1)
            return int(cbad.sum())
        bad = np.where(gn | en, gn != en, bad)
    return int(bad.sum())


@pytest.mark.parametrize('dtname,opname,kind,size', SWEEP,
                         ids=['%s-%s' % (s[0], s[1]) for s in SWEEP])
def test_random_parity(R, H, oracle, dtname, opname, kind, size):
    dt, op = getattr(H, dtname), getattr(H, opname)
    assert R.is_supported(op, dt), (dtname, opname)
    ext = R.datatype_extent(dt)
    n = max(1, SWEEP_BYTES // ext) + 7          # ragged: not a multiple of any packet
    rng = np.random.default_rng((0x5EED0003 * 31 + dt * 7 + op) & 0xffffffff)
    a = make_operand(rng, kind, size, n, dtname)
    b = make_operand(rng, kind, size, n, dtname)
    exp = a.copy()
    assert oracle.reduce_local(b.copy(), exp, n, dt, op) == 0
    da, db = dev(a), dev(b)
    assert R.MPI_Reduce_local(db, da, n, dt, op) == 0
    got = host(da)
    assert np.array_equal(host(db), b)          # inbuf untouched
    assert compare(got, exp, kind, size, opname, ext) == 0


@pytest.mark.parametrize('case', gu.load_cases(), ids=lambda c: c['id'] + ' ' + c['name'])
def test_golden_on_gpu(R, case):
    # every golden case has a GPU path, the MPI_LONG_DOUBLE_INT MAXLOC/MINLOC
    # cases (opmaxloc.c / opminloc.c) included since round 4
    assert R.is_supported(case['op'], case['datatype'])

    def fn(inb, inoutb, count, dt, op):
        di, dio = dev(inb), dev(inoutb)
        rc = R.MPI_Reduce_local(di, dio, count, dt, op)
        inoutb[:] = host(dio)
        return rc
    rc, acc = gu.fold(case, fn)
    assert rc == 0
    assert gu.mismatches(case, acc) == 0


@pytest.mark.parametrize('case', gu.load_cases(), ids=lambda c: c['id'] + ' ' + c['name'])
def test_golden_on_gpu_async(R, case):
    """the same golden cases through the stream-ordered entry (caller's
    stream, no library wait) -- same bits as the synchronous calls."""
    if not R.is_supported(case['op'], case['datatype']):
        return
    s = torch.cuda.current_stream()

    def fn(inb, inoutb, count, dt, op):
        di, dio = dev(inb), dev(inoutb)
        rc = R.reduce_local_async(di, dio, count, dt, op, s)
        inoutb[:] = host(dio)
        return rc
    rc, acc = gu.fold(case, fn)
    assert rc == 0
    assert gu.mismatches(case, acc) == 0


@pytest.mark.parametrize('tname', ['MPI_INT8_T', 'MPIX_C_FLOAT16', 'MPI_FLOAT', 'MPI_DOUBLE',
                                   'MPI_C_DOUBLE_COMPLEX', 'MPI_2INT', 'MPI_DOUBLE_INT'])
@pytest.mark.parametrize('delta', [-1, 0, 1])
@pytest.mark.parametrize('offs', [(0, 0), (0, 2), (6, 0)])
def test_small_kernel_boundary(R, H, oracle, tname, delta, offs):
    """counts around 16 KiB per operand for 1- to 16-byte elements, with
    byte-offset operands (head/tail, unaligned-load and element paths)."""
    dt = getattr(H, tname)
    ext = R.datatype_extent(dt)
    op = H.MPI_MAXLOC if 'INT' in tname and tname.startswith('MPI_2') or tname == 'MPI_DOUBLE_INT' \
        else H.MPI_SUM
    count = (16384 // ext) + delta
    nb = count * ext + 16
    rng = np.random.default_rng(count * 7 + offs[1])
    a = rng.integers(0, 4, nb).astype(np.uint8)
    b = rng.integers(0, 4, nb).astype(np.uint8)
    da, db = dev(a), dev(b)
    oa, ob = offs
    assert R.MPI_Reduce_local(db.data_ptr() + ob, da.data_ptr() + oa, count, dt, op) == 0
    exp = a.copy()
    oracle.reduce_local(b[ob:ob + count * ext].copy(), exp[oa:], count, dt, op)
    assert np.array_equal(host(da), exp)


@pytest.mark.parametrize('count', [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 1023, 4099,
                                   (1 << 20) + 3])
@pytest.mark.parametrize('offs', [(0, 0), (4, 4), (8, 8), (12, 12), (0, 4), (4, 0), (8, 12)])
def test_ragged_and_misaligned(R, H, oracle, count, offs):
    """head/tail element paths and the element-wise (relatively misaligned)
    kernel, fp32 SUM, against the oracle."""
    rng = np.random.default_rng(count * 131 + offs[0] * 7 + offs[1])
    a = rng.uniform(-1, 1, count + 8).astype(np.float32)
    b = rng.uniform(-1, 1, count + 8).astype(np.float32)
    da, db = dev(a), dev(b)
    oa, ob = offs
    assert R.MPI_Reduce_local(db.data_ptr() + ob, da.data_ptr() + oa, count, H.MPI_FLOAT,
                              H.MPI_SUM) == 0
    exp = a.copy()
    ev = exp.view(np.uint8)[oa:oa + 4 * count].view(np.float32)
    bv = b.view(np.uint8)[ob:ob + 4 * count].view(np.float32).copy()
    oracle.reduce_local(bv, ev, count, H.MPI_FLOAT, H.MPI_SUM)
    assert np.array_equal(host(da).view(np.float32), exp)


@pytest.mark.parametrize('dtname,opname,kind,size', SWEEP,
                         ids=['%s-%s' % (s[0], s[1]) for s in SWEEP])
def test_relative_misalignment(R, H, oracle, dtname, opname, kind, size):
    """every (op, type) with `in` and `inout` at different 16-byte phases
    (the packet kernel's unaligned-`in` form) and, for multi-byte units, at
    byte offsets that are not even element-aligned (the element-wise kernel);
    ragged counts, inbuf untouched, the sweep's parity rule"""
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = R.datatype_extent(dt)
    n = (1 << 16) // ext + 5
    rng = np.random.default_rng((0x5EED0007 * 17 + dt * 5 + op) & 0xffffffff)
    offs = [(0, ext), (ext, 0), (3 * ext, 16 - ext if ext < 16 else 32)]
    if ext > 1:
        offs += [(1, 0), (0, 3)]
    for oa, ob in offs:
        a = make_operand(rng, kind, size, n, dtname).view(np.uint8)
        b = make_operand(rng, kind, size, n, dtname).view(np.uint8)
        pa = np.zeros(n * ext + 64, np.uint8)
        pb = np.zeros(n * ext + 64, np.uint8)
        pa[oa:oa + n * ext] = a
        pb[ob:ob + n * ext] = b
        da, db = dev(pa), dev(pb)
        assert R.MPI_Reduce_local(db.data_ptr() + ob, da.data_ptr() + oa, n, dt, op) == 0
        exp = a.copy()
        assert oracle.reduce_local(b.copy(), exp, n, dt, op) == 0
        got = host(da)
        assert not got[:oa].any() and not got[oa + n * ext:].any(), (oa, ob)   # no spill-over
        assert np.array_equal(host(db)[ob:ob + n * ext], b)
        assert compare(got[oa:oa + n * ext].copy(), exp, kind, size, opname, ext) == 0, (oa, ob)


@pytest.mark.parametrize('dtname,ext', [('MPI_CHAR', 1), ('MPI_SHORT', 2), ('MPI_DOUBLE', 8),
                                        ('MPI_C_DOUBLE_COMPLEX', 16)])
def test_ragged_small_units(R, H, oracle, dtname, ext):
    dt = getattr(H, dtname)
    for count in (1, 7, 15, 33, 1000):
        for off in (0, ext, 3 * ext):
            rng = np.random.default_rng(count + off)
            a = rng.integers(0, 256, (count + 8) * ext, dtype=np.uint8)
            b = rng.integers(0, 256, (count + 8) * ext, dtype=np.uint8)
            if dtname == 'MPI_DOUBLE' or 'COMPLEX' in dtname:
                a = rng.uniform(-1, 1, len(a) // 8).view(np.uint8)
                b = rng.uniform(-1, 1, len(b) // 8).view(np.uint8)
            da, db = dev(a), dev(b)
            assert R.MPI_Reduce_local(db.data_ptr() + off, da.data_ptr() + off, count, dt,
                                      H.MPI_SUM) == 0
            exp = a.copy()
            oracle.reduce_local(b[off:off + count * ext].copy(), exp[off:], count, dt, H.MPI_SUM)
            assert np.array_equal(host(da), exp)


def test_host_buffers_are_staged(R, H, oracle):
    """host (pageable numpy) operands go H2D -> kernel -> D2H in chunks."""
    rng = np.random.default_rng(7)
    n = (3 << 20) + 5
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    exp = a.copy()
    oracle.reduce_local(b, exp, n, H.MPI_FLOAT, H.MPI_SUM)
    got = a.copy()
    assert R.MPI_Reduce_local(b, got, n, H.MPI_FLOAT, H.MPI_SUM) == 0
    assert np.array_equal(got, exp)
    # mixed: device in, host inout; and pinned host
    got = a.copy()
    assert R.MPI_Reduce_local(dev(b), got, n, H.MPI_FLOAT, H.MPI_SUM) == 0
    assert np.array_equal(got, exp)
    pa = torch.from_numpy(a.copy()).pin_memory()
    pb = torch.from_numpy(b.copy()).pin_memory()
    assert R.MPI_Reduce_local(pb, pa, n, H.MPI_FLOAT, H.MPI_SUM) == 0
    assert np.array_equal(pa.numpy(), exp)


@pytest.mark.parametrize('nbytes', [1, 8, 4096, 65536, (1 << 20) - 8, 1 << 20, (1 << 20) + 8,
                                    1 << 21])
@pytest.mark.parametrize('place', ['both_host', 'host_in', 'host_inout', 'pinned_in'])
def test_small_pageable_bounce(R, H, oracle, nbytes, place):
    """pageable operands up to MPIX_REDOP_BOUNCE_BYTES (1 MiB) go through the
    pinned bounce buffer, larger ones through the staged path; results must
    not depend on the route.  MAXLOC on MPI_2INT and int8 SUM as well."""
    rng = np.random.default_rng(nbytes)
    for dt, op, T in ((H.MPI_FLOAT, H.MPI_SUM, np.float32), (H.MPI_INT8_T, H.MPI_SUM, np.int8),
                      (H.MPI_2INT, H.MPI_MAXLOC, np.int32)):
        ext = R.datatype_extent(dt)
        n = max(1, nbytes // ext)
        w = n * ext // np.dtype(T).itemsize
        if T == np.float32:
            a = rng.uniform(-1, 1, w).astype(T)
            b = rng.uniform(-1, 1, w).astype(T)
        else:
            a = rng.integers(-8, 8, w).astype(T)
            b = rng.integers(-8, 8, w).astype(T)
        exp = a.copy()
        oracle.reduce_local(b.copy(), exp, n, dt, op)
        got = a.copy()
        if place == 'both_host':
            assert R.MPI_Reduce_local(b, got, n, dt, op) == 0
        elif place == 'host_in':
            dgot = dev(got)
            assert R.MPI_Reduce_local(b, dgot, n, dt, op) == 0
            got = host(dgot).view(T)
        elif place == 'host_inout':
            assert R.MPI_Reduce_local(dev(b), got, n, dt, op) == 0
        else:
            pb = torch.from_numpy(b.copy()).pin_memory()
            assert R.MPI_Reduce_local(pb, got, n, dt, op) == 0
        assert np.array_equal(got.view(np.uint8), exp.view(np.uint8)), (dt, place)


def test_async_on_torch_stream(R, H, oracle):
    rng = np.random.default_rng(11)
    n = 1 << 22
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        da = torch.from_numpy(a).cuda(non_blocking=False)
        db = torch.from_numpy(b).cuda(non_blocking=False)
        for _ in range(3):
            assert R.reduce_local_async(db, da, n, H.MPI_FLOAT, H.MPI_SUM) == 0
    s.synchronize()
    exp = a.copy()
    for _ in range(3):
        oracle.reduce_local(b, exp, n, H.MPI_FLOAT, H.MPI_SUM)
    assert np.array_equal(da.cpu().numpy(), exp)


def test_op_table_functions(R, H, oracle):
    """MPIR_op_function ABI (mpir_op.h:206): len and type by pointer."""
    L = R.lib()
    tab = (ctypes.c_void_p * 16).in_dll(L, 'MPIX_Op_table')
    fnt = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.POINTER(ctypes.c_ssize_t), ctypes.POINTER(ctypes.c_int))
    rng = np.random.default_rng(3)
    n = 100003
    for opi in (1, 2, 3, 4, 6, 8, 10):
        a = rng.integers(-1000, 1000, n).astype(np.int32)
        b = rng.integers(-1000, 1000, n).astype(np.int32)
        da, db = dev(a), dev(b)
        ln = ctypes.c_ssize_t(n)
        ty = ctypes.c_int(H.as_c_int(0x4c810405))       # MPIR_INT32 | MPI_INT's index
        fnt(tab[opi])(db.data_ptr(), da.data_ptr(), ctypes.byref(ln), ctypes.byref(ty))
        assert L.MPIX_Redop_last_error() == 0
        exp = a.copy()
        oracle.reduce_local(b, exp, n, 0x4c810405, 0x58000000 | opi)
        assert np.array_equal(host(da).view(np.int32), exp), opi


def test_errors_on_gpu(R, H):
    x = torch.zeros(1 << 16, device='cuda')
    y = torch.zeros(1 << 16, device='cuda')
    assert R.MPI_Reduce_local(x, x, 1024, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(-1, y, 1024, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    assert R.MPI_Reduce_local(x, y, 1024, H.MPIX_BFLOAT16, H.MPI_MIN) == H.MPI_ERR_TYPE
    assert R.MPI_Reduce_local(x, y, 1024, H.MPIX_BFLOAT16, H.MPI_MAX) == H.MPI_ERR_TYPE
    assert R.MPI_Reduce_local(x, y, 10, H.MPI_FLOAT, H.MPI_LXOR) == H.MPI_ERR_OP
    assert R.MPI_Reduce_local(x, y, 0, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_SUCCESS


def test_fortran_booleans(R, H, oracle):
    """MPII_TO/FROM_FLOG with a non-default .TRUE. (e.g. -1)."""
    rng = np.random.default_rng(5)
    n = 4097
    a = rng.integers(-2, 3, n).astype(np.int32)
    b = rng.integers(-2, 3, n).astype(np.int32)
    try:
        R.set_fortran_booleans(-1, 0)
        oracle.set_fortran_booleans(-1, 0)
        for op in (H.MPI_LAND, H.MPI_LOR, H.MPI_LXOR):
            da, db = dev(a), dev(b)
            assert R.MPI_Reduce_local(db, da, n, H.MPI_LOGICAL, op) == 0
            exp = a.copy()
            oracle.reduce_local(b, exp, n, H.MPI_LOGICAL, op)
            assert np.array_equal(host(da).view(np.int32), exp)
    finally:
        R.set_fortran_booleans(1, 0)
        oracle.set_fortran_booleans(1, 0)


def _flog_operand(rng, n, size, tv, fv):
    """n logicals of `size` bytes: the kind's own truncations of .TRUE. and
    .FALSE., 0, 1, -1 and random words; LOGICAL16 words are sign-extended
    int64 or carry random high halves (the comparison is full width)"""
    pick = np.array([tv, fv, 0, 1, -1], dtype=np.int64)
    lo = np.where(rng.random(n) < 0.8, pick[rng.integers(0, 5, n)],
                  rng.integers(-(1 << 62), 1 << 62, n))
    if size == 16:
        hi = np.where(lo < 0, -1, 0)
        hi = np.where(rng.random(n) < 0.1, rng.integers(-(1 << 62), 1 << 62, n), hi)
        return np.stack([lo, hi], 1).astype(np.int64).view(np.uint8).reshape(-1)
    return lo.astype({1: np.int8, 2: np.int16, 4: np.int32, 8: np.int64}[size]).view(np.uint8)


@pytest.mark.parametrize('kind,size', [('MPI_LOGICAL1', 1), ('MPI_LOGICAL2', 2), ('MPI_LOGICAL4', 4),
                                       ('MPI_LOGICAL8', 8), ('MPI_LOGICAL16', 16)])
@pytest.mark.parametrize('tv,fv', [(1, 0), (-1, 0), (5, -3), (300, 7), (7, 300), (0, 1)])
def test_fortran_logical_kinds(R, H, oracle, kind, size, tv, fv):
    """MPII_FROM_FLOG compares each kind after C's promotion against an int
    .FALSE. (mpii_fortlogical.h:13,29) and MPII_TO_FLOG casts .TRUE./.FALSE.
    back to the kind: every logical kind, booleans that do and do not fit it"""
    dt = getattr(H, kind)
    n = 20011
    rng = np.random.default_rng(size * 1000 + (tv & 0xff) * 7 + (fv & 0xff))
    a = _flog_operand(rng, n, size, tv, fv)
    b = _flog_operand(rng, n, size, tv, fv)
    try:
        R.set_fortran_booleans(tv, fv)
        oracle.set_fortran_booleans(tv, fv)
        for op in (H.MPI_LAND, H.MPI_LOR, H.MPI_LXOR):
            da, db = dev(a), dev(b)
            assert R.MPI_Reduce_local(db, da, n, dt, op) == 0
            exp = a.copy()
            assert oracle.reduce_local(b.copy(), exp, n, dt, op) == 0
            assert np.array_equal(host(da), exp), (kind, tv, fv, op)
    finally:
        R.set_fortran_booleans(1, 0)
        oracle.set_fortran_booleans(1, 0)


@pytest.mark.parametrize('blocklen,stride', [(1, 2), (1, 3), (3, 7), (4, 4), (5, 8)])
def test_vector_target(R, H, oracle, blocklen, stride):
    """config 5 semantics (typerep_op.c:115-150): vector target, packed source;
    gap elements must be untouched."""
    rng = np.random.default_rng(blocklen * 10 + stride)
    count = 100003
    src = rng.uniform(-1, 1, count * blocklen)
    dst = rng.uniform(-1, 1, count * stride)
    dd, ds = dev(dst), dev(src)
    assert R.reduce_local_vector(ds, dd, count, blocklen, stride, H.MPI_DOUBLE, H.MPI_SUM,
                                 sync=True) == 0
    exp = dst.copy()
    oracle.reduce_local_vector(src, exp, count, blocklen, stride, H.MPI_DOUBLE, H.MPI_SUM)
    assert np.array_equal(host(dd).view(np.float64), exp)


def test_acc_pairtype_on_gpu(R, H):
    """test/mpi/rma/acc_pairtype.c's check (MAXLOC of {1.0, 1} pairs into a
    zeroed vector(10, 3, 5) target; MPI_DOUBLE_INT for the x87 pair)."""
    from tests.test_oracle_golden import _acc_pairtype_case
    src, tgt, exp = _acc_pairtype_case()
    dt = dev(tgt.view(np.uint8))
    assert R.reduce_local_vector(dev(src.view(np.uint8)), dt, 10, 3, 5, H.MPI_DOUBLE_INT,
                                 H.MPI_MAXLOC, sync=True) == 0
    assert host(dt).tobytes() == exp.view(np.uint8).tobytes()


@pytest.mark.parametrize('tname', ['MPI_2INT', 'MPI_FLOAT_INT', 'MPI_DOUBLE_INT', 'MPI_LONG_INT',
                                   'MPI_SHORT_INT', 'MPI_2DOUBLE_PRECISION'])
@pytest.mark.parametrize('blocklen,stride', [(1, 2), (3, 5)])
def test_vector_target_pairs(R, H, oracle, tname, blocklen, stride):
    """MAXLOC / MINLOC through the vector target for every pair layout
    (ties and random padding included) against the oracle."""
    dt = getattr(H, tname)
    ext = R.datatype_extent(dt)
    rng = np.random.default_rng(ext * 31 + stride)
    count = 20011
    for op in (H.MPI_MAXLOC, H.MPI_MINLOC):
        src = rng.integers(0, 3, count * blocklen * ext).astype(np.uint8)
        dst = rng.integers(0, 3, count * stride * ext).astype(np.uint8)
        dd = dev(dst)
        assert R.reduce_local_vector(dev(src), dd, count, blocklen, stride, dt, op,
                                     sync=True) == 0
        exp = dst.copy()
        assert oracle.reduce_local_vector(src, exp, count, blocklen, stride, dt, op) == 0
        assert np.array_equal(host(dd), exp), (tname, op)


def test_full_1gib_fp32_sum(R, H, oracle):
    """BASELINE config 2 at its largest size: 1 GiB per operand, checked
    element-for-element against the oracle (8 host threads)."""
    n = 1 << 28
    rng = np.random.default_rng(0x5EED0001)
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    da = torch.from_numpy(a).cuda()
    db = torch.from_numpy(b).cuda()
    torch.cuda.synchronize()
    assert R.MPI_Reduce_local(db, da, n, H.MPI_FLOAT, H.MPI_SUM) == 0
    oracle.reduce_local(b, a, n, H.MPI_FLOAT, H.MPI_SUM, nthreads=8)
    got = da.cpu().numpy()
    assert np.array_equal(got, a)
    del da, db
    torch.cuda.empty_cache()


def test_full_vector_stride2_fp64(R, H, oracle):
    """BASELINE config 5 at full size: vector(67108864, 1, 2, MPI_DOUBLE)."""
    count = 67108864
    rng = np.random.default_rng(0x5EED0005)
    src = rng.uniform(-1, 1, count)
    dst = rng.uniform(-1, 1, 2 * count)
    dd, ds = torch.from_numpy(dst).cuda(), torch.from_numpy(src).cuda()
    torch.cuda.synchronize()
    assert R.reduce_local_vector(ds, dd, count, 1, 2, H.MPI_DOUBLE, H.MPI_SUM, sync=True) == 0
    oracle.reduce_local_vector(src, dst, count, 1, 2, H.MPI_DOUBLE, H.MPI_SUM)
    assert np.array_equal(dd.cpu().numpy(), dst)
    del dd, ds
    torch.cuda.empty_cache()


@pytest.mark.parametrize('k', [1, 2, 7, 16])
@pytest.mark.parametrize('dtname,opname', [('MPI_FLOAT', 'MPI_SUM'), ('MPI_DOUBLE', 'MPI_PROD'),
                                           ('MPI_INT', 'MPI_MAX'), ('MPI_2INT', 'MPI_MINLOC'),
                                           ('MPIX_C_FLOAT16', 'MPI_SUM'),
                                           ('MPI_C_FLOAT_COMPLEX', 'MPI_PROD')])
def test_multi_input_combine(R, H, oracle, k, dtname, opname):
    """MPIX_Reduce_local_multi_async == k sequential MPI_Reduce_local calls
    (same association, so bit-exact), incl. ragged/unaligned element paths."""
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = R.datatype_extent(dt)
    for n, off in ((100003, 0), (4097, ext)):
        rng = np.random.default_rng(k * 1000 + n)
        if dtname in ('MPI_INT', 'MPI_2INT'):
            mk = lambda: rng.integers(-50, 50, n * ext // 4 + 4).astype(np.int32).view(np.uint8)  # noqa
        elif dtname == 'MPIX_C_FLOAT16':
            mk = lambda: rng.uniform(-1, 1, n + 8).astype(np.float16).view(np.uint8)  # noqa
        else:
            mk = lambda: rng.uniform(-1, 1, n * ext // 4 + 4).astype(np.float32).view(np.uint8) \
                if ext % 4 == 0 and dtname != 'MPI_DOUBLE' else \
                rng.uniform(-1, 1, n * ext // 8 + 2).astype(np.float64).view(np.uint8)  # noqa
        acc = mk()
        ins = [mk() for _ in range(k)]
        exp = acc.copy()
        for x in ins:
            oracle.reduce_local(x[off:off + n * ext].copy(), exp[off:], n, dt, op)
        dacc = dev(acc)
        dins = [dev(x) for x in ins]
        rc = R.reduce_local_multi_async([d.data_ptr() + off for d in dins], dacc.data_ptr() + off,
                                        n, dt, op)
        assert rc == 0
        got = host(dacc)
        kind = 'cplx' if 'COMPLEX' in dtname else \
            ('fp' if 'FLOAT' in dtname or 'DOUBLE' in dtname else 'int')
        assert compare(got[off:off + n * ext], exp[off:off + n * ext], kind,
                       {'MPI_FLOAT': 4, 'MPI_DOUBLE': 8, 'MPIX_C_FLOAT16': 2}.get(dtname, 4),
                       opname, ext) == 0


def _special_f64(rng, n):
    """doubles with NaN (two payloads), +-0, +-Inf mixed in: MAX/MIN pick by
    operand role, so the tree's inout/in assignment shows in the bits"""
    x = rng.uniform(-1, 1, n)
    pick = rng.integers(0, 8, n)
    x[pick == 0] = 0.0
    x[pick == 1] = -0.0
    x[pick == 2] = np.frombuffer(np.array([0x7ff8000000000001], np.uint64).tobytes(), np.float64)[0]
    x[pick == 3] = np.frombuffer(np.array([0xfff8000000000abc], np.uint64).tobytes(), np.float64)[0]
    x[pick == 4] = np.inf
    return x


@pytest.mark.parametrize('k', [2, 4, 8, 16])
@pytest.mark.parametrize('dtname,opname', [('MPI_FLOAT', 'MPI_SUM'), ('MPI_DOUBLE', 'MPI_MAX'),
                                           ('MPI_DOUBLE', 'MPI_MIN'), ('MPI_INT', 'MPI_PROD'),
                                           ('MPI_2INT', 'MPI_MAXLOC'), ('MPI_DOUBLE_INT', 'MPI_MINLOC'),
                                           ('MPIX_BFLOAT16', 'MPI_SUM'),
                                           ('MPI_C_DOUBLE_COMPLEX', 'MPI_PROD'),
                                           ('MPI_FLOAT', 'MPI_REPLACE'), ('MPI_FLOAT', 'MPI_NO_OP')])
def test_tree_combine(R, H, oracle, k, dtname, opname):
    """MPIX_Reduce_local_tree_async == the level-by-level fold done with
    MPI_Reduce_local calls (slot s = slot s OP slot s+m, m = 1, 2, 4, ...;
    an absent slot's partner passes through): bit-exact, NaN payloads and +-0
    included; packet path, unaligned element path and in place (out = slot 0)"""
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = R.datatype_extent(dt)
    # in_place: None, or the slot whose buffer is also the output
    for n, off, in_place in ((100003, 0, None), (4097, 4 if ext % 8 else 8, None),
                             (65536 + 5, 0, 0), (65536 + 5, 0, 1)):
        rng = np.random.default_rng(k * 7919 + n + (0 if in_place is None else 1 + in_place))
        nb = n * ext + 64

        def mk():
            if dtname in ('MPI_INT', 'MPI_2INT'):
                return rng.integers(0, 4, nb // 4).astype(np.int32).view(np.uint8)
            if dtname == 'MPI_DOUBLE_INT':      # {double value; int loc} + pad: ties likely
                a = np.zeros(nb // 16, dtype=[('v', '<f8'), ('l', '<i4'), ('p', '<i4')])
                a['v'] = rng.integers(0, 3, a.size)
                a['l'] = rng.integers(0, 50, a.size)
                return a.view(np.uint8).copy()
            if dtname == 'MPIX_BFLOAT16':
                return (rng.integers(0, 1 << 16, nb // 2).astype(np.uint16) & 0x7f7f).view(np.uint8)
            if dtname == 'MPI_DOUBLE' or 'COMPLEX' in dtname:
                return _special_f64(rng, nb // 8).view(np.uint8) if dtname == 'MPI_DOUBLE' else \
                    rng.uniform(-1, 1, nb // 8).view(np.uint8)
            return rng.uniform(-1, 1, nb // 4).astype(np.float32).view(np.uint8)
        ins = [mk() for _ in range(k)]
        # absent slots (None): every odd slot above k/2, as the fold of a
        # non-power-of-two world leaves them (slot 0 always present)
        absent = {q for q in range(k) if q % 2 and q > k // 2} if k >= 4 else set()
        v = [None if q in absent else x[off:off + n * ext].copy() for q, x in enumerate(ins)]
        m = 1
        while m < k:
            for q in range(0, k, 2 * m):
                if v[q] is not None and v[q + m] is not None:
                    oracle.reduce_local(v[q + m], v[q], n, dt, op)
                elif v[q + m] is not None:
                    v[q] = v[q + m]
            m *= 2
        exp = v[0]
        dins = [None if q in absent else dev(x) for q, x in enumerate(ins)]
        if in_place is not None:
            dout, oo = dins[in_place], off
        else:
            dout, oo = dev(np.zeros(nb, np.uint8)), off
        rc = R.reduce_local_tree_async([None if d is None else d.data_ptr() + off for d in dins],
                                       dout.data_ptr() + oo, n, dt, op)
        assert rc == 0, rc
        got = host(dout)[oo:oo + n * ext]
        assert got.tobytes() == exp.tobytes(), (n, off, in_place)


def test_concurrent_callers(R, H, oracle):
    """MPIR_Reduce_local is reentrant (called with the global CS held by
    different threads under MPI_THREAD_MULTIPLE): per-thread streams, no
    shared state on the data path."""
    import threading
    n = (1 << 20) + 11
    rng = np.random.default_rng(99)
    jobs = []
    for t in range(8):
        a = rng.uniform(-1, 1, n).astype(np.float32)
        b = rng.uniform(-1, 1, n).astype(np.float32)
        exp = a.copy()
        for _ in range(5):
            oracle.reduce_local(b, exp, n, H.MPI_FLOAT, H.MPI_SUM)
        jobs.append((dev(a), dev(b), exp))
    errs = []

    def work(da, db):
        torch.cuda.set_device(0)
        for _ in range(5):
            rc = R.MPI_Reduce_local(db, da, n, H.MPI_FLOAT, H.MPI_SUM)
            if rc:
                errs.append(rc)
        R.finalize()        # per-thread streams released; later calls re-create them

    th = [threading.Thread(target=work, args=(da, db)) for da, db, _ in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    for da, _, exp in jobs:
        assert np.array_equal(host(da).view(np.float32), exp)
    # library still usable from this thread after other threads finalized theirs
    x, y = dev(np.ones(1000, np.float32)), dev(np.ones(1000, np.float32))
    assert R.MPI_Reduce_local(x, y, 1000, H.MPI_FLOAT, H.MPI_SUM) == 0
    assert np.all(host(y).view(np.float32) == 2)


@pytest.mark.parametrize('n', [1, 7, 4096, 4100, 8192, 65536, 65540, 65600, 300000])
@pytest.mark.parametrize('off', [0, 4, 2])
def test_sync_result_visible_on_return(R, H, n, off):
    """The synchronous call returns when the completion word arrives -- for
    small launches the kernel stores it itself (Params::done, up to 4
    workgroups, the last one counted on a device word).  The result must be
    complete then: copied on torch's stream (not ordered after the library's
    stream) and read from zero-copy pinned memory with no synchronisation at
    all.  off = 2 bytes: int32 not element-aligned, the element-wise kernel
    (stream-written word); off = 4: the packet kernel with a head."""
    rng = np.random.default_rng(n + off)
    a = rng.integers(-1000, 1000, n, dtype=np.int32)
    b = rng.integers(-1000, 1000, n, dtype=np.int32)
    exp = a + b
    pad = np.zeros(off, np.uint8)
    da = dev(np.concatenate([pad, a.view(np.uint8)]))
    db = dev(b)
    for rep in range(3):
        if rep:     # inout back to a, then a full device sync
            da[off:] = dev(a)
            torch.cuda.synchronize()
        assert R.MPI_Reduce_local(db, da[off:], n, H.MPI_INT, H.MPI_SUM) == 0
        snap = da[off:].clone()             # torch stream, no wait on the library's
        assert np.array_equal(host(snap).view(np.int32), exp)
    # zero-copy pinned inout, read by the host right after the call
    hio = torch.from_numpy(a.copy()).pin_memory()
    assert R.MPI_Reduce_local(db, hio, n, H.MPI_INT, H.MPI_SUM) == 0
    assert np.array_equal(hio.numpy(), exp)


def test_thread_churn(R, H):
    """Worker threads that exit without finalizing hand their streams to a
    pool that later threads take over (redop_capi.cpp DevHolder): 96
    short-lived threads, 8 at a time, each reducing its own slice."""
    import threading
    n, nthreads = 4099, 96
    a = dev(np.arange(n * nthreads, dtype=np.int64))
    b = dev(np.full(n * nthreads, 3, np.int64))
    errs = []

    def work(t):
        torch.cuda.set_device(0)
        off = t * n * 8
        rc = R.MPI_Reduce_local(b[off:], a[off:], n, H.MPI_LONG, H.MPI_SUM)
        if rc:
            errs.append(rc)

    for base in range(0, nthreads, 8):
        th = [threading.Thread(target=work, args=(t,)) for t in range(base, base + 8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not errs
    assert np.array_equal(host(a).view(np.int64), np.arange(n * nthreads, dtype=np.int64) + 3)


@pytest.mark.parametrize('dtname,opname', [('MPI_DOUBLE', 'MPI_SUM'), ('MPI_INT', 'MPI_BXOR'),
                                           ('MPI_C_FLOAT_COMPLEX', 'MPI_PROD'),
                                           ('MPI_SHORT', 'MPI_MIN')])
def test_iov_target(R, H, oracle, dtname, opname):
    """general derived target via its flattened iov (MPI_Type_indexed-like,
    ragged segments incl. empty ones) against the oracle."""
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = R.datatype_extent(dt)
    rng = np.random.default_rng(ext * 17)
    nseg = 20000
    cnts = rng.integers(0, 9, nseg)
    gaps = rng.integers(0, 5, nseg)
    offs, pos = [], 0
    for c, g in zip(cnts, gaps):
        pos += int(g)
        offs.append(pos * ext)
        pos += int(c)
    total = int(cnts.sum())
    if ext >= 4:
        src = rng.uniform(-1, 1, total * ext // 4).astype(np.float32).view(np.uint8)
        dst = rng.uniform(-1, 1, pos * ext // 4 + 4).astype(np.float32).view(np.uint8)
    else:
        src = rng.integers(-30000, 30000, total).astype(np.int16).view(np.uint8)
        dst = rng.integers(-30000, 30000, pos + 8).astype(np.int16).view(np.uint8)
    if dtname == 'MPI_DOUBLE':
        src = rng.uniform(-1, 1, total).view(np.uint8)
        dst = rng.uniform(-1, 1, pos + 1).view(np.uint8)
    dd, ds = dev(dst), dev(src)
    assert R.reduce_local_iov_async(ds, dd, offs, [int(c) for c in cnts], dt, op) == 0
    exp = dst.copy()
    assert oracle.reduce_local_iov(src, exp, offs, [int(c) for c in cnts], dt, op) == 0
    assert np.array_equal(host(dd), exp)


def test_async_is_graph_capturable(R, H, oracle):
    """The stream-ordered entry can be captured into a HIP graph (via
    torch.cuda.graph) and replayed: launch-bound chunked reductions replay
    without per-call host launch cost."""
    n, chunks = 1 << 16, 64
    rng = np.random.default_rng(1234)
    a = rng.uniform(-1, 1, n * chunks).astype(np.float32)
    b = rng.uniform(-1, 1, n * chunks).astype(np.float32)
    da, db = dev(a), dev(b)
    fa = da.view(torch.float32)
    fb = db.view(torch.float32)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for k in range(chunks):
                rc = R.reduce_local_async(fb[k * n:], fa[k * n:], n, H.MPI_FLOAT, H.MPI_SUM)
                assert rc == 0
    torch.cuda.synchronize()
    # capture does not execute: inout unchanged
    assert np.array_equal(host(da).view(np.float32), a)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    exp = a.copy()
    for _ in range(3):
        oracle.reduce_local(b, exp, n * chunks, H.MPI_FLOAT, H.MPI_SUM)
    assert np.array_equal(host(da).view(np.float32), exp)


def test_async_refuses_pageable_host(R, H):
    """a pageable host pointer in a stream-ordered call must be refused
    (a kernel touching it would fault the GPU), pinned host is accepted."""
    a = np.ones(4096, np.float32)
    b = np.ones(4096, np.float32)
    assert R.reduce_local_async(b, a, 4096, H.MPI_FLOAT, H.MPI_SUM) == H.MPI_ERR_BUFFER
    pa = torch.ones(4096).pin_memory()
    pb = torch.ones(4096).pin_memory()
    assert R.reduce_local_async(pb, pa, 4096, H.MPI_FLOAT, H.MPI_SUM) == 0
    torch.cuda.synchronize()
    assert torch.all(pa == 2)
    assert R.reduce_local_multi_async([b], torch.zeros(4096, device='cuda'), 4096, H.MPI_FLOAT,
                                      H.MPI_SUM) == H.MPI_ERR_BUFFER


@pytest.mark.parametrize('nbytes', [8, 9, 24, 4099, (1 << 20) + 13])
def test_equal_op(R, H, oracle, nbytes):
    """MPIX_EQUAL (opequal.c:20-35) on the GPU against the oracle."""
    rng = np.random.default_rng(nbytes)
    base = rng.integers(0, 256, nbytes, dtype=np.uint8)
    base[:8] = np.array([1], '<u8').view(np.uint8)
    variants = [base.copy()]
    if nbytes > 8:
        v = base.copy()
        v[int(rng.integers(8, nbytes))] ^= 0x40
        variants.append(v)
    v = base.copy()
    v[:8] = 0
    variants.append(v)
    for other in variants:
        for a, b in ((base, other), (other, base)):
            da, db = dev(a), dev(b)
            assert R.MPI_Reduce_local(db, da, nbytes, H.MPI_BYTE, 0x5800000f) == 0
            exp = a.copy()
            assert oracle.reduce_local(b.copy(), exp, nbytes, H.MPI_BYTE, 0x5800000f) == 0
            assert np.array_equal(host(da), exp)
    assert R.MPI_Reduce_local(dev(base), dev(base), nbytes, H.MPI_INT, 0x5800000f) != 0


@pytest.mark.parametrize('dtname,opname,npdt', [('MPI_DOUBLE', 'MPI_SUM', np.float64),
                                               ('MPI_FLOAT', 'MPI_PROD', np.float32),
                                               ('MPI_INT', 'MPI_BXOR', np.int32)])
def test_chunked_pipeline_ragged(R, H, oracle, dtname, opname, npdt):
    """the per-chunk pattern of a pipelined collective: three incoming
    vectors, each combined into the result as ragged chunks (odd offsets,
    one-element and empty-free pieces) by back-to-back async calls on one
    stream; bit-equal to the oracle applying the three inputs in order"""
    rng = np.random.default_rng(0x5EED0C)
    n = 1_000_003
    dt, op = getattr(H, dtname), getattr(H, opname)
    if npdt is np.int32:
        ins = [rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32) for _ in range(3)]
        acc = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    else:
        ins = [rng.uniform(0.5, 1.5, n).astype(npdt) for _ in range(3)]
        acc = rng.uniform(-1, 1, n).astype(npdt)
    cuts = np.unique(np.concatenate([[0, 1, 2, n - 1, n], rng.integers(3, n - 1, 37)]))
    d_acc = torch.from_numpy(acc.copy()).cuda()
    d_ins = [torch.from_numpy(x).cuda() for x in ins]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for x in d_ins:
            for lo, hi in zip(cuts[:-1], cuts[1:]):
                assert R.reduce_local_async(x[lo:hi], d_acc[lo:hi], int(hi - lo), dt, op, s) == 0
    s.synchronize()
    exp = acc.copy()
    for x in ins:
        oracle.reduce_local(x, exp, n, dt, op)
    got = d_acc.cpu().numpy()
    assert np.array_equal(got.view(np.uint8), exp.view(np.uint8))


@pytest.mark.parametrize('threads,chunk', [(1, 65536), (4, 65536), (8, 256 << 10), (16, 128 << 10)])
@pytest.mark.parametrize('place', ['both_host', 'host_in', 'host_inout', 'pinned_in'])
def test_pageable_worker_pipeline(R, H, oracle, threads, chunk, place):
    """large pageable operands through the host workers' pinned slots
    (MPIX_Redop_set_pageable): ragged last chunk, mixed placements, fp32 SUM
    and MPI_2INT MAXLOC with ties; bit-equal to the oracle and to the
    hipMemcpyAsync staging path"""
    prev = R.get_pageable()
    rng = np.random.default_rng(0x5EED0F + threads)
    n = (1 << 21) + 77
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    m = (1 << 20) + 3
    p = rng.integers(0, 4, (m, 2)).astype(np.int32)
    q = rng.integers(0, 4, (m, 2)).astype(np.int32)
    exp_f = a.copy()
    oracle.reduce_local(b, exp_f, n, H.MPI_FLOAT, H.MPI_SUM)
    exp_p = p.copy()
    oracle.reduce_local(q, exp_p, m, H.MPI_2INT, H.MPI_MAXLOC)

    def place_ops(x_in, x_io):
        if place == 'host_in':
            return x_in, torch.from_numpy(x_io.copy()).cuda()
        if place == 'host_inout':
            return torch.from_numpy(x_in).cuda(), x_io
        if place == 'pinned_in':
            return torch.from_numpy(x_in.copy()).pin_memory(), x_io
        return x_in, x_io

    try:
        for mode in (threads, 0):
            assert R.set_pageable(mode, chunk) == 0
            for x_in, x_io, cnt, dt, op, exp in ((b, a, n, H.MPI_FLOAT, H.MPI_SUM, exp_f),
                                                 (q, p, m, H.MPI_2INT, H.MPI_MAXLOC, exp_p)):
                i_op, io_op = place_ops(x_in, x_io.copy())
                torch.cuda.synchronize()
                assert R.MPI_Reduce_local(i_op, io_op, cnt, dt, op) == 0
                got = io_op.cpu().numpy() if isinstance(io_op, torch.Tensor) else io_op
                assert np.array_equal(got, exp), (mode, dt)
    finally:
        R.set_pageable(prev['threads'], prev['chunk_bytes'])


_PAGEABLE_MODE = r'''
import sys, numpy as np, torch
sys.path.insert(0, %r)
from mpich_amd import redop as R, handles as H
from oracle import oracle as orc
orc.build()
rng = np.random.default_rng(7)
n = (1 << 22) + 13
a = rng.uniform(-1, 1, n).astype(np.float32); b = rng.uniform(-1, 1, n).astype(np.float32)
e = a.copy(); orc.reduce_local(b, e, n, H.MPI_FLOAT, H.MPI_SUM)
assert R.set_pageable(5, 256 << 10) == 0          # 64+ chunks, ragged last one
for rep in range(2):
    x = a.copy()
    assert R.MPI_Reduce_local(b, x, n, H.MPI_FLOAT, H.MPI_SUM) == 0
    assert np.array_equal(x, e), rep
print('mode ok')
'''


@pytest.mark.parametrize('db,aff,mode', [('0', 'none', 'worker'), ('1', 'gpu', 'worker'),
                                         ('1', '0-3,5', 'worker'), ('0', 'gpu', 'worker'),
                                         ('1', 'none', 'wave'), ('1', 'gpu', 'wave')])
def test_pageable_worker_modes(db, aff, mode):
    """the workers' modes from the environment: one buffer (copy and kernel in
    turn) or two (the next chunk copied during the kernel), pinned to the
    GPU's NUMA node or an explicit cpulist, and the wave form (all workers on
    one chunk, one kernel per chunk, three buffers in rotation); same bits as
    the oracle"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, '-c', _PAGEABLE_MODE % root], capture_output=True,
                       text=True, timeout=300,
                       env=dict(os.environ, MPIX_REDOP_PAGEABLE_DB=db,
                                MPIX_REDOP_PAGEABLE_AFFINITY=aff, MPIX_REDOP_PAGEABLE_MODE=mode))
    assert p.returncode == 0 and 'mode ok' in p.stdout, p.stdout + p.stderr


def test_pageable_knob_errors(R):
    prev = R.get_pageable()
    assert R.set_pageable(-1, 1 << 20) == 12
    assert R.set_pageable(17, 1 << 20) == 12
    assert R.set_pageable(4, 1024) == 12
    assert R.get_pageable() == prev


def test_pageable_slots_after_shrink(R, H, oracle):
    """regression: slots re-allocated for fewer workers at a larger chunk,
    then more workers at a smaller chunk again (every worker needs a slot)"""
    prev = R.get_pageable()
    rng = np.random.default_rng(0x5EED10)
    n = (1 << 21) + 5
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    exp = a.copy()
    oracle.reduce_local(b, exp, n, H.MPI_FLOAT, H.MPI_SUM)
    try:
        for threads, chunk in ((16, 128 << 10), (4, 512 << 10), (16, 128 << 10), (2, 64 << 10)):
            assert R.set_pageable(threads, chunk) == 0
            got = a.copy()
            assert R.MPI_Reduce_local(b, got, n, H.MPI_FLOAT, H.MPI_SUM) == 0
            assert np.array_equal(got, exp), (threads, chunk)
    finally:
        R.set_pageable(prev['threads'], prev['chunk_bytes'])


def test_pageable_workers_concurrent_callers(R, H, oracle):
    """two application threads in the pageable worker path at once (each
    caller has its own slots and streams); both results bit-equal"""
    import threading
    prev = R.get_pageable()
    rng = np.random.default_rng(0x5EED11)
    n = (1 << 21) + 9
    ops = []
    for _ in range(2):
        a = rng.uniform(-1, 1, n).astype(np.float64)
        b = rng.uniform(-1, 1, n).astype(np.float64)
        e = a.copy()
        oracle.reduce_local(b, e, n, H.MPI_DOUBLE, H.MPI_SUM)
        ops.append((b, a, e))
    rcs = [None, None]

    def run(i):
        b, a, _ = ops[i]
        rcs[i] = [R.MPI_Reduce_local(b, a, n, H.MPI_DOUBLE, H.MPI_SUM) for _ in range(1)]

    try:
        assert R.set_pageable(4, 256 << 10) == 0
        ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        assert rcs == [[0], [0]]
        for b, a, e in ops:
            assert np.array_equal(a, e)
    finally:
        R.set_pageable(prev['threads'], prev['chunk_bytes'])


def test_bf16_sum_specials_on_gpu(R, H, oracle):
    """bf16 SUM's half-away store (op_fns.c:473-483) on the HIP path: every
    pair of the special / tie patterns of tests/test_bf16_oracle.py, bit-exact
    against the oracle except that a NaN only has to be a NaN"""
    from tests.test_bf16_oracle import BF16_PATTERNS as pats
    a = np.repeat(pats, len(pats))
    b = np.tile(pats, len(pats))
    da, db = dev(a), dev(b)
    assert R.MPI_Reduce_local(db, da, len(a), H.MPIX_BFLOAT16, H.MPI_SUM) == 0
    exp = a.copy()
    assert oracle.reduce_local(b.copy(), exp, len(a), H.MPIX_BFLOAT16, H.MPI_SUM) == 0
    got = host(da).view(np.uint16)
    assert compare(got.view(np.uint8), exp.view(np.uint8), 'bf16', 2, 'MPI_SUM', 2) == 0


@pytest.mark.parametrize('dtname,npt', [('MPIX_C_FLOAT16', np.float16), ('MPI_FLOAT', np.float32),
                                        ('MPI_DOUBLE', np.float64)])
@pytest.mark.parametrize('opname', ['MPI_MAX', 'MPI_MIN'])
def test_maxmin_select_specials_on_gpu(R, H, oracle, dtname, npt, opname):
    """MPL_MAX/MPL_MIN are selects, (a>b)?a:b and (a<b)?a:b (mpl_base.h:105-106):
    with a NaN on either side the result is the in operand bit for bit
    (payload and sign kept), and on equal values (+0 vs -0) it is the in
    operand too.  Every pair of the special values, against the oracle and
    against numpy's select, bit-exact"""
    fi = np.finfo(npt)
    nanbits = {np.float16: [0x7e00, 0xfe01, 0x7c01, 0x7fff],
               np.float32: [0x7fc00000, 0xffc00001, 0x7f800001, 0x7fffffff],
               np.float64: [0x7ff8000000000000, 0xfff8000000000001, 0x7ff0000000000001,
                            0x7fffffffffffffff]}[npt]
    uint = {np.float16: np.uint16, np.float32: np.uint32, np.float64: np.uint64}[npt]
    vals = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, fi.max, -fi.max, fi.tiny, -fi.tiny,
                     fi.smallest_subnormal, -fi.smallest_subnormal, 0.5, 2.0], npt)
    vals = np.concatenate([vals, np.array(nanbits, uint).view(npt)])
    a = np.repeat(vals, len(vals))
    b = np.tile(vals, len(vals))
    da, db = dev(a), dev(b)
    op = getattr(H, opname)
    assert R.MPI_Reduce_local(db, da, len(a), getattr(H, dtname), op) == 0
    got = host(da).view(uint)
    exp = a.copy()
    assert oracle.reduce_local(b.copy(), exp, len(a), getattr(H, dtname), op) == 0
    sel = np.where(a > b, a, b) if opname == 'MPI_MAX' else np.where(a < b, a, b)
    assert np.array_equal(exp.view(uint), sel.view(uint))
    assert np.array_equal(got, exp.view(uint))


@pytest.mark.parametrize('dtname,npt', [('MPI_C_FLOAT_COMPLEX', np.float32),
                                        ('MPI_C_DOUBLE_COMPLEX', np.float64),
                                        ('MPI_COMPLEX', np.float32),
                                        ('MPI_DOUBLE_COMPLEX', np.float64),
                                        ('MPI_COMPLEX4', np.float16)])
@pytest.mark.parametrize('opname', ['MPI_PROD', 'MPI_SUM'])
def test_complex_specials_on_gpu(R, H, oracle, dtname, npt, opname):
    """complex SUM / PROD on every pair of 21 special values (zeros of both
    signs, infinities and NaNs in either component, overflow and subnormal
    magnitudes): C `_Complex` products with the Annex G recovery of a
    both-NaN result, struct complex without it (op_fns.c:61-91), SUM per
    component; against the oracle under the sweep's rule (a NaN component
    only has to be a NaN)"""
    inf, nan = np.inf, np.nan
    big = np.finfo(npt).max / 2
    sub = np.finfo(npt).smallest_subnormal
    z = [(0, 0), (-0.0, 0), (0, -0.0), (1, 0), (0, 1), (-1, -1), (inf, 0), (0, inf),
         (-inf, 1), (1, -inf), (inf, inf), (nan, 0), (0, nan), (nan, nan), (inf, nan),
         (nan, -inf), (big, big), (big, -big), (sub, sub), (3, -2), (0.5, 0.25)]
    vals = np.array(z, npt).reshape(-1)
    n = len(z)
    a = np.repeat(vals.reshape(n, 2), n, axis=0).reshape(-1)
    b = np.tile(vals.reshape(n, 2), (n, 1)).reshape(-1)
    dt, op = getattr(H, dtname), getattr(H, opname)
    da, db = dev(a), dev(b)
    with np.errstate(all='ignore'):
        assert R.MPI_Reduce_local(db, da, n * n, dt, op) == 0
        exp = a.copy()
        assert oracle.reduce_local(b.copy(), exp, n * n, dt, op) == 0
    size = np.dtype(npt).itemsize
    got = host(da)
    assert compare(got, exp.view(np.uint8), 'cplx', size, opname, 2 * size) == 0


@pytest.mark.parametrize('dtname', ['MPI_FLOAT_INT', 'MPI_2REAL', 'MPI_DOUBLE_INT',
                                    'MPI_2DOUBLE_PRECISION', 'MPIR_2FLOAT16'])
@pytest.mark.parametrize('opname', ['MPI_MAXLOC', 'MPI_MINLOC'])
def test_loc_specials_on_gpu(R, H, oracle, dtname, opname):
    """MAXLOC / MINLOC (op_fns.c:299-352) on every pair of special values:
    a strict winner takes (value, loc), equal values (+0 and -0 included)
    keep the smaller loc, a NaN on either side leaves inout unchanged;
    padding bytes are inout's.  Bit-exact against the oracle"""
    entry = next(s for s in SWEEP if s[0] == dtname and s[1] == opname)
    vdt, ldt, ext, loff = entry[2][1:]
    vals = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 2.0, 1.0, -np.nan],
                    np.dtype(vdt))
    nv = len(vals)
    rng = np.random.default_rng(0x5EED0011)

    def pack(v, locs):
        buf = rng.integers(0, 256, len(v) * ext, dtype=np.uint8).reshape(len(v), ext)
        buf[:, :np.dtype(vdt).itemsize] = v.view(np.uint8).reshape(len(v), -1)
        buf[:, loff:loff + np.dtype(ldt).itemsize] = \
            locs.astype(ldt).view(np.uint8).reshape(len(v), -1)
        return buf.reshape(-1)

    la = rng.integers(0, 4, nv * nv)
    lb = rng.integers(0, 4, nv * nv)
    a = pack(np.repeat(vals, nv), la)
    b = pack(np.tile(vals, nv), lb)
    dt, op = getattr(H, dtname), getattr(H, opname)
    da, db = dev(a), dev(b)
    assert R.MPI_Reduce_local(db, da, nv * nv, dt, op) == 0
    exp = a.copy()
    assert oracle.reduce_local(b.copy(), exp, nv * nv, dt, op) == 0
    assert np.array_equal(host(da), exp)


@pytest.mark.parametrize('tn', ['MPI_INT8_T', 'MPI_UINT8_T', 'MPI_BYTE', 'MPI_C_BOOL', 'MPI_CHAR'])
def test_one_byte_ops_every_pair_on_gpu(R, H, oracle, tn):
    """round 3's four-bytes-per-dword logicals (and the 1-byte kernels of
    every other op the type has) on every pair of byte values, in every byte
    lane of a dword and every 16-byte packet position of a tile, against the
    oracle: 65536 pairs x 16 rotations"""
    dt = getattr(H, tn)
    a8, b8 = np.meshgrid(np.arange(256, dtype=np.uint8), np.arange(256, dtype=np.uint8))
    a8, b8 = a8.ravel(), b8.ravel()
    # rotate the pair sequence so every pair lands in every byte of a packet
    A = np.concatenate([np.roll(a8, r) for r in range(16)])
    B = np.concatenate([np.roll(b8, r) for r in range(16)])
    n = A.size
    ran = 0
    for on, op in H.OPS.items():
        if op in (H.MPI_REPLACE, H.MPI_NO_OP, H.MPIX_EQUAL) or not R.is_supported(op, dt):
            continue
        da, db = dev(A), dev(B)
        assert R.MPI_Reduce_local(db, da, n, dt, op) == 0
        exp = A.copy()
        oracle.reduce_local(B, exp, n, dt, op)
        assert np.array_equal(host(da), exp), (tn, on)
        ran += 1
    assert ran >= 3, tn


def test_complex_prod_sparse_specials_in_tiles(R, H, oracle):
    """the Annex G product's recovery runs once per tile when any lane's
    element needs it: ordinary products with sparse (inf, nan) / (nan, nan)
    pairs scattered through many tiles, every lane position, C float and
    double complex and the fp16 struct complex -- bit-exact where the
    result is a number, NaN where it is a NaN"""
    rng = np.random.default_rng(0x5EED0A6)
    inf, nan = np.inf, np.nan
    specials = [(inf, nan), (nan, inf), (nan, nan), (inf, 0.0), (0.0, inf), (-inf, 1.0),
                (1.0, -inf), (nan, 0.0)]
    for tn, ft in (('MPI_C_FLOAT_COMPLEX', np.float32), ('MPI_C_DOUBLE_COMPLEX', np.float64),
                   ('MPI_COMPLEX4', np.float16)):
        dt = getattr(H, tn)
        n = (1 << 18) + 37
        a = rng.uniform(-2, 2, (n, 2)).astype(ft)
        b = rng.uniform(-2, 2, (n, 2)).astype(ft)
        for arr in (a, b):
            idx = rng.choice(n, n // 500, replace=False)
            for i in idx:
                arr[i] = specials[rng.integers(len(specials))]
        da, db = dev(a), dev(b)
        assert R.MPI_Reduce_local(db, da, n, dt, H.MPI_PROD) == 0
        exp = a.copy()
        oracle.reduce_local(b, exp, n, dt, H.MPI_PROD)
        got = host(da).view(ft).reshape(n, 2)
        both_nan = np.isnan(got) & np.isnan(exp)
        same = (got.view(np.uint8).reshape(n, 2, -1) == exp.view(np.uint8).reshape(n, 2, -1)).all(-1)
        assert np.all(same | both_nan), tn
