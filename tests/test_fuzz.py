"""Property-based parity (hypothesis, derandomised so every run draws the
same examples).

CPU: the oracle against an independent numpy restatement of the op rules
(mpir_op_util.h:46-53 with MPL_MAX/MPL_MIN of mpl_base.h:105-106: integers
wrap, MAX/MIN select `(a>b)?a:b` / `(a<b)?a:b` so any NaN yields the in
operand, logical ops give 0/1, FP SUM/PROD one IEEE op) over random sizes,
values and specials -- a second pin for the oracle beyond the golden vectors.

GPU: the HIP path against the oracle over random (op, type) cases of the
parity sweep, counts, byte offsets of both operands (packet, unaligned-load
and element-wise kernels) and entry points (synchronous, stream-ordered,
pinned and pageable host operands).
"""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from mpich_amd import handles as H

INT_TYPES = {'MPI_INT8_T': np.int8, 'MPI_INT16_T': np.int16, 'MPI_INT32_T': np.int32,
             'MPI_INT64_T': np.int64, 'MPI_UINT8_T': np.uint8, 'MPI_UINT16_T': np.uint16,
             'MPI_UINT32_T': np.uint32, 'MPI_UINT64_T': np.uint64}
FP_TYPES = {'MPI_FLOAT': np.float32, 'MPI_DOUBLE': np.float64}


def numpy_rule(opname, a, b):
    """inout = OP(inout=a, in=b), restated with numpy"""
    with np.errstate(over='ignore', invalid='ignore'):
        if opname == 'MPI_SUM':
            return a + b
        if opname == 'MPI_PROD':
            return a * b
        if opname == 'MPI_MAX':
            return np.where(a > b, a, b)
        if opname == 'MPI_MIN':
            return np.where(a < b, a, b)
        if opname == 'MPI_BAND':
            return a & b
        if opname == 'MPI_BOR':
            return a | b
        if opname == 'MPI_BXOR':
            return a ^ b
        if opname == 'MPI_LAND':
            return ((a != 0) & (b != 0)).astype(a.dtype)
        if opname == 'MPI_LOR':
            return ((a != 0) | (b != 0)).astype(a.dtype)
        if opname == 'MPI_LXOR':
            return ((a != 0) != (b != 0)).astype(a.dtype)
    raise ValueError(opname)


INT_OPS = ['MPI_SUM', 'MPI_PROD', 'MPI_MAX', 'MPI_MIN', 'MPI_BAND', 'MPI_BOR', 'MPI_BXOR',
           'MPI_LAND', 'MPI_LOR', 'MPI_LXOR']
FP_OPS = ['MPI_SUM', 'MPI_PROD', 'MPI_MAX', 'MPI_MIN']
CPU_CASES = [(t, o) for t in INT_TYPES for o in INT_OPS] + [(t, o) for t in FP_TYPES for o in FP_OPS]


def fp_values(rng, n, npt):
    x = rng.uniform(-3, 3, n).astype(npt)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, np.finfo(npt).tiny / 4,
                   np.finfo(npt).max], npt)
    k = rng.random(n) < 0.05
    x[k] = sp[rng.integers(0, len(sp), int(k.sum()))]
    return x


@settings(max_examples=200, derandomize=True, deadline=None,
          suppress_health_check=[HealthCheck.too_slow])
@given(case=st.sampled_from(CPU_CASES), n=st.integers(0, 3000), seed=st.integers(0, 2 ** 32 - 1))
def test_oracle_matches_numpy_rules(oracle, case, n, seed):
    tname, opname = case
    rng = np.random.default_rng(seed)
    if tname in INT_TYPES:
        npt = INT_TYPES[tname]
        info = np.iinfo(npt)
        a = rng.integers(info.min, info.max, n, dtype=npt, endpoint=True)
        b = rng.integers(info.min, info.max, n, dtype=npt, endpoint=True)
        if opname.startswith('MPI_L'):                  # plenty of zeros
            a[rng.random(n) < 0.4] = 0
            b[rng.random(n) < 0.4] = 0
    else:
        npt = FP_TYPES[tname]
        a, b = fp_values(rng, n, npt), fp_values(rng, n, npt)
    exp = numpy_rule(opname, a, b)
    got = a.copy()
    assert oracle.reduce_local(b, got, n, getattr(H, tname), getattr(H, opname)) == 0
    if tname in FP_TYPES and opname in ('MPI_SUM', 'MPI_PROD'):
        gn, en = np.isnan(got), np.isnan(exp)      # arithmetic NaN payloads are unpinned
        assert np.array_equal(gn, en)
        assert got[~gn].tobytes() == exp[~en].tobytes()
    else:
        assert got.tobytes() == exp.tobytes()


# ------------------------------------------------------------------- GPU
@pytest.fixture(scope='module')
def R():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


def _sweep():
    from tests.test_gpu_parity import SWEEP
    return SWEEP


@pytest.mark.gpu
@settings(max_examples=int(os.environ.get('MPIX_FUZZ_EXAMPLES', 300)),
          derandomize=not os.environ.get('MPIX_FUZZ_RANDOM'), deadline=None,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(k=st.integers(0, 10 ** 6), n=st.one_of(st.integers(0, 2000), st.integers(2000, 70000)),
       off_io=st.integers(0, 3), off_in=st.integers(0, 3), sub=st.sampled_from([0, 0, 0, 1]),
       entry=st.sampled_from(['sync', 'async', 'pinned', 'pageable']),
       seed=st.integers(0, 2 ** 32 - 1))
def test_gpu_matches_oracle_random(R, oracle, k, n, off_io, off_in, sub, entry, seed):
    """offsets in elements (0..3) plus, with `sub`, one extra byte on `in`
    (relatively misaligned operands: the element-wise kernel)"""
    import torch
    from tests.test_gpu_parity import compare, make_operand
    sweep = _sweep()
    dtname, opname, kind, size = sweep[k % len(sweep)]
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = R.datatype_extent(dt)
    rng = np.random.default_rng(seed)
    a = make_operand(rng, kind, size, n + 8, dtname)
    b = make_operand(rng, kind, size, n + 8, dtname)
    oa, ob = off_io * ext, off_in * ext + sub
    exp = a.copy()
    bb = b[ob:ob + n * ext].copy()
    assert oracle.reduce_local(bb, exp[oa:], n, dt, op) == 0
    if entry in ('sync', 'async'):
        da = torch.from_numpy(a.copy()).cuda()
        db = torch.from_numpy(np.concatenate([b, np.zeros(8, np.uint8)])).cuda()
        torch.cuda.synchronize()
        if entry == 'sync':
            rc = R.MPI_Reduce_local(db.data_ptr() + ob, da.data_ptr() + oa, n, dt, op)
        else:
            rc = R.reduce_local_async(db.data_ptr() + ob, da.data_ptr() + oa, n, dt, op)
        torch.cuda.synchronize()
        got = da.cpu().numpy()
    elif entry == 'pinned':
        pa = torch.from_numpy(a.copy()).pin_memory()
        pb = torch.from_numpy(b.copy()).pin_memory()
        rc = R.MPI_Reduce_local(pb.data_ptr() + ob, pa.data_ptr() + oa, n, dt, op)
        got = pa.numpy()
    else:
        got = a.copy()
        bh = b.copy()
        rc = R.MPI_Reduce_local(bh.ctypes.data + ob, got.ctypes.data + oa, n, dt, op)
    assert rc == 0
    assert got[:oa].tobytes() == a[:oa].tobytes()                  # bytes before: untouched
    assert got[oa + n * ext:].tobytes() == a[oa + n * ext:].tobytes()   # bytes after: untouched
    assert compare(got[oa:oa + n * ext], exp[oa:oa + n * ext], kind, size, opname, ext) == 0
