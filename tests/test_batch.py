"""MPIX_Reduce_local_batch_async: k ready chunks in one launch, the same bits
as k MPIX_Reduce_local_async calls (each segment split into head / packets /
tail exactly as its own call would split it).  The engines it serves call
MPIR_Reduce_local once per ready vertex (gentran_utils.c:157-167,
mpidu_sched.c:309-316); the oracle checks every segment.

CPU: the argument checks, all made before any device work.  GPU: random
batches over every kind of combiner (packet kernel at equal and unequal
16-byte phases, the element-wise fallback for operands that are not even
element-aligned, the 32-byte units' own batch kernel, REPLACE), zero counts, k = 1 and
k = MPIX_BATCH_MAX, a large segment spanning many blocks, and the bits of
the same triples issued as separate calls."""
import ctypes

import numpy as np
import pytest

MPI_FLOAT, MPI_SUM, MPI_MAXLOC, MPI_2INT = 0x4c00040a, 0x58000003, 0x5800000c, 0x4c000816


def _call(R, ins, ios, counts, dt=MPI_FLOAT, op=MPI_SUM, k=None):
    k = len(counts) if k is None else k
    n = max(len(counts), 1)
    a = (ctypes.c_void_p * n)(*ins)
    b = (ctypes.c_void_p * n)(*ios)
    c = (ctypes.c_ssize_t * n)(*counts)
    return R.lib().MPIX_Reduce_local_batch_async(a, b, c, k, dt, op, None)


def test_batch_argument_errors():
    from mpich_amd import handles as H
    from mpich_amd import redop as R
    assert _call(R, [], [], [], k=0) == H.MPI_ERR_ARG
    assert _call(R, [4096] * 65, [1 << 30] * 65, [1] * 65) == H.MPI_ERR_ARG
    assert R.lib().MPIX_Reduce_local_batch_async(None, None, None, 1, MPI_FLOAT, MPI_SUM,
                                                 None) == H.MPI_ERR_ARG
    assert _call(R, [4096], [8192], [-1]) == H.MPI_ERR_COUNT
    assert _call(R, [4096], [8192], [10], op=0x58000006) == H.MPI_ERR_OP    # BAND on float
    assert _call(R, [4096], [4100], [10]) == H.MPI_ERR_BUFFER              # in overlaps inout
    # target i overlaps target j, or source j
    assert _call(R, [1 << 20, 2 << 20], [4096, 4096 + 36], [10, 10]) == H.MPI_ERR_BUFFER
    assert _call(R, [1 << 20, 4096 + 36], [4096, 3 << 20], [10, 10]) == H.MPI_ERR_BUFFER
    # zero counts never overlap; all-zero batches succeed without a launch
    assert _call(R, [1 << 20, 2 << 20], [4096, 4096], [0, 0]) == H.MPI_SUCCESS


# ------------------------------------------------------------------ GPU
torch = pytest.importorskip('torch')


@pytest.fixture(scope='module')
def R():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


def _layout(rng, k, ext, max_count, odd=False):
    """k disjoint (in_off, io_off, count) byte regions of one pool: counts
    random (some 0, some 1), offsets element-aligned with random 16-byte
    phases (or, with odd, some off the element grid)"""
    trip, at = [], 0
    for _ in range(k):
        c = int(rng.choice([0, 1, 3, int(rng.integers(1, max_count + 1))]))
        sh_in = int(rng.integers(0, 16)) * (1 if odd and rng.random() < 0.3 else ext) % 64
        sh_io = int(rng.integers(0, 16)) * ext % 64
        in_off = at + 64 + sh_in
        io_off = in_off + c * ext + 64 + sh_io
        at = io_off + c * ext + 64
        trip.append((in_off, io_off, c))
    return trip, at + 64


@pytest.mark.gpu
@pytest.mark.parametrize('dtname,opname,odd', [
    ('MPI_FLOAT', 'MPI_SUM', False), ('MPI_FLOAT', 'MPI_SUM', True), ('MPI_INT8_T', 'MPI_LXOR', False),
    ('MPI_DOUBLE', 'MPI_MAX', False), ('MPI_2INT', 'MPI_MAXLOC', True),
    ('MPI_COMPLEX4', 'MPI_PROD', False), ('MPI_C_DOUBLE_COMPLEX', 'MPI_PROD', False),
    ('MPI_LONG_DOUBLE_INT', 'MPI_MINLOC', False), ('MPI_LONG_DOUBLE_INT', 'MPI_MINLOC', True),
    ('MPI_C_LONG_DOUBLE_COMPLEX', 'MPI_SUM', False), ('MPI_INT64_T', 'MPI_REPLACE', False),
    ('MPIX_C_FLOAT16', 'MPI_SUM', True)])
@pytest.mark.parametrize('k', [1, 7, 64])
def test_batch_matches_oracle_and_single_calls(R, oracle, dtname, opname, odd, k):
    from mpich_amd import handles as H
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = R.datatype_extent(dt)
    rng = np.random.default_rng((0x5EED0700 + 97 * k + dt + op) & 0xffffffff)
    trip, nbytes = _layout(rng, k, ext, 40000 if k < 64 else 3000, odd)
    pool = rng.integers(0, 256, nbytes, dtype=np.uint8)
    if dtname in ('MPI_FLOAT', 'MPI_DOUBLE', 'MPI_COMPLEX4', 'MPI_C_DOUBLE_COMPLEX',
                  'MPIX_C_FLOAT16'):
        # finite values: arithmetic NaN payloads are outside this test
        fl = {'MPI_FLOAT': np.float32, 'MPI_DOUBLE': np.float64, 'MPI_COMPLEX4': np.float16,
              'MPI_C_DOUBLE_COMPLEX': np.float64, 'MPIX_C_FLOAT16': np.float16}[dtname]
        v = rng.uniform(-2, 2, nbytes // np.dtype(fl).itemsize).astype(fl)
        pool[:v.nbytes] = v.view(np.uint8)
    want = pool.copy()
    for i_off, o_off, c in trip:
        if c:
            src = want[i_off:i_off + c * ext].copy()
            dst = want[o_off:o_off + c * ext]
            assert oracle.reduce_local(src, dst, c, dt, op) == 0
    s = torch.cuda.Stream()
    d = torch.from_numpy(pool.copy()).cuda()
    torch.cuda.synchronize()
    base = d.data_ptr()
    rc = R.reduce_local_batch_async([base + t[0] for t in trip], [base + t[1] for t in trip],
                                    [t[2] for t in trip], dt, op, s)
    assert rc == 0
    s.synchronize()
    got = d.cpu().numpy()

    def same(x, y):
        # fp16 results compare NaN-equivalent: the odd offsets cut random bit
        # patterns, and fp16 NaN payloads differ between gfx950 and the x86
        # loop when both operands are NaN
        if dtname != 'MPIX_C_FLOAT16' or np.array_equal(x, y):
            return np.array_equal(x, y)
        fx, fy = x.view(np.float16), y.view(np.float16)
        return bool(np.all((x.view(np.uint16) == y.view(np.uint16)) | (np.isnan(fx) & np.isnan(fy))))
    for q, (i_off, o_off, c) in enumerate(trip):
        assert same(got[o_off:o_off + c * ext], want[o_off:o_off + c * ext]), (q, c)
    outside = np.ones(len(got), bool)
    for _, o_off, c in trip:
        outside[o_off:o_off + c * ext] = False
    assert np.array_equal(got[outside], want[outside])      # nothing outside the targets moved
    # the same triples as separate stream-ordered calls: identical bits
    d2 = torch.from_numpy(pool.copy()).cuda()
    torch.cuda.synchronize()
    b2 = d2.data_ptr()
    for i_off, o_off, c in trip:
        assert R.reduce_local_async(b2 + i_off, b2 + o_off, c, dt, op, s) == 0
    s.synchronize()
    assert np.array_equal(d2.cpu().numpy(), got)            # bit for bit, NaNs included


@pytest.mark.gpu
def test_batch_large_segment(R, oracle):
    """one 64 MiB segment between small ones: many blocks, the block ->
    segment lookup at its edges"""
    from mpich_amd import handles as H
    n_big = (64 << 20) // 4 + 5
    rng = np.random.default_rng(0x5EED0701)
    sizes = [3, n_big, 1, 1000, 17]
    ins = [torch.from_numpy(rng.uniform(-1, 1, c).astype(np.float32)).cuda() for c in sizes]
    ios = [torch.from_numpy(rng.uniform(-1, 1, c).astype(np.float32)).cuda() for c in sizes]
    want = []
    for a, b in zip(ins, ios):
        w = b.cpu().numpy().copy()
        assert oracle.reduce_local(a.cpu().numpy(), w, len(w), H.MPI_FLOAT, H.MPI_SUM) == 0
        want.append(w)
    torch.cuda.synchronize()
    R.check(R.reduce_local_batch_async(ins, ios, sizes, H.MPI_FLOAT, H.MPI_SUM))
    torch.cuda.synchronize()
    for b, w in zip(ios, want):
        assert np.array_equal(b.cpu().numpy(), w)


@pytest.mark.gpu
def test_batch_refuses_host_operand(R):
    from mpich_amd import handles as H
    x = torch.ones(1024, device='cuda')
    h = np.ones(1024, np.float32)
    y = torch.ones(1024, device='cuda')
    rc = R.reduce_local_batch_async([x, h], [y, torch.ones(1024, device='cuda')], [1024, 1024],
                                    H.MPI_FLOAT, H.MPI_SUM)
    assert rc == H.MPI_ERR_BUFFER
    torch.cuda.synchronize()
    assert bool(torch.all(y == 1))          # refused before any launch


@pytest.mark.gpu
def test_batch_with_page_locked_operands(R, oracle):
    """a triple with a page-locked host operand (in, inout or
    both) runs as its own zero-copy call, with the capped looping grid every
    kernel reading host memory gets; the device triples of the same batch
    still go as one launch.  Every triple = the oracle."""
    from mpich_amd import handles as H
    rng = np.random.default_rng(0x5EED0702)
    sizes = [4099, (4 << 20) // 4 + 3, 1000, (1 << 20) + 1, 17]
    kinds = [('dev', 'dev'), ('pin', 'dev'), ('dev', 'dev'), ('pin', 'pin'), ('dev', 'pin')]

    def buf(kind, v):
        t = torch.from_numpy(v.copy())
        return t.pin_memory() if kind == 'pin' else t.cuda()
    ins, ios, want = [], [], []
    for c, (ki, ko) in zip(sizes, kinds):
        a = rng.uniform(-1, 1, c).astype(np.float32)
        b = rng.uniform(-1, 1, c).astype(np.float32)
        w = b.copy()
        assert oracle.reduce_local(a, w, c, H.MPI_FLOAT, H.MPI_SUM) == 0
        ins.append(buf(ki, a))
        ios.append(buf(ko, b))
        want.append(w)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    R.check(R.reduce_local_batch_async(ins, ios, sizes, H.MPI_FLOAT, H.MPI_SUM, s))
    s.synchronize()
    for q, (b, w) in enumerate(zip(ios, want)):
        assert np.array_equal(b.cpu().numpy(), w), q
