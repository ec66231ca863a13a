"""Derived targets given as their raw iov (typerep_op_fallback,
src/mpi/datatype/typerep/src/typerep_op.c:69-155), incl. the pairtype
gather of :117-145, and MPI_REPLACE as a typemap copy on padded pairs
(op_fns.c:445-457 -> MPIR_Localcopy).

CPU tests pin the oracle's restatement against expectations computed here
independently with numpy (MAXLOC/MINLOC rule of op_fns.c:314-319; the iov a
derived type of pairs flattens to, by the pair type maps of
pairtypes.c:24-62).  GPU tests compare the C-ABI (MPIX_Reduce_local_iovec_async,
MPIX_Reduce_local_iov_async, REPLACE on every entry point) with the oracle,
padding bytes included.  No reference test runs a pairtype accumulate on a
split iov except acc_pairtype.c (restated below through the iovec form);
the rest is "parity pinned by code reading".
"""
import numpy as np
import pytest

MAXLOC, MINLOC, REPLACE, SUM = 0x5800000c, 0x5800000b, 0x5800000d, 0x58000003
DOUBLE_INT, LONG_INT, SHORT_INT, FLOAT_INT = 0x8c000001, 0x8c000002, 0x8c000003, 0x8c000000
MPI_DOUBLE, MPI_INT = 0x4c00080b, 0x4c000405

# value dtype, value bytes, int offset, extent (pairtypes.c:15-24 on LP64)
PAIRS = {
    DOUBLE_INT: ('<f8', 8, 8, 16),
    LONG_INT: ('<i8', 8, 8, 16),
    SHORT_INT: ('<i2', 2, 4, 8),
    FLOAT_INT: ('<f4', 4, 4, 8),
}


def pair_dtype(dt):
    vt, vb, lo, ext = PAIRS[dt]
    return np.dtype({'names': ['v', 'loc'], 'formats': [vt, '<i4'], 'offsets': [0, lo],
                     'itemsize': ext})


def pair_iov(dt, positions, merge):
    """the iov of a target whose elements sit at `positions` (element
    indices, increasing): per element the type map's pieces {value, int}
    (pairtypes.c:60-62), adjacent pieces merged when `merge` (as a flattening
    that coalesces contiguous bytes does)."""
    _, vb, lo, ext = PAIRS[dt]
    segs = []
    for p in positions:
        for off, ln in ((p * ext, vb), (p * ext + lo, 4)):
            if merge and segs and segs[-1][0] + segs[-1][1] == off:
                segs[-1][1] += ln
            else:
                segs.append([off, ln])
    return [s[0] for s in segs], [s[1] for s in segs]


def bytecopy(a):
    """copy keeping padding bytes (a structured .copy() zeroes them)"""
    return a.view(np.uint8).copy().view(a.dtype)


def loc_expected(tgt, src, positions, op):
    """op_fns.c:314-319 per element, numpy restatement (no oracle)"""
    out = bytecopy(tgt)
    for k, p in enumerate(positions):
        a, b = out[p], src[k]
        av, bv = a['v'], b['v']
        take = (av < bv) if op == MAXLOC else (av > bv)
        if take:
            out['v'][p], out['loc'][p] = bv, b['loc']
        elif av == bv:
            out['loc'][p] = min(a['loc'], b['loc'])
    return out


def random_pairs(rng, dt, n):
    """values in {0..3} (ties), random locs, random padding bytes"""
    raw = rng.integers(0, 256, n * PAIRS[dt][3], dtype=np.uint8)
    a = raw.view(pair_dtype(dt))
    a['v'] = rng.integers(0, 4, n)
    a['loc'] = rng.integers(0, 6, n)
    return a


# ------------------------------------------------------------------- CPU
def test_acc_pairtype_through_iovec(oracle):
    """acc_pairtype.c:30-95 (vector(10, 3, 5) target of zeroed pairs, {1.0, 1}
    origin pairs, MAXLOC; MPI_DOUBLE_INT for the x87 pair) through the raw
    iov: one 12-byte segment per element."""
    dt = pair_dtype(DOUBLE_INT)
    tgt = np.zeros(50, dt)
    src = np.zeros(30, dt)
    src['v'], src['loc'] = 1.0, 1
    pos = [b * 5 + k for b in range(10) for k in range(3)]
    offs, lens = pair_iov(DOUBLE_INT, pos, merge=True)
    assert set(lens) == {12}
    t = tgt.view(np.uint8).copy()
    assert oracle.reduce_local_iovec(src.view(np.uint8).copy(), t, offs, lens, DOUBLE_INT,
                                     MAXLOC) == 0
    got = t.view(dt)
    sel = np.arange(50) % 5 < 3
    assert np.all(got['v'][sel] == 1.0) and np.all(got['loc'][sel] == 1)
    assert np.all(got['v'][~sel] == 0) and np.all(got['loc'][~sel] == 0)


@pytest.mark.parametrize('dt', [SHORT_INT, DOUBLE_INT, LONG_INT])
@pytest.mark.parametrize('merge', [False, True])
@pytest.mark.parametrize('op', [MAXLOC, MINLOC])
def test_pairtype_gather(oracle, dt, merge, op):
    """split {value, int} segments are gathered into one element each; with
    a contiguous run of SHORT_INT the merged iov is [2][6][6]..[4] and every
    element after the first is completed from a segment's leftover
    (typerep_op.c:141-145)"""
    rng = np.random.default_rng(dt & 0xff)
    n = 300
    pos = sorted(set(rng.integers(0, 2 * n, n).tolist()))
    pos[:40] = list(range(40))          # a contiguous stretch exercises the leftovers
    pos = sorted(set(pos))
    tgt = random_pairs(rng, dt, 2 * n)
    src = random_pairs(rng, dt, len(pos))
    offs, lens = pair_iov(dt, pos, merge)
    t = tgt.view(np.uint8).copy()
    assert oracle.reduce_local_iovec(src.view(np.uint8).copy(), t, offs, lens, dt, op) == 0
    exp = loc_expected(tgt, src, pos, op)
    assert t.tobytes() == exp.view(np.uint8).tobytes()     # padding untouched too


def test_iovec_basic_type_needs_whole_elements(oracle):
    rng = np.random.default_rng(7)
    src = rng.uniform(-1, 1, 6)
    dst = rng.uniform(-1, 1, 20)
    exp = dst.copy()
    assert oracle.reduce_local_iov(src, exp, [0, 64], [2, 4], MPI_DOUBLE, SUM) == 0
    got = dst.copy()
    assert oracle.reduce_local_iovec(src, got, [0, 64], [16, 32], MPI_DOUBLE, SUM) == 0
    assert np.array_equal(got, exp)
    assert oracle.reduce_local_iovec(src, dst.copy(), [0], [12], MPI_DOUBLE, SUM) == 12


@pytest.mark.parametrize('dt', [DOUBLE_INT, LONG_INT, SHORT_INT, FLOAT_INT])
def test_replace_is_a_typemap_copy(oracle, dt):
    """MPI_REPLACE = MPIR_Localcopy: value and int copied, padding of inout kept"""
    rng = np.random.default_rng(11)
    n = 257
    src, tgt = random_pairs(rng, dt, n), random_pairs(rng, dt, n)
    t = tgt.view(np.uint8).copy()
    assert oracle.reduce_local(src.view(np.uint8).copy(), t, n, dt, REPLACE) == 0
    exp = bytecopy(tgt)
    exp['v'], exp['loc'] = src['v'], src['loc']
    assert t.tobytes() == exp.view(np.uint8).tobytes()


def test_type_sizes(oracle):
    from mpich_amd import handles as H
    from mpich_amd import redop
    assert [oracle.size(d) for d in (FLOAT_INT, DOUBLE_INT, LONG_INT, SHORT_INT, 0x8c000004)] == \
        [8, 12, 12, 6, 20]
    for name in dir(H):
        if name.startswith('MPI_') and isinstance(getattr(H, name), int):
            h = getattr(H, name)
            if 0x4c000000 <= h < 0x4d000000 or (h & 0xffffff00) == 0x8c000000:
                assert redop.datatype_size(h) == oracle.size(h), name


# ------------------------------------------------------------------- GPU
def _dev(a):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()
    torch.cuda.synchronize()
    return t


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(scope='module')
def R():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


@pytest.mark.gpu
@pytest.mark.parametrize('dt', [SHORT_INT, DOUBLE_INT, LONG_INT, FLOAT_INT])
@pytest.mark.parametrize('merge', [False, True])
@pytest.mark.parametrize('op', [MAXLOC, MINLOC, REPLACE])
def test_iovec_pairs_on_gpu(R, oracle, dt, merge, op):
    rng = np.random.default_rng((dt & 0xff) * 3 + merge)
    n = 40000
    pos = np.unique(rng.integers(0, 2 * n, n))
    pos[:1000] = np.arange(1000)
    pos = np.unique(pos).tolist()
    tgt = random_pairs(rng, dt, 2 * n)
    src = random_pairs(rng, dt, len(pos))
    offs, lens = pair_iov(dt, pos, merge)
    dd, ds = _dev(tgt), _dev(src)
    exp = tgt.view(np.uint8).copy()
    rc = oracle.reduce_local_iovec(src.view(np.uint8).copy(), exp, offs, lens, dt, op)
    # FLOAT_INT has no padding (size == extent): not a pairtype, so a 4-byte
    # segment is not a whole element -- the reference's assert (:147)
    assert rc == (12 if dt == FLOAT_INT and not merge else 0)
    assert R.reduce_local_iovec_async(ds, dd, offs, lens, dt, op) == rc
    assert _host(dd).tobytes() == exp.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize('shift', [0, 4, -12])
def test_iov_offsets_any_residue_on_gpu(R, oracle, shift):
    """runs at byte offsets that are not multiples of the extent (doubles at
    4 mod 8) and negative offsets (a target whose lb < 0): split into one
    launch per residue, packed source kept in run order"""
    import torch
    rng = np.random.default_rng(99 + shift)
    nseg = 5000
    cnts = rng.integers(0, 7, nseg)
    apos, pos = [], 0                     # absolute byte positions in the buffer
    for c in cnts:
        pos += int(rng.integers(1, 5)) * 8 + int(rng.integers(0, 2)) * 4
        apos.append(pos)
        pos += int(c) * 8
    total = int(cnts.sum())
    src = rng.uniform(-1, 1, total)
    buf = rng.uniform(-1, 1, pos // 8 + 2).view(np.uint8)
    base = 4096 + shift                   # the inout pointer, inside the buffer
    offs = [a - base for a in apos]
    assert min(offs) < 0
    db, ds = _dev(buf), _dev(src)
    assert R.reduce_local_iov_async(ds, db[base:], offs, [int(c) for c in cnts], MPI_DOUBLE,
                                    SUM) == 0
    torch.cuda.synchronize()
    exp = buf.copy()
    assert oracle.reduce_local_iov(src, exp[base:], offs, [int(c) for c in cnts], MPI_DOUBLE,
                                   SUM) == 0
    assert _host(db).tobytes() == exp.tobytes()


@pytest.mark.gpu
def test_iov_misaligned_offset_refused(R):
    d = _dev(np.zeros(64, np.float64))
    s = _dev(np.zeros(4, np.float64))
    assert R.reduce_local_iov_async(s, d, [2], [1], MPI_DOUBLE, SUM) == 12
    assert R.reduce_local_iovec_async(s, d, [0], [12], MPI_DOUBLE, SUM) == 12


@pytest.mark.gpu
@pytest.mark.parametrize('dt', [DOUBLE_INT, LONG_INT, SHORT_INT, FLOAT_INT])
def test_replace_keeps_padding_on_gpu(R, oracle, dt):
    """MPI_REPLACE on every entry point: contiguous (sync), vector target,
    multi-input, all against the oracle's typemap copy"""
    from mpich_amd import handles as H
    rng = np.random.default_rng(dt & 0xff)
    n = 10007
    src, tgt = random_pairs(rng, dt, n), random_pairs(rng, dt, n)
    dd = _dev(tgt)
    assert R.MPI_Reduce_local(_dev(src), dd, n, dt, H.MPI_REPLACE) == 0
    exp = tgt.view(np.uint8).copy()
    oracle.reduce_local(src.view(np.uint8).copy(), exp, n, dt, REPLACE)
    assert _host(dd).tobytes() == exp.tobytes()
    for bl, st, cnt in ((1, 2, 3001), (3, 5, 2000), (700, 701, 3)):
        s2 = random_pairs(rng, dt, cnt * bl)
        t2 = random_pairs(rng, dt, cnt * st)
        d2 = _dev(t2)
        assert R.reduce_local_vector(_dev(s2), d2, cnt, bl, st, dt, H.MPI_REPLACE, sync=True) == 0
        e2 = t2.view(np.uint8).copy()
        oracle.reduce_local_vector(s2.view(np.uint8).copy(), e2, cnt, bl, st, dt, REPLACE)
        assert _host(d2).tobytes() == e2.tobytes(), (bl, st)
    ins = [random_pairs(rng, dt, n) for _ in range(3)]
    d3 = _dev(tgt)
    assert R.reduce_local_multi_async([_dev(x) for x in ins], d3, n, dt, H.MPI_REPLACE) == 0
    e3 = tgt.view(np.uint8).copy()
    oracle.reduce_local(ins[-1].view(np.uint8).copy(), e3, n, dt, REPLACE)
    assert _host(d3).tobytes() == e3.tobytes()


@pytest.mark.gpu
def test_iov_tables_on_two_streams(R, oracle):
    """back-to-back iov calls on different streams from one thread: a call's
    run table must not overwrite one a queued kernel still reads (two table
    slots used in turn: the third call reuses the first call's slot)"""
    import torch
    rng = np.random.default_rng(4242)
    jobs = []
    for j in range(3):
        nseg = 400000 - 150000 * j
        cnts = rng.integers(1, 5, nseg)
        offs, pos = [], 0
        for c in cnts:
            pos += int(rng.integers(0, 3))
            offs.append(pos * 8)
            pos += int(c)
        src = rng.uniform(-1, 1, int(cnts.sum()))
        dst = rng.uniform(-1, 1, pos + 1)
        jobs.append((offs, [int(c) for c in cnts], src, dst))
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    devs = [(_dev(dst), _dev(src)) for _, _, src, dst in jobs]
    for (offs, cnts, _, _), (dd, ds), st in zip(jobs, devs, streams):
        assert R.reduce_local_iov_async(ds, dd, offs, cnts, MPI_DOUBLE, SUM, st) == 0
    torch.cuda.synchronize()
    for (offs, cnts, src, dst), (dd, _) in zip(jobs, devs):
        exp = dst.copy()
        assert oracle.reduce_local_iov(src, exp, offs, cnts, MPI_DOUBLE, SUM) == 0
        assert _host(dd).tobytes() == exp.view(np.uint8).tobytes()
