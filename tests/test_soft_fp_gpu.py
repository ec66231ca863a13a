"""x87 extended and IEEE binary128 SUM / PROD (and their complex forms) on
gfx950 (mpich_amd/csrc/redop_soft.h) against the oracle's gcc-built loops,
every byte compared (padding included): the specials tables and random
values of tests/test_soft_fp.py (which checks the same code built for the
host on millions of pairs), here through the synchronous kernel path, the
stream-ordered one, the multi-input fold and a host (pageable) operand.
Reference: op_fns.c:19-91 over mpir_op_util.h:211-236."""
import numpy as np
import pytest
import torch

from tests import test_soft_fp as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def R():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


def dev(a):
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()
    torch.cuda.synchronize()
    return t


def _gpu_vs_oracle(R, oracle, dt, op, a, b, ext):
    n = len(a.reshape(-1)) // ext
    want = a.reshape(-1).copy()
    assert oracle.reduce_local(b.reshape(-1).copy(), want, n, dt, op) == 0
    da, db = dev(a), dev(b)
    assert R.MPI_Reduce_local(db, da, n, dt, op) == 0
    got = da.cpu().numpy()
    bad = np.flatnonzero((got.reshape(n, ext) != want.reshape(n, ext)).any(1))
    assert bad.size == 0, ('%d of %d differ' % (bad.size, n), bad[:4])
    return want


CASES = [('x87 SUM', S.LD, S.MPI_SUM), ('x87 PROD', S.LD, S.MPI_PROD),
         ('quad SUM', S.REAL16, S.MPI_SUM), ('quad PROD', S.REAL16, S.MPI_PROD)]


@pytest.mark.parametrize('name,dt,op', CASES, ids=[c[0] for c in CASES])
def test_specials_and_random(R, oracle, name, dt, op):
    rng = np.random.default_rng(0x5EED0900 + op + dt)
    if name.startswith('x87'):
        a, b = S.all_pairs(S.x87_specials(), rng, 10)
        ra, rb = S.x87_random(rng, 300000, True), S.x87_random(rng, 300000, False)
    else:
        a, b = S.all_pairs(S.quad_specials(), rng, 16)
        ra, rb = S.quad_random(rng, 300000, tiny=True), S.quad_random(rng, 300000, close=True)
    _gpu_vs_oracle(R, oracle, dt, op, a, b, 16)
    _gpu_vs_oracle(R, oracle, dt, op, ra, rb, 16)


@pytest.mark.parametrize('dt,op', [(S.COMPLEX32, S.MPI_SUM), (S.COMPLEX32, S.MPI_PROD),
                                   (S.C_LD_COMPLEX, S.MPI_SUM), (S.C_LD_COMPLEX, S.MPI_PROD)])
def test_complex(R, oracle, dt, op):
    rng = np.random.default_rng(0x5EED0910 + op + dt)
    n = 100000
    x87 = dt == S.C_LD_COMPLEX
    gen = (lambda: S.x87_random(rng, n, True)) if x87 else (lambda: S.quad_random(rng, n, True))
    sp = np.stack(S.x87_specials() if x87 else S.quad_specials())
    parts = [gen() for _ in range(4)]
    for p in parts:
        p[::9] = sp[rng.integers(0, len(sp), len(p[::9]))]
    a = np.concatenate(parts[:2], axis=1)
    b = np.concatenate(parts[2:], axis=1)
    _gpu_vs_oracle(R, oracle, dt, op, a, b, 32)


def test_entry_points(R, oracle):
    """x87 SUM (16-byte packets) through the stream-ordered call, a 3-input
    fold in one pass, and a pageable host inout"""
    rng = np.random.default_rng(0x5EED0920)
    n = 50001
    a = S.x87_random(rng, n, True)
    bs = [S.x87_random(rng, n, True) for _ in range(3)]

    def orc(b, inout):
        assert oracle.reduce_local(b.reshape(-1).copy(), inout.reshape(-1), n, S.LD, S.MPI_SUM) == 0
        return inout
    da = dev(a)
    assert R.reduce_local_async(dev(bs[0]), da, n, S.LD, S.MPI_SUM) == 0
    torch.cuda.synchronize()
    assert np.array_equal(da.cpu().numpy().reshape(n, 16), orc(bs[0], a.copy()))
    want = a.copy()
    for b in bs:
        orc(b, want)
    da = dev(a)
    R.check(R.reduce_local_multi_async([dev(b) for b in bs], da, n, S.LD, S.MPI_SUM))
    torch.cuda.synchronize()
    assert np.array_equal(da.cpu().numpy().reshape(n, 16), want)
    h = a.copy()
    assert R.MPI_Reduce_local(bs[0].copy(), h, n, S.LD, S.MPI_SUM) == 0
    assert np.array_equal(h, orc(bs[0], a.copy()))


@pytest.mark.parametrize('name,dt,op,short,ba,bb', [
    ('x87 PROD ties', S.LD, S.MPI_PROD, S._short_x87, 32, 34),
    ('quad PROD ties', S.REAL16, S.MPI_PROD, S._short_quad, 57, 58),
    ('x87 SUM ties', S.LD, S.MPI_SUM, S._short_x87, 40, 40),
    ('quad SUM ties', S.REAL16, S.MPI_SUM, S._short_quad, 80, 80)])
def test_fast_path_rounding_ties(R, oracle, name, dt, op, short, ba, bb):
    """the normal-operand fast paths (round 5) on gfx950: short significands
    whose products and sums land on rounding ties, carries and (sums with
    exponents close together) near-cancellations -- the sets
    tests/test_soft_fp.py checks on the host build, here through the AMDGPU
    code generation of the same 128-bit arithmetic"""
    rng = np.random.default_rng(0x5EED0930 + ba + op)
    n = 200000
    a, b = short(rng, n, ba), short(rng, n, bb)
    if op == S.MPI_SUM:         # exponents of b within +-8 of a's: carries and cancellations
        if dt == S.LD:
            ea = a[:, 8:10].copy().view(np.uint16).reshape(-1) & 0x7fff
            eb = np.clip(ea.astype(np.int64) + rng.integers(-8, 9, n), 1, 0x7ffe).astype(np.uint16)
            sb = b[:, 8:10].copy().view(np.uint16).reshape(-1) & 0x8000
            b[:, 8:10] = (sb | eb).view(np.uint8).reshape(n, 2)
        else:
            ha = a[:, 8:].copy().view(np.uint64).reshape(-1)
            hb = b[:, 8:].copy().view(np.uint64).reshape(-1)
            ea = ((ha >> np.uint64(48)) & np.uint64(0x7fff)).astype(np.int64)
            eb = np.clip(ea + rng.integers(-8, 9, n), 1, 0x7ffe).astype(np.uint64)
            hb = (hb & ~np.uint64(0x7fff << 48)) | (eb << np.uint64(48))
            b[:, 8:] = hb.view(np.uint8).reshape(n, 8)
    _gpu_vs_oracle(R, oracle, dt, op, a, b, 16)


# ------------------------------------------------ split combiners (round 6)
# The soft complex products run their normal-operand fast paths in the
# streaming kernel and leave any unit where one declined unchanged, recorded
# in a per-(device, stream) word buffer; a second launch combines those units
# with the general paths (redop_kernels.h is_split, k_fixup32).  Every entry
# that reaches k_contig32 -- the synchronous and stream-ordered calls, the
# two-slot tree into a separate output (recursive halving's combine_to), the
# batch -- on ragged counts (a partial last tile), declined units placed at
# word edges and inside full and partial tiles, and a buffer that grows
# between calls on one stream.
def _split_operands(rng, dt, n, special_at):
    x87 = dt == S.C_LD_COMPLEX
    gen = (lambda: S.x87_random(rng, n, True)) if x87 else (lambda: S.quad_random(rng, n, True))
    sp = np.stack(S.x87_specials() if x87 else S.quad_specials())
    parts = [gen() for _ in range(4)]
    for i, u in enumerate(special_at):
        parts[i % 4][u] = sp[rng.integers(0, len(sp))]
    return np.concatenate(parts[:2], axis=1), np.concatenate(parts[2:], axis=1)


def _oracle_prod(oracle, dt, a, b):
    n = len(a)
    want = a.reshape(-1).copy()
    assert oracle.reduce_local(b.reshape(-1).copy(), want, n, dt, S.MPI_PROD) == 0
    return want


def _same(got, want, n, what):
    bad = np.flatnonzero((got.reshape(n, 32) != want.reshape(n, 32)).any(1))
    assert bad.size == 0, (what, '%d of %d differ' % (bad.size, n), bad[:6])


@pytest.mark.parametrize('dt', [S.COMPLEX32, S.C_LD_COMPLEX], ids=['complex32', 'c_long_double'])
def test_split_product_every_entry(R, oracle, dt):
    import ctypes
    rng = np.random.default_rng(0x5EED0930 + dt)
    s = torch.cuda.current_stream()
    for n in (37, 64, 4099, 70001):
        special_at = sorted({0, 63, 64, n - 1, n // 2, n // 3} | set(rng.integers(0, n, 40).tolist()))
        special_at = [u for u in special_at if u < n]
        a, b = _split_operands(rng, dt, n, special_at)
        want = _oracle_prod(oracle, dt, a, b)
        # synchronous, in place
        da, db = dev(a), dev(b)
        assert R.MPI_Reduce_local(db, da, n, dt, S.MPI_PROD) == 0
        _same(da.cpu().numpy(), want, n, ('sync', n))
        # stream-ordered, in place
        da = dev(a)
        assert R.reduce_local_async(db, da, n, dt, S.MPI_PROD, s) == 0
        s.synchronize()
        _same(da.cpu().numpy(), want, n, ('async', n))
        # two-slot tree into a separate output: out = slot0 OP slot1 (slot 0
        # in the inout role), both slots left as they were
        da = dev(a)
        out = torch.full_like(da, 0x5A)
        assert R.reduce_local_tree_async([da, db], out, n, dt, S.MPI_PROD, s) == 0
        s.synchronize()
        _same(out.cpu().numpy(), want, n, ('tree', n))
        assert np.array_equal(da.cpu().numpy(), a.reshape(-1).view(np.uint8)), ('tree slot 0', n)
        # batch: this call's triple beside a small one of the same type
        da = dev(a)
        a2, b2 = _split_operands(rng, dt, 5, [2])
        want2 = _oracle_prod(oracle, dt, a2, b2)
        da2, db2 = dev(a2), dev(b2)
        ins = (ctypes.c_void_p * 2)(db2.data_ptr(), db.data_ptr())
        ios = (ctypes.c_void_p * 2)(da2.data_ptr(), da.data_ptr())
        cnt = (ctypes.c_ssize_t * 2)(5, n)
        assert R.lib().MPIX_Reduce_local_batch_async(ins, ios, cnt, 2, dt, S.MPI_PROD,
                                                     s.cuda_stream) == 0
        s.synchronize()
        _same(da.cpu().numpy(), want, n, ('batch', n))
        _same(da2.cpu().numpy(), want2, 5, ('batch small', n))


def test_split_fixup_buffer_grows_on_a_stream(R, oracle):
    """a small call, then one needing a larger word buffer on the same
    stream (the library synchronises the stream and reallocates), then the
    small one again -- each against the oracle"""
    rng = np.random.default_rng(0x5EED0940)
    s = torch.cuda.Stream()
    dt = S.COMPLEX32
    for n in (1000, (1 << 20) + 17, 1000):      # the middle one needs > 64 KiB of words
        special_at = [0, n - 1] + rng.integers(0, n, 16).tolist()
        a, b = _split_operands(rng, dt, n, special_at)
        want = _oracle_prod(oracle, dt, a, b)
        da, db = dev(a), dev(b)
        with torch.cuda.stream(s):
            assert R.reduce_local_async(db, da, n, dt, S.MPI_PROD, s) == 0
        s.synchronize()
        _same(da.cpu().numpy(), want, n, ('grow', n))


@pytest.mark.parametrize('dt', [S.COMPLEX32, S.C_LD_COMPLEX], ids=['complex32', 'c_long_double'])
def test_split_product_every_unit_declined(R, oracle, dt):
    """real values stored as complex: every product has a zero operand, so
    the fast kernel declines every unit and the fixup launch combines whole
    words of them (densely marked words, ragged tails, the tree form)"""
    rng = np.random.default_rng(0x5EED0940 + dt)
    s = torch.cuda.current_stream()
    for n in (1, 63, 64, 65, 4099, 70001):
        a, b = _split_operands(rng, dt, n, [])
        a[:, 16:] = 0           # the imaginary parts: +0
        b[:, 16:] = 0
        want = _oracle_prod(oracle, dt, a, b)
        da, db = dev(a), dev(b)
        assert R.MPI_Reduce_local(db, da, n, dt, S.MPI_PROD) == 0
        _same(da.cpu().numpy(), want, n, ('sync', n))
        da = dev(a)
        assert R.reduce_local_async(db, da, n, dt, S.MPI_PROD, s) == 0
        s.synchronize()
        _same(da.cpu().numpy(), want, n, ('async', n))
        da = dev(a)
        out = torch.full_like(da, 0x5A)
        assert R.reduce_local_tree_async([da, db], out, n, dt, S.MPI_PROD, s) == 0
        s.synchronize()
        _same(out.cpu().numpy(), want, n, ('tree', n))
