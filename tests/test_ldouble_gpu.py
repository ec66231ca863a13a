"""MAX/MIN on MPI_LONG_DOUBLE (x87 80-bit extended in a 16-byte slot) and
MPI_REAL16 (IEEE binary128), MAXLOC/MINLOC on MPI_LONG_DOUBLE_INT and
MPIR_2FLOAT128 -- the compare-and-select ops of MPIR_OP_TYPE_GROUP(
FLOATING_POINT)'s ALT_FLOAT128 / FLOAT128 members (mpir_op_util.h:211-217,
op_fns.c:257-435), done on gfx950 in integer arithmetic.

Checked bit for bit (all 16 / 32 bytes, padding included) against the oracle,
whose loops gcc compiles to the same x87 fcomi + fstpt and libgcc __gttf2 /
__lttf2 code MPICH's op_fns.c becomes on x86-64: every ordered pair of a
specials table (zeros, denormals, pseudo-denormals, normals, extremes,
infinities, quiet / signalling NaNs and, for x87, the unsupported encodings:
unnormals, pseudo-infinities, pseudo-NaNs -- each with random padding), plus
random bytes, through the synchronous, stream-ordered, multi-input, tree,
vector-target and host-resident entry points."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


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
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()
    torch.cuda.synchronize()
    return t


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def x87(sign, exp, mant):
    """16-byte slot: significand (explicit J bit 63), sign | exponent, padding"""
    b = np.zeros(16, np.uint8)
    b[:8] = np.frombuffer(np.uint64(mant).tobytes(), np.uint8)
    b[8:10] = np.frombuffer(np.uint16((sign << 15) | exp).tobytes(), np.uint8)
    return b


def x87_specials():
    J = 1 << 63
    mags = [
        (0, 0),                         # zero
        (0, 1), (0, J - 1), (0, 12345),  # denormals
        (0, J), (0, J | 7),             # pseudo-denormals (compare as exponent 1)
        (1, J), (1, J | 7), (1, J + 1),  # smallest normals
        (0x3fff, J), (0x3fff, J | 1), (0x4000, J), (0x3ffe, (1 << 64) - 1),
        (0x7ffe, (1 << 64) - 1),        # largest finite
        (0x7fff, J),                    # infinity
        (0x7fff, J | (1 << 62)), (0x7fff, J | (1 << 62) | 5),   # quiet NaNs
        (0x7fff, J | 1), (0x7fff, J | 0x1234),                  # signalling NaNs
        (0x7fff, 0), (0x7fff, 5),       # pseudo-infinity, pseudo-NaN (J = 0)
        (1, 0), (0x3fff, 1 << 62), (0x7ffe, 5),                 # unnormals (J = 0)
    ]
    return [x87(s, e, m) for s in (0, 1) for e, m in mags]


def quad(sign, exp, hi48, lo):
    b = np.zeros(16, np.uint8)
    b[:8] = np.frombuffer(np.uint64(lo).tobytes(), np.uint8)
    hi = (sign << 63) | (exp << 48) | hi48
    b[8:] = np.frombuffer(np.uint64(hi).tobytes(), np.uint8)
    return b


def quad_specials():
    F = (1 << 48) - 1
    mags = [(0, 0, 0), (0, 0, 1), (0, F, (1 << 64) - 1), (1, 0, 0), (1, 0, 1), (0x3fff, 0, 0),
            (0x3fff, 0, 1), (0x3fff, 1, 0), (0x7ffe, F, (1 << 64) - 1), (0x7fff, 0, 0),
            (0x7fff, 1 << 47, 0), (0x7fff, 1 << 47, 9), (0x7fff, 0, 1), (0x7fff, 5, 0)]
    return [quad(s, e, h, lo) for s in (0, 1) for e, h, lo in mags]


def pairs_of(specials, rng, pad_from=10):
    """every ordered pair (a, b) of the specials, then random values of the
    same table; random padding bytes (from byte pad_from) on every element"""
    k = len(specials)
    S = np.stack(specials)
    ia, ib = np.meshgrid(np.arange(k), np.arange(k), indexing='ij')
    a, b = S[ia.reshape(-1)].copy(), S[ib.reshape(-1)].copy()
    extra = 4099
    a = np.concatenate([a, S[rng.integers(0, k, extra)]])
    b = np.concatenate([b, S[rng.integers(0, k, extra)]])
    for x in (a, b):
        x[:, pad_from:] = rng.integers(0, 256, (len(x), 16 - pad_from), dtype=np.uint8)
    return a, b


def check(R, oracle, a, b, dt, op, ext):
    n = len(a.reshape(-1)) // ext
    exp = a.reshape(-1).copy()
    assert oracle.reduce_local(b.reshape(-1).copy(), exp, n, dt, op) == 0
    da, db = dev(a), dev(b)
    assert R.MPI_Reduce_local(db, da, n, dt, op) == 0
    got = host(da)
    bad = np.flatnonzero((got.reshape(n, ext) != exp.reshape(n, ext)).any(1))
    assert bad.size == 0, (hex(op), bad[:5], got.reshape(n, ext)[bad[:3]], exp.reshape(n, ext)[bad[:3]])
    return exp


@pytest.mark.parametrize('opname', ['MPI_MAX', 'MPI_MIN'])
def test_long_double_specials(R, H, oracle, opname):
    rng = np.random.default_rng(0x5EED0600)
    a, b = pairs_of(x87_specials(), rng)
    assert R.is_supported(getattr(H, opname), H.MPI_LONG_DOUBLE)
    exp = check(R, oracle, a, b, H.MPI_LONG_DOUBLE, getattr(H, opname), 16)
    # fstpt stores 10 bytes: inout's padding survives whatever was selected
    assert np.array_equal(exp.reshape(-1, 16)[:, 10:], a[:, 10:])


@pytest.mark.parametrize('opname', ['MPI_MAX', 'MPI_MIN'])
def test_long_double_random_bytes(R, H, oracle, opname):
    rng = np.random.default_rng(0x5EED0601)
    n = (1 << 18) + 5
    a = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    b = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    a[::2, 7] |= 0x80       # half of them with J set, so the ordered cases are common
    b[::3, 7] |= 0x80
    check(R, oracle, a, b, H.MPI_LONG_DOUBLE, getattr(H, opname), 16)


@pytest.mark.parametrize('opname', ['MPI_MAX', 'MPI_MIN'])
def test_real16_specials(R, H, oracle, opname):
    rng = np.random.default_rng(0x5EED0602)
    a, b = pairs_of(quad_specials(), rng, pad_from=16)
    check(R, oracle, a, b, H.MPI_REAL16, getattr(H, opname), 16)


def loc_records(vals_a, vals_b, rng, vbytes):
    """32-byte records {value 16 B, loc, padding}: MPI_LONG_DOUBLE_INT keeps
    an int at 16 (bytes 20-31 padding), MPIR_2FLOAT128 a binary128 loc"""
    n = len(vals_a)
    A = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    B = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    A[:, :vbytes] = vals_a[:, :vbytes]
    B[:, :vbytes] = vals_b[:, :vbytes]
    # locs from a small range so ties on equal values meet both orders
    for X in (A, B):
        X[:, 16:20] = np.frombuffer(rng.integers(-3, 4, n).astype('<i4').tobytes(),
                                    np.uint8).reshape(n, 4)
    return A, B


@pytest.mark.parametrize('opname', ['MPI_MAXLOC', 'MPI_MINLOC'])
def test_long_double_int_specials(R, H, oracle, opname):
    rng = np.random.default_rng(0x5EED0603)
    a, b = pairs_of(x87_specials(), rng)
    A, B = loc_records(a, b, rng, 16)
    assert R.is_supported(getattr(H, opname), H.MPI_LONG_DOUBLE_INT)
    exp = check(R, oracle, A, B, H.MPI_LONG_DOUBLE_INT, getattr(H, opname), 32)
    e = exp.reshape(-1, 32)
    assert np.array_equal(e[:, 10:16], A[:, 10:16]) and np.array_equal(e[:, 20:], A[:, 20:])


@pytest.mark.parametrize('opname', ['MPI_MAXLOC', 'MPI_MINLOC'])
def test_2float128_specials(R, H, oracle, opname):
    rng = np.random.default_rng(0x5EED0604)
    a, b = pairs_of(quad_specials(), rng, pad_from=16)
    la, lb = pairs_of(quad_specials(), rng, pad_from=16)
    A = np.concatenate([a, la[:len(a)]], axis=1)
    B = np.concatenate([b, lb[:len(b)]], axis=1)
    # equal values with locs in both orders (the MPL_MIN tie rule)
    B[::5, :16] = A[::5, :16]
    check(R, oracle, A, B, H.MPIR_2FLOAT128, getattr(H, opname), 32)


def test_long_double_int_other_entry_points(R, H, oracle):
    """the 32-byte unit through the element-wise kernels of every entry:
    stream-ordered, 4-input multi (one pass), tree of 4, vector target,
    and pageable host operands"""
    rng = np.random.default_rng(0x5EED0605)
    dt, op = H.MPI_LONG_DOUBLE_INT, H.MPI_MAXLOC
    n = 20011
    spec = np.stack(x87_specials())
    ins = []
    for _ in range(5):
        v = spec[rng.integers(0, len(spec), n)]
        X, _ = loc_records(v, v, rng, 16)
        ins.append(X)
    a, bs = ins[0], ins[1:]

    def orc(inb, inout):
        cnt = len(inout)        # records (rows of 32 bytes)
        assert len(inb) == cnt
        assert oracle.reduce_local(inb.reshape(-1).copy(), inout.reshape(-1), cnt, dt, op) == 0
        return inout
    # stream-ordered
    da = dev(a)
    assert R.reduce_local_async(dev(bs[0]), da, n, dt, op, torch.cuda.current_stream()) == 0
    assert np.array_equal(host(da).reshape(n, 32), orc(bs[0], a.copy()))
    # multi: ((a op b0) op b1) ...
    want = a.copy()
    for b in bs:
        orc(b, want)
    da = dev(a)
    R.check(R.reduce_local_multi_async([dev(b) for b in bs], da, n, dt, op))
    assert np.array_equal(host(da).reshape(n, 32), want)
    # tree of 4 slots: (s0 op s1) op (s2 op s3), slot s the inout of its pair
    want_tree = orc(orc(bs[3], bs[2].copy()), orc(bs[1], bs[0].copy()))
    out = torch.empty(n * 32, dtype=torch.uint8, device='cuda')
    R.check(R.reduce_local_tree_async([dev(b) for b in bs], out, n, dt, op))
    assert np.array_equal(host(out).reshape(n, 32), want_tree)
    # vector target (count, blocklen 1, stride 3)
    m = n // 3
    tgt = a.copy()
    src = bs[0][:m].copy()
    want_v = tgt.copy()
    sel = want_v[0:3 * m:3].copy()         # the target's payload records
    orc(src, sel)
    want_v[0:3 * m:3] = sel
    dt_ = dev(tgt)
    R.check(R.reduce_local_vector(dev(src), dt_, m, 1, 3, dt, op))
    assert np.array_equal(host(dt_).reshape(n, 32), want_v)
    # pageable host operands (staged / bounced by the library)
    ha = a.copy()
    assert R.MPI_Reduce_local(bs[0].copy(), ha, n, dt, op) == 0
    assert np.array_equal(ha, orc(bs[0], a.copy()))


@pytest.mark.parametrize('n', [1, 63, 64, 511, 512, 513, 3 * 512 + 7, 20011])
@pytest.mark.parametrize('offs', [(0, 0), (16, 0), (0, 16), (16, 16), (8, 8)])
def test_contig32_tiles_and_offsets(R, H, oracle, n, offs):
    """k_contig32 (32-byte units, whole-line packet loads plus an adjacent-lane
    swap; 512-unit tiles of 256 lanes x 2 runs) across the tile boundaries and
    the last partial tile, with in / inout at 16-byte offsets that keep the
    packet path (0, 16: units on or off the 32-byte grid) and both 8 bytes off
    the 16-byte grid (the element-wise kernel); MAXLOC on MPI_LONG_DOUBLE_INT
    specials, bit for bit with the padding"""
    rng = np.random.default_rng(0x5EED0610 + n)
    dt, op = H.MPI_LONG_DOUBLE_INT, H.MPI_MAXLOC
    spec = np.stack(x87_specials())
    A, B = loc_records(spec[rng.integers(0, len(spec), n)], spec[rng.integers(0, len(spec), n)],
                       rng, 16)
    exp = A.reshape(-1).copy()
    assert oracle.reduce_local(B.reshape(-1).copy(), exp, n, dt, op) == 0
    oi, oo = offs
    bi = torch.zeros(n * 32 + 64, dtype=torch.uint8, device='cuda')
    bo = torch.zeros(n * 32 + 64, dtype=torch.uint8, device='cuda')
    bi[oi:oi + n * 32] = torch.from_numpy(B.reshape(-1).copy()).cuda()
    bo[oo:oo + n * 32] = torch.from_numpy(A.reshape(-1).copy()).cuda()
    guard = bo.cpu().numpy().copy()
    assert R.MPI_Reduce_local(bi[oi:], bo[oo:], n, dt, op) == 0
    got = host(bo)
    assert np.array_equal(got[oo:oo + n * 32], exp)
    # nothing outside the target span is written
    assert np.array_equal(got[:oo], guard[:oo]) and np.array_equal(got[oo + n * 32:],
                                                                   guard[oo + n * 32:])


@pytest.mark.parametrize('n', [1, 511, 512, 1500, 20011])
@pytest.mark.parametrize('target', ['separate', 'slot0', 'slot1'])
def test_contig32_two_slot_tree(R, H, oracle, n, target):
    """out = slot 0 OP slot 1 on MPI_LONG_DOUBLE_INT (recursive halving's
    combine_to on 32-byte units): k_contig32 with slot 0 in the inout role,
    into a separate output or in place over either slot; bit for bit with
    the oracle's reduce_local(in = slot 1, inout = slot 0)"""
    rng = np.random.default_rng(0x5EED0620 + n)
    dt, op = H.MPI_LONG_DOUBLE_INT, H.MPI_MAXLOC
    spec = np.stack(x87_specials())
    A, B = loc_records(spec[rng.integers(0, len(spec), n)], spec[rng.integers(0, len(spec), n)],
                       rng, 16)
    exp = A.reshape(-1).copy()
    assert oracle.reduce_local(B.reshape(-1).copy(), exp, n, dt, op) == 0
    da, db = dev(A), dev(B)
    out = {'separate': torch.zeros(n * 32, dtype=torch.uint8, device='cuda'), 'slot0': da,
           'slot1': db}[target]
    torch.cuda.synchronize()
    assert R.reduce_local_tree_async([da, db], out, n, dt, op) == 0
    assert np.array_equal(host(out), exp)
