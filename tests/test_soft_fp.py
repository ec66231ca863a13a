"""The software x87 extended / IEEE binary128 SUM and PROD of
mpich_amd/csrc/redop_soft.h, built for the host (tests/c/soft_check.cpp),
against the oracle's gcc-built loops -- x87 hardware (fldt/faddp/fmulp/fstpt)
and libgcc soft-fp (__addtf3 / __subtf3 / __multf3) -- on every ordered pair
of a specials table and on random values chosen to hit cancellation, carries,
ties, overflow and gradual underflow.  All 16 / 32 bytes are compared,
padding included.  The same functions run on gfx950 in
tests/test_soft_fp_gpu.py; this CPU leg checks millions of pairs in seconds.
Reference: op_fns.c:19-91 over MPIR_OP_TYPE_GROUP(FLOATING_POINT) /
(COMPLEX) / (C_COMPLEX) (mpir_op_util.h:211-236)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MPI_SUM, MPI_PROD = 0x58000003, 0x58000004
LD, REAL16, COMPLEX32, C_LD_COMPLEX = 0x4c00100c, 0x4c00102b, 0x4c00202c, 0x4c002036


@pytest.fixture(scope='module')
def soft(tmp_path_factory):
    d = tmp_path_factory.mktemp('soft')
    so = str(d / 'libsoft_check.so')
    subprocess.run(['g++', '-O2', '-std=c++17', '-shared', '-fPIC', '-D__HIP_PLATFORM_AMD__',
                    '-I/opt/rocm/include', '-I' + os.path.join(ROOT, 'mpich_amd', 'csrc'),
                    '-I' + os.path.join(ROOT, 'include'), '-o', so,
                    os.path.join(ROOT, 'tests', 'c', 'soft_check.cpp')], check=True)
    L = ctypes.CDLL(so)
    L.soft_reduce.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    return L


def x87(sign, exp, mant, pad=0):
    b = np.zeros(16, np.uint8)
    b[:8] = np.frombuffer(np.uint64(mant).tobytes(), np.uint8)
    b[8:10] = np.frombuffer(np.uint16((sign << 15) | exp).tobytes(), np.uint8)
    return b


def x87_specials():
    J = 1 << 63
    mags = [(0, 0), (0, 1), (0, J - 1), (0, 12345), (0, J), (0, J | 7), (1, J), (1, J | 7),
            (1, J + 1), (2, J), (0x3fff, J), (0x3fff, J | 1), (0x3fff, (1 << 64) - 1),
            (0x4000, J), (0x3ffe, (1 << 64) - 1), (0x403e, J), (0x3fc0, J | 3), (0x7ffe, J),
            (0x7ffe, (1 << 64) - 1), (0x7fff, J), (0x7fff, J | (1 << 62)),
            (0x7fff, J | (1 << 62) | 5), (0x7fff, J | 1), (0x7fff, J | 0x1234), (0x7fff, 0),
            (0x7fff, 5), (1, 0), (0x3fff, 1 << 62), (0x7ffe, 5), (0x2000, J | 0xabcdef)]
    return [x87(s, e, m) for s in (0, 1) for e, m in mags]


def quad(sign, exp, hi48, lo):
    b = np.zeros(16, np.uint8)
    b[:8] = np.frombuffer(np.uint64(lo).tobytes(), np.uint8)
    b[8:] = np.frombuffer(np.uint64((sign << 63) | (exp << 48) | hi48).tobytes(), np.uint8)
    return b


def quad_specials():
    F = (1 << 48) - 1
    L = (1 << 64) - 1
    mags = [(0, 0, 0), (0, 0, 1), (0, F, L), (0, 1 << 47, 0), (1, 0, 0), (1, 0, 1), (2, 0, 0),
            (0x3fff, 0, 0), (0x3fff, 0, 1), (0x3fff, F, L), (0x4000, 0, 0), (0x3ffe, F, L),
            (0x406f, 0, 0), (0x3f8f, 5, 3), (0x7ffe, 0, 0), (0x7ffe, F, L), (0x7fff, 0, 0),
            (0x7fff, 1 << 47, 0), (0x7fff, (1 << 47) | 9, 0), (0x7fff, 0, 1), (0x7fff, 5, 0),
            (0x2000, 0xabcdef, 77)]
    return [quad(s, e, h, lo) for s in (0, 1) for e, h, lo in mags]


def all_pairs(specials, rng, pad_from):
    S = np.stack(specials)
    k = len(S)
    ia, ib = np.meshgrid(np.arange(k), np.arange(k), indexing='ij')
    a, b = S[ia.reshape(-1)].copy(), S[ib.reshape(-1)].copy()
    if pad_from < 16:
        a[:, pad_from:] = rng.integers(0, 256, (len(a), 16 - pad_from), dtype=np.uint8)
        b[:, pad_from:] = rng.integers(0, 256, (len(b), 16 - pad_from), dtype=np.uint8)
    return a, b


def x87_random(rng, n, close=False):
    """normal values (J set) with exponents spread over the whole range, or
    (close) pairs whose exponents differ by 0..3, so sums cancel and carry;
    every sixteenth a denormal or pseudo-denormal"""
    m = rng.integers(0, 1 << 63, n, dtype=np.uint64) | np.uint64(1 << 63)
    e = rng.integers(1, 0x7fff, n).astype(np.uint64)
    if close:
        e = rng.integers(0x3f00, 0x4100, n).astype(np.uint64)
    s = rng.integers(0, 2, n).astype(np.uint64)
    den = rng.random(n) < 1 / 16
    m[den] &= rng.choice(np.array([(1 << 63) - 1, (1 << 64) - 1], np.uint64), den.sum())
    e[den] = 0
    out = np.zeros((n, 16), np.uint8)
    out[:, :8] = m.view(np.uint8).reshape(n, 8)
    out[:, 8:10] = ((s << 15) | e).astype(np.uint16).view(np.uint8).reshape(n, 2)
    out[:, 10:] = rng.integers(0, 256, (n, 6), dtype=np.uint8)
    return out


def quad_random(rng, n, close=False, tiny=False):
    lo = rng.integers(0, 1 << 64, n, dtype=np.uint64)
    hi48 = rng.integers(0, 1 << 48, n, dtype=np.uint64)
    e = rng.integers(1, 0x7fff, n).astype(np.uint64)
    if close:
        e = rng.integers(0x3f00, 0x4100, n).astype(np.uint64)
    if tiny:        # products near and below the denormal boundary
        e = rng.integers(0, 0x2000, n).astype(np.uint64)
    s = rng.integers(0, 2, n).astype(np.uint64)
    out = np.zeros((n, 16), np.uint8)
    out[:, :8] = lo.view(np.uint8).reshape(n, 8)
    hi = (s << np.uint64(63)) | (e << np.uint64(48)) | hi48
    out[:, 8:] = hi.view(np.uint8).reshape(n, 8)
    return out


def _check(soft, oracle, which, dt, op, a, b, ext):
    n = len(a.reshape(-1)) // ext
    want = a.reshape(-1).copy()
    assert oracle.reduce_local(b.reshape(-1).copy(), want, n, dt, op) == 0
    got = a.reshape(-1).copy()
    assert soft.soft_reduce(which, b.reshape(-1).ctypes.data, got.ctypes.data, n) == 0
    g, w = got.reshape(n, ext), want.reshape(n, ext)
    bad = np.flatnonzero((g != w).any(1))
    assert bad.size == 0, ('%d of %d differ' % (bad.size, n), bad[:4],
                           a.reshape(n, ext)[bad[:2]], b.reshape(n, ext)[bad[:2]], g[bad[:2]],
                           w[bad[:2]])


@pytest.mark.parametrize('which,op', [(0, MPI_SUM), (1, MPI_PROD)])
def test_x87_specials(soft, oracle, which, op):
    rng = np.random.default_rng(0x5EED0800 + which)
    a, b = all_pairs(x87_specials(), rng, 10)
    _check(soft, oracle, which, LD, op, a, b, 16)


@pytest.mark.parametrize('which,op', [(0, MPI_SUM), (1, MPI_PROD)])
@pytest.mark.parametrize('close', [False, True])
def test_x87_random(soft, oracle, which, op, close):
    rng = np.random.default_rng(0x5EED0810 + 2 * which + close)
    n = 400000
    a, b = x87_random(rng, n, close), x87_random(rng, n, close)
    if close and which == 0:
        b[::7, :10] = a[::7, :10]       # exact cancellations (sign flipped below)
        b[::7, 9] ^= 0x80
    _check(soft, oracle, which, LD, op, a, b, 16)


@pytest.mark.parametrize('which,op', [(2, MPI_SUM), (3, MPI_PROD)])
def test_quad_specials(soft, oracle, which, op):
    rng = np.random.default_rng(0x5EED0820 + which)
    a, b = all_pairs(quad_specials(), rng, 16)
    _check(soft, oracle, which, REAL16, op, a, b, 16)


@pytest.mark.parametrize('which,op', [(2, MPI_SUM), (3, MPI_PROD)])
@pytest.mark.parametrize('kind', ['wide', 'close', 'tiny'])
def test_quad_random(soft, oracle, which, op, kind):
    rng = np.random.default_rng(0x5EED0830 + 3 * which + len(kind))
    n = 400000
    a = quad_random(rng, n, close=kind == 'close', tiny=kind == 'tiny')
    b = quad_random(rng, n, close=kind == 'close', tiny=kind == 'tiny')
    if kind == 'close' and which == 2:
        b[::7] = a[::7]
        b[::7, 15] ^= 0x80
    _check(soft, oracle, which, REAL16, op, a, b, 16)


@pytest.mark.parametrize('which,dt,op', [(4, COMPLEX32, MPI_SUM), (5, COMPLEX32, MPI_PROD),
                                         (6, C_LD_COMPLEX, MPI_SUM), (7, C_LD_COMPLEX, MPI_PROD),
                                         (10, COMPLEX32, MPI_PROD), (11, C_LD_COMPLEX, MPI_PROD)])
def test_complex(soft, oracle, which, dt, op):
    rng = np.random.default_rng(0x5EED0840 + which)
    n = 200000
    if which in (6, 7, 11):
        parts = [x87_random(rng, n, close=True) for _ in range(4)]
        sp = np.stack(x87_specials())
    else:
        parts = [quad_random(rng, n, close=True) for _ in range(4)]
        sp = np.stack(quad_specials())
    # every tenth part a special value
    for p in parts:
        p[::10] = sp[rng.integers(0, len(sp), len(p[::10]))]
    a = np.concatenate([parts[0], parts[1]], axis=1)
    b = np.concatenate([parts[2], parts[3]], axis=1)
    _check(soft, oracle, which, dt, op, a, b, 32)


@pytest.mark.parametrize('which,dt', [(7, C_LD_COMPLEX), (5, COMPLEX32), (11, C_LD_COMPLEX),
                                      (10, COMPLEX32)])
def test_complex_prod_special_parts(soft, oracle, which, dt):
    """every (a, b, c, d) of 9 special parts: the Annex G recovery branches
    of __mulxc3 (inf boxed, NaNs zeroed, overflowed products) for x87, the
    plain struct formula for binary128"""
    J = 1 << 63
    if which in (7, 11):
        parts = [x87(0, 0, 0), x87(1, 0x3fff, J), x87(0, 0x7fff, J), x87(1, 0x7fff, J),
                 x87(0, 0x7fff, J | (1 << 62) | 3), x87(0, 0x7ffe, J), x87(1, 0x3ffe, J | 5),
                 x87(0, 0x3fff, 1 << 62), x87(1, 0, 3)]
    else:
        parts = [quad(0, 0, 0, 0), quad(1, 0x3fff, 0, 0), quad(0, 0x7fff, 0, 0),
                 quad(1, 0x7fff, 0, 0), quad(0, 0x7fff, (1 << 47) | 3, 0), quad(0, 0x7ffe, 0, 0),
                 quad(1, 0x3ffe, 5, 0), quad(0, 0, 1, 0), quad(1, 0x4000, 7, 9)]
    P = np.stack(parts)
    k = len(P)
    idx = np.array(np.meshgrid(*[np.arange(k)] * 4, indexing='ij')).reshape(4, -1)
    a = np.concatenate([P[idx[0]], P[idx[1]]], axis=1)
    b = np.concatenate([P[idx[2]], P[idx[3]]], axis=1)
    rng = np.random.default_rng(0x5EED0850 + which)
    if which in (7, 11):    # random padding in both parts of both operands
        for X in (a, b):
            X[:, 10:16] = rng.integers(0, 256, (len(X), 6), dtype=np.uint8)
            X[:, 26:32] = rng.integers(0, 256, (len(X), 6), dtype=np.uint8)
    _check(soft, oracle, which, dt, MPI_PROD, a, b, 32)


def _short_x87(rng, n, bits):
    """normal x87 values whose significand has only `bits` significant bits,
    so a product of two lands on or next to a rounding tie"""
    top = rng.integers(0, 1 << (bits - 1), n, dtype=np.uint64)
    m = (top << np.uint64(64 - bits)) | np.uint64(1 << 63)
    e = rng.integers(0x3e00, 0x4200, n).astype(np.uint64)
    e[::5] = rng.integers(1, 0x7fff, len(e[::5])).astype(np.uint64)   # near both ends too
    s = rng.integers(0, 2, n).astype(np.uint64)
    out = np.zeros((n, 16), np.uint8)
    out[:, :8] = m.view(np.uint8).reshape(n, 8)
    out[:, 8:10] = ((s << 15) | e).astype(np.uint16).view(np.uint8).reshape(n, 2)
    out[:, 10:] = rng.integers(0, 256, (n, 6), dtype=np.uint8)
    return out


def _short_quad(rng, n, bits):
    """normal binary128 values with `bits` significant bits (implicit one
    included): products of two hit the 113-bit rounding ties"""
    f = bits - 1                # fraction bits kept, from the top of the 112
    top = rng.integers(0, 1 << min(f, 48), n, dtype=np.uint64)
    hi48 = top << np.uint64(48 - min(f, 48))
    lo = np.zeros(n, np.uint64)
    if f > 48:
        lo = rng.integers(0, 1 << (f - 48), n, dtype=np.uint64) << np.uint64(64 - (f - 48))
    e = rng.integers(0x3e00, 0x4200, n).astype(np.uint64)
    e[::5] = rng.integers(1, 0x7fff, len(e[::5])).astype(np.uint64)
    s = rng.integers(0, 2, n).astype(np.uint64)
    out = np.zeros((n, 16), np.uint8)
    out[:, :8] = lo.view(np.uint8).reshape(n, 8)
    out[:, 8:] = ((s << np.uint64(63)) | (e << np.uint64(48)) | hi48).view(np.uint8).reshape(n, 8)
    return out


@pytest.mark.parametrize('ba,bb', [(32, 34), (33, 33), (31, 34)])
def test_x87_prod_rounding_ties(soft, oracle, ba, bb):
    """products of short significands (ba + bb - 1 or ba + bb bits) round at
    the 64-bit cut with the sticky bits often all zero: ties to even, and the
    carry out of an all-ones significand"""
    rng = np.random.default_rng(0x5EED0860 + ba)
    n = 200000
    _check(soft, oracle, 1, LD, MPI_PROD, _short_x87(rng, n, ba), _short_x87(rng, n, bb), 16)


@pytest.mark.parametrize('ba,bb', [(57, 58), (56, 58), (60, 55)])
def test_quad_prod_rounding_ties(soft, oracle, ba, bb):
    """the same at binary128's 113-bit cut"""
    rng = np.random.default_rng(0x5EED0870 + ba)
    n = 200000
    _check(soft, oracle, 3, REAL16, MPI_PROD, _short_quad(rng, n, ba), _short_quad(rng, n, bb), 16)


@pytest.mark.parametrize('which,dt,ext_bits,spread', [(0, LD, 40, 30), (2, REAL16, 80, 40)])
def test_sum_rounding_ties(soft, oracle, which, dt, ext_bits, spread):
    """sums of short significands whose exponents differ by 0..spread: the
    exact sum lands on rounding ties (RNE), carries into a new binade and
    cancels, on both sides of every fixed cut of the normal-operand path"""
    rng = np.random.default_rng(0x5EED0880 + which)
    n = 300000
    make = _short_x87 if which == 0 else _short_quad
    a = make(rng, n, ext_bits)
    b = make(rng, n, ext_bits)
    if which == 0:
        ea = a[:, 8:10].copy().view(np.uint16).reshape(-1) & 0x7fff
        k = rng.integers(0, spread + 1, n).astype(np.uint16)
        eb = np.clip(ea.astype(np.int64) + k - spread // 2, 1, 0x7ffe).astype(np.uint16)
        sb = b[:, 8:10].copy().view(np.uint16).reshape(-1) & 0x8000
        b[:, 8:10] = (sb | eb).view(np.uint8).reshape(n, 2)
    else:
        ha = a[:, 8:].copy().view(np.uint64).reshape(-1)
        hb = b[:, 8:].copy().view(np.uint64).reshape(-1)
        ea = ((ha >> np.uint64(48)) & np.uint64(0x7fff)).astype(np.int64)
        k = rng.integers(0, spread + 1, n)
        eb = np.clip(ea + k - spread // 2, 1, 0x7ffe).astype(np.uint64)
        hb = (hb & ~np.uint64(0x7fff << 48)) | (eb << np.uint64(48))
        b[:, 8:] = hb.view(np.uint8).reshape(n, 8)
    _check(soft, oracle, which, dt, MPI_SUM, a, b, 16)


@pytest.mark.parametrize('fast,general,dt,ext_bits', [(0, 8, LD, 40), (2, 9, REAL16, 80)])
@pytest.mark.parametrize('kind', ['wide', 'close', 'ties'])
def test_sum_fast_path_equals_general_path(soft, oracle, fast, general, dt, ext_bits, kind):
    """x87_add / quad_add's FAST = false instantiation (the general
    path alone) against the shipped fast path, bit for bit, on normal
    operands -- wide exponents, close ones (cancellation, carries) and short
    significands on rounding ties -- and both against the oracle"""
    rng = np.random.default_rng(0x5EED0890 + fast + len(kind))
    n = 200000
    if kind == 'ties':
        make = _short_x87 if fast == 0 else _short_quad
        a, b = make(rng, n, ext_bits), make(rng, n, ext_bits)
    else:
        make = x87_random if fast == 0 else quad_random
        a, b = make(rng, n, close=kind == 'close'), make(rng, n, close=kind == 'close')
    got = {}
    for which in (fast, general):
        r = a.reshape(-1).copy()
        assert soft.soft_reduce(which, b.reshape(-1).ctypes.data, r.ctypes.data, n) == 0
        got[which] = r
    assert np.array_equal(got[fast], got[general])
    _check(soft, oracle, general, dt, MPI_SUM, a, b, 16)


def _with_exponents(rng, base_a, base_b, enc, n=4000):
    """n copies of one operand pair with random signs and exponent offsets
    (the same offset on both keeps a sum's alignment; products may reach the
    ends of the exponent range and leave the fast path)"""
    a = np.repeat(base_a[None], n, 0).copy()
    b = np.repeat(base_b[None], n, 0).copy()
    if enc == 'x87':
        off = rng.integers(-16000, 16000, n)
        for X in (a, b):
            se = X[:, 8:10].copy().view(np.uint16).reshape(-1).astype(np.int64)
            e = np.clip((se & 0x7fff) + off, 1, 0x7ffe)
            s = rng.integers(0, 2, n) << 15
            X[:, 8:10] = (s | e).astype(np.uint16).view(np.uint8).reshape(n, 2)
    else:
        off = rng.integers(-16000, 16000, n)
        for X in (a, b):
            hi = X[:, 8:].copy().view(np.uint64).reshape(-1)
            e = np.clip(((hi >> np.uint64(48)) & np.uint64(0x7fff)).astype(np.int64) + off, 1, 0x7ffe)
            s = rng.integers(0, 2, n).astype(np.uint64) << np.uint64(63)
            hi = s | (e.astype(np.uint64) << np.uint64(48)) | (hi & np.uint64((1 << 48) - 1))
            X[:, 8:] = hi.view(np.uint8).reshape(n, 8)
    return a, b


@pytest.mark.parametrize('case', ['quad_prod', 'x87_prod', 'quad_sum', 'x87_sum'])
def test_rounding_carries_out_of_the_significand(soft, oracle, case):
    """operands whose exactly rounded result carries out of the significand
    (all ones + round up -> the next power of two): the 32-bit-limb fast
    paths' overflow step, against the oracle.  binary128 product: (1 + 2^-112)
    x (2 - 2^-111) = 2 - 2^-223 -> 2; x87: (1 + 2^-63) x (2 - 2^-62); sums:
    (2 - ulp) + ulp / 2, a tie to even that rounds up"""
    rng = np.random.default_rng(0x5EED08A0 + len(case))
    J = 1 << 63
    if case == 'quad_prod':
        a0, b0 = quad(0, 0x3fff, 0, 1), quad(0, 0x3fff, (1 << 48) - 1, (1 << 64) - 2)
    elif case == 'x87_prod':
        a0, b0 = x87(0, 0x3fff, J | 1), x87(0, 0x3fff, (1 << 64) - 2)
    elif case == 'quad_sum':
        a0, b0 = quad(0, 0x3fff, (1 << 48) - 1, (1 << 64) - 1), quad(0, 0x3fff - 113, 0, 0)
    else:
        a0, b0 = x87(0, 0x3fff, (1 << 64) - 1), x87(0, 0x3fff - 64, J)
    enc = 'x87' if case.startswith('x87') else 'quad'
    a, b = _with_exponents(rng, a0, b0, enc)
    if case.endswith('sum'):        # a sum keeps its operands' signs equal (no cancellation)
        b[:, 9 if enc == 'x87' else 15] = (b[:, 9 if enc == 'x87' else 15] & 0x7f) | \
            (a[:, 9 if enc == 'x87' else 15] & 0x80)
    which = {'quad_prod': 3, 'x87_prod': 1, 'quad_sum': 2, 'x87_sum': 0}[case]
    dt = LD if enc == 'x87' else REAL16
    op = MPI_PROD if case.endswith('prod') else MPI_SUM
    _check(soft, oracle, which, dt, op, a, b, 16)
    # the unscaled pair itself lands on the next power of two
    r = a0.copy()
    assert soft.soft_reduce(which, b0.ctypes.data, r.ctypes.data, 1) == 0
    if enc == 'quad':
        assert r[:8].view(np.uint64)[0] == 0 and r[8:].view(np.uint64)[0] == (0x4000 << 48), r
    else:
        assert r[:8].view(np.uint64)[0] == J and r[8:10].view(np.uint16)[0] == 0x4000, r
