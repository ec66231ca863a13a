"""CPU check of the four-bytes-per-dword forms of the 1-byte logical ops
(redop_ops.h: nz_bytes, ILand/ILor/ILxor::apply4) against the per-element
rule of op_fns.c:99-187 ((a != 0) OP (b != 0), 0/1 in the element type), on
every pair of byte values in every lane position.  The formulas are restated
here in numpy with uint32 arithmetic (wrap-around as on the GPU); the GPU
sweeps (test_gpu_parity.py, test_c3_full.py) run the kernels themselves."""
import numpy as np


def nz_bytes(x):
    x = x.astype(np.uint32)
    return (((x & np.uint32(0x7f7f7f7f)) + np.uint32(0x7f7f7f7f)) | x) & np.uint32(0x80808080)


def test_swar_logicals_every_byte_pair():
    a8, b8 = np.meshgrid(np.arange(256, dtype=np.uint8), np.arange(256, dtype=np.uint8))
    a8, b8 = a8.ravel(), b8.ravel()
    rng = np.random.default_rng(0x5EED5A)
    for lane in range(4):
        # the pair in one lane, random bytes in the other three (carries must not leak)
        fill_a = rng.integers(0, 256, (a8.size, 4), dtype=np.uint8)
        fill_b = rng.integers(0, 256, (a8.size, 4), dtype=np.uint8)
        fill_a[:, lane], fill_b[:, lane] = a8, b8
        A = fill_a.copy().view(np.uint32).ravel()
        B = fill_b.copy().view(np.uint32).ravel()
        got = {'land': (nz_bytes(A) & nz_bytes(B)) >> 7,
               'lor': nz_bytes(A | B) >> 7,
               'lxor': (nz_bytes(A) ^ nz_bytes(B)) >> 7}
        exp = {'land': (fill_a != 0) & (fill_b != 0), 'lor': (fill_a != 0) | (fill_b != 0),
               'lxor': (fill_a != 0) ^ (fill_b != 0)}
        for k in got:
            g = got[k].astype(np.uint32).view(np.uint8).reshape(-1, 4)
            assert np.array_equal(g, exp[k].astype(np.uint8)), (k, lane)


def _to_int32(v):
    """C's (int) conversion of a long long (two's complement wrap)"""
    v &= 0xffffffff
    return v - (1 << 32) if v >= (1 << 31) else v


def test_swar_fortran_logical1_every_byte_pair():
    """FLand/FLor/FLxor<int8_t>::apply4p (redop_ops.h: flog_true_bytes,
    flog_to_bytes) against the per-element rule of mpii_fortlogical.h:13-29 as
    the kernels' apply() restates it: a byte is .TRUE. unless (int) byte ==
    (int) .FALSE., and the result is (int8_t) (.TRUE. or .FALSE.), for
    .TRUE./.FALSE. encodings inside and outside the kind's range"""
    a8, b8 = np.meshgrid(np.arange(256, dtype=np.uint8), np.arange(256, dtype=np.uint8))
    a8, b8 = a8.ravel(), b8.ravel()
    rng = np.random.default_rng(0x5EED5B)
    for ftrue, ffalse in ((1, 0), (-1, 0), (0, 1), (255, 0), (1, -1), (7, 300), (1, 1 << 33),
                          (-1 << 40, 0x80)):
        f = _to_int32(ffalse)
        fits = -128 <= f <= 127
        trb, fab = np.uint32(ftrue & 0xff), np.uint32(ffalse & 0xff)
        for lane in range(4):
            fill_a = rng.integers(0, 256, (a8.size, 4), dtype=np.uint8)
            fill_b = rng.integers(0, 256, (a8.size, 4), dtype=np.uint8)
            fill_a[:, lane], fill_b[:, lane] = a8, b8
            A = fill_a.copy().view(np.uint32).ravel()
            B = fill_b.copy().view(np.uint32).ravel()

            def true_bytes(x):
                if not fits:
                    return np.full_like(x, 0x80808080)
                return nz_bytes(x ^ np.uint32((f & 0xff) * 0x01010101))

            def to_bytes(t):
                m = (t >> np.uint32(7)) * np.uint32(0xff)
                return (trb * np.uint32(0x01010101) & m) | (fab * np.uint32(0x01010101) & ~m)
            ta, tb = true_bytes(A), true_bytes(B)
            got = {'land': to_bytes(ta & tb), 'lor': to_bytes(ta | tb), 'lxor': to_bytes(ta ^ tb)}
            la = fill_a.astype(np.int8).astype(np.int32) != f      # flog_from in int
            lb = fill_b.astype(np.int8).astype(np.int32) != f
            for k, c in (('land', la & lb), ('lor', la | lb), ('lxor', la ^ lb)):
                exp = np.where(c, np.uint8(ftrue & 0xff), np.uint8(ffalse & 0xff))
                g = got[k].astype(np.uint32).view(np.uint8).reshape(-1, 4)
                assert np.array_equal(g, exp), (k, lane, ftrue, ffalse)


def _minmax_bytes(A, B, signed, is_max):
    """IMax / IMin<1-byte T>::apply4 (redop_ops.h minmax_bytes): each byte in
    the high half of a 16-bit lane (low half zero), a packed 16-bit max / min
    of that signedness for the odd and for the even bytes, then the bytes
    interleaved back"""
    m = np.uint32(0xff00ff00)
    t = np.int16 if signed else np.uint16
    f = np.maximum if is_max else np.minimum
    ro = f((A & m).view(t), (B & m).view(t)).view(np.uint32)
    re = f(((A << np.uint32(8)) & m).view(t), ((B << np.uint32(8)) & m).view(t)).view(np.uint32)
    # v_perm_b32(ro, re, 0x07030501): bytes re.b1, ro.b1, re.b3, ro.b3
    rb, ob = re.view(np.uint8).reshape(-1, 4), ro.view(np.uint8).reshape(-1, 4)
    return np.stack([rb[:, 1], ob[:, 1], rb[:, 3], ob[:, 3]], 1)


def test_swar_minmax_every_byte_pair():
    """1-byte MAX / MIN four per dword against (a > b) ? a : b and
    (a < b) ? a : b (mpl_base.h:105-106 via op_fns.c), signed and unsigned,
    every pair of byte values in every lane beside random neighbours"""
    a8, b8 = np.meshgrid(np.arange(256, dtype=np.uint8), np.arange(256, dtype=np.uint8))
    a8, b8 = a8.ravel(), b8.ravel()
    rng = np.random.default_rng(0x5EED5C)
    for lane in range(4):
        fill_a = rng.integers(0, 256, (a8.size, 4), dtype=np.uint8)
        fill_b = rng.integers(0, 256, (a8.size, 4), dtype=np.uint8)
        fill_a[:, lane], fill_b[:, lane] = a8, b8
        A = fill_a.copy().view(np.uint32).ravel()
        B = fill_b.copy().view(np.uint32).ravel()
        for signed in (False, True):
            va = fill_a.view(np.int8) if signed else fill_a
            vb = fill_b.view(np.int8) if signed else fill_b
            for is_max in (True, False):
                exp = np.where(va > vb, va, vb) if is_max else np.where(va < vb, va, vb)
                got = _minmax_bytes(A, B, signed, is_max)
                assert np.array_equal(got, exp.view(np.uint8)), (lane, signed, is_max)
