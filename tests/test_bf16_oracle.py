"""The oracle's bf16 SUM against an independent numpy restatement of
op_fns.c:464-493 (bfloat16_load widens the 16 bits into the top of an fp32,
the sum is one fp32 add, bfloat16_store keeps the top 16 bits and adds one
when bit 15 is set: half-away on the magnitude bits, not round-to-nearest-
even, no NaN special case).  Exhaustive over special and tie patterns plus
random pairs.  The GPU path is checked against this oracle by the parity
sweep (test_gpu_parity.py, MPIX_BFLOAT16 SUM)."""
import numpy as np

from mpich_amd import handles as H


def _restate(a, b):
    fa = (a.astype(np.uint32) << 16).view(np.float32)
    fb = (b.astype(np.uint32) << 16).view(np.float32)
    with np.errstate(over='ignore', invalid='ignore'):
        u = (fa + fb).view(np.uint32)
    return ((u >> 16) + ((u >> 15) & 1)).astype(np.uint16)


def _is_nan(x):
    return ((x & 0x7f80) == 0x7f80) & ((x & 0x7f) != 0)


def _check(oracle, a, b):
    got = a.copy()
    assert oracle.reduce_local(b.copy(), got, len(a), H.MPIX_BFLOAT16, H.MPI_SUM) == 0
    exp = _restate(a, b)
    gn, en = _is_nan(got), _is_nan(exp)
    assert np.array_equal(gn, en)                     # NaN payloads are unpinned
    assert np.array_equal(got[~gn], exp[~en])


# ±0, ±subnormals, ±1, values one ulp apart whose fp32 sums land exactly on
# the 0x8000 tie, ±max, ±inf, NaNs
BF16_PATTERNS = np.array([0x0000, 0x8000, 0x0001, 0x8001, 0x007f, 0x807f, 0x0080, 0x8080,
                         0x3f80, 0xbf80, 0x3f81, 0xbf81, 0x3f7f, 0xbf7f, 0x4000, 0xc000,
                         0x4001, 0xc001, 0x3b80, 0xbb80, 0x3b81, 0x3c00, 0x3c01, 0x4b00,
                         0x4b01, 0xcb00, 0x7f7f, 0xff7f, 0x7f7e, 0xff7e, 0x7f80, 0xff80,
                         0x7fc0, 0xffc0, 0x7f81, 0xff81, 0x7fff, 0xffff, 0x0100, 0x8100,
                         0x3380, 0x3400, 0x3480, 0xb380, 0x4780, 0x4781, 0xc780, 0x4f00,
                         0x4f01, 0x5f00, 0x2f00, 0x2f01, 0x1f80, 0x1f81, 0x0a00, 0x8a00,
                         0x3e80, 0x3e81, 0x3d80, 0x3d81, 0x4280, 0x4281, 0xc280, 0xc281],
                        np.uint16)


def test_oracle_bf16_sum_specials_exhaustive(oracle):
    """every pair of the 64 BF16_PATTERNS"""
    a = np.repeat(BF16_PATTERNS, len(BF16_PATTERNS))
    b = np.tile(BF16_PATTERNS, len(BF16_PATTERNS))
    _check(oracle, a, b)


def test_oracle_bf16_sum_random(oracle):
    rng = np.random.default_rng(0x5EED0016)
    n = 1 << 20
    a = rng.integers(0, 1 << 16, n, dtype=np.uint16)
    b = rng.integers(0, 1 << 16, n, dtype=np.uint16)
    # half the pairs within a few exponents of each other, so the fp32 sum
    # keeps low bits that the store rounds
    close = rng.random(n) < 0.5
    b[close] = (a[close] & 0xff80) ^ rng.integers(0, 0x180, int(close.sum()), dtype=np.uint16)
    _check(oracle, a, b)
