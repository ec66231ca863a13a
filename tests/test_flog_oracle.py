"""The oracle's Fortran-logical rules against an independent numpy restatement
of mpii_fortlogical.h:13-29 (MPII_FROM_FLOG(a) = a == MPIR_fortran_false ? 0
: 1 after C's usual promotion against an int; MPII_TO_FLOG(c) = c ? .TRUE. :
.FALSE. converted to the kind) for every logical kind and for .TRUE./.FALSE.
encodings that do and do not fit the kind.  The GPU parity test
test_gpu_parity.py::test_fortran_logical_kinds checks the HIP path against
this oracle on the same encodings."""
import numpy as np
import pytest

from mpich_amd import handles as H

KINDS = [('MPI_LOGICAL1', np.int8), ('MPI_LOGICAL2', np.int16), ('MPI_LOGICAL4', np.int32),
         ('MPI_LOGICAL8', np.int64)]
BOOLS = [(1, 0), (-1, 0), (5, -3), (300, 7), (7, 300), (0, 1), (-70000, 70000)]


def _restate(a, b, op, tv, fv, npdt):
    # promotion: every kind up to 8 bytes compares exactly in int64 against
    # the int .FALSE. (signed kinds, int fits int64)
    fa = a.astype(np.int64) != fv
    fb = b.astype(np.int64) != fv
    r = {H.MPI_LAND: fa & fb, H.MPI_LOR: fa | fb, H.MPI_LXOR: fa ^ fb}[op]
    # conversion of the int .TRUE./.FALSE. to the kind: modulo 2^bits
    t = np.array([tv], np.int64).astype(npdt)[0]
    f = np.array([fv], np.int64).astype(npdt)[0]
    return np.where(r, t, f).astype(npdt)


@pytest.mark.parametrize('kind,npdt', KINDS)
@pytest.mark.parametrize('tv,fv', BOOLS)
def test_oracle_flog_matches_restatement(oracle, kind, npdt, tv, fv):
    dt = getattr(H, kind)
    rng = np.random.default_rng(abs(tv) * 31 + abs(fv) + np.dtype(npdt).itemsize)
    n = 4099
    pick = np.array([tv, fv, 0, 1, -1], np.int64)
    a = np.where(rng.random(n) < 0.8, pick[rng.integers(0, 5, n)],
                 rng.integers(-(1 << 62), 1 << 62, n)).astype(npdt)
    b = np.where(rng.random(n) < 0.8, pick[rng.integers(0, 5, n)],
                 rng.integers(-(1 << 62), 1 << 62, n)).astype(npdt)
    try:
        oracle.set_fortran_booleans(tv, fv)
        for op in (H.MPI_LAND, H.MPI_LOR, H.MPI_LXOR):
            got = a.copy()
            assert oracle.reduce_local(b.copy(), got, n, dt, op) == 0
            assert np.array_equal(got, _restate(a, b, op, tv, fv, npdt)), (kind, tv, fv, op)
    finally:
        oracle.set_fortran_booleans(1, 0)


@pytest.mark.parametrize('tv,fv', BOOLS)
def test_oracle_flog16_matches_restatement(oracle, tv, fv):
    """LOGICAL16: the 128-bit word is compared in full (a word whose low half
    equals .FALSE. but whose high half is not its sign extension is .TRUE.)"""
    rng = np.random.default_rng(abs(tv) + 7 * abs(fv))
    n = 2003

    def words():
        lo = np.where(rng.random(n) < 0.8, np.array([tv, fv, 0, 1, -1], np.int64)[
            rng.integers(0, 5, n)], rng.integers(-(1 << 62), 1 << 62, n))
        hi = np.where(lo < 0, -1, 0)
        hi = np.where(rng.random(n) < 0.2, rng.integers(-(1 << 62), 1 << 62, n), hi)
        return np.stack([lo, hi], 1).astype(np.int64)

    a, b = words(), words()
    fhi = -1 if fv < 0 else 0

    def truth(w):
        return ~((w[:, 0] == fv) & (w[:, 1] == fhi))

    try:
        oracle.set_fortran_booleans(tv, fv)
        for op in (H.MPI_LAND, H.MPI_LOR, H.MPI_LXOR):
            got = a.copy()
            assert oracle.reduce_local(b.copy(), got, n, H.MPI_LOGICAL16, op) == 0
            ta, tb = truth(a), truth(b)
            r = {H.MPI_LAND: ta & tb, H.MPI_LOR: ta | tb, H.MPI_LXOR: ta ^ tb}[op]
            exp = np.where(r[:, None], [[tv, -1 if tv < 0 else 0]],
                           [[fv, fhi]]).astype(np.int64)
            assert np.array_equal(got, exp), (tv, fv, op)
    finally:
        oracle.set_fortran_booleans(1, 0)
