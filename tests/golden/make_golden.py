#!/usr/bin/env python3
"""Generate the golden vectors that pin the oracle (and the HIP path).

Every case here is DATA: per-rank input vectors plus the expected result,
taken from the closed forms the reference's own tests assert, or from a
semantic rule read off the reference source (cited per case).  Nothing
here runs, imports or compiles reference code, and nothing here calls the
oracle: expected values come from the rules below, computed with numpy.

A case folds its P inputs left to right exactly like a chain of
MPI_Reduce_local calls:  acc = inputs[0];  for r in 1..P-1:
reduce_local(in=inputs[r], inout=acc).  For the two-operand edge cases
inputs[0] is the inout operand a and inputs[1] the in operand b, so the
expected value is OP(a, b) in the reference's a = OP(a, b) order
(src/include/mpir_op_util.h:46-53).

Outputs (committed): tests/golden/kat_manifest.json + kat_vectors.npz.
Run:  python tests/golden/make_golden.py
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# ---- handles (src/include/mpi.h.in:166-311) -------------------------------
OPS = dict(MAX=0x58000001, MIN=0x58000002, SUM=0x58000003, PROD=0x58000004,
           LAND=0x58000005, BAND=0x58000006, LOR=0x58000007, BOR=0x58000008,
           LXOR=0x58000009, BXOR=0x5800000a, MINLOC=0x5800000b,
           MAXLOC=0x5800000c, REPLACE=0x5800000d, NO_OP=0x5800000e, EQUAL=0x5800000f)

DT = dict(
    MPI_CHAR=0x4c000101, MPI_UNSIGNED_CHAR=0x4c000102, MPI_SHORT=0x4c000203,
    MPI_UNSIGNED_SHORT=0x4c000204, MPI_INT=0x4c000405, MPI_UNSIGNED=0x4c000406,
    MPI_LONG=0x4c000807, MPI_UNSIGNED_LONG=0x4c000808, MPI_LONG_LONG=0x4c000809,
    MPI_FLOAT=0x4c00040a, MPI_DOUBLE=0x4c00080b, MPI_LONG_DOUBLE=0x4c00100c,
    MPI_BYTE=0x4c00010d, MPI_2INT=0x4c000816, MPI_SIGNED_CHAR=0x4c000118,
    MPI_LOGICAL=0x4c00041d, MPI_DOUBLE_COMPLEX=0x4c001022,
    MPI_INT8_T=0x4c000137, MPI_INT16_T=0x4c000238, MPI_INT32_T=0x4c000439,
    MPI_INT64_T=0x4c00083a, MPI_UINT8_T=0x4c00013b, MPI_UINT16_T=0x4c00023c,
    MPI_UINT32_T=0x4c00043d, MPI_UINT64_T=0x4c00083e, MPI_C_BOOL=0x4c00013f,
    MPI_C_FLOAT_COMPLEX=0x4c000840, MPI_C_DOUBLE_COMPLEX=0x4c001041,
    MPI_AINT=0x4c000843, MPI_OFFSET=0x4c000844, MPI_COUNT=0x4c000845,
    MPIX_C_FLOAT16=0x4c000246, MPIX_BFLOAT16=0x4c00024c,
    MPI_FLOAT_INT=0x8c000000, MPI_DOUBLE_INT=0x8c000001, MPI_LONG_INT=0x8c000002,
    MPI_SHORT_INT=0x8c000003, MPI_LONG_DOUBLE_INT=0x8c000004,
    MPI_2REAL=0x4c000821, MPI_2DOUBLE_PRECISION=0x4c001023,
)

# numpy layouts of one element (x86-64 LP64; pair padding as pairtypes.c:15-21)
PAIR = {
    'MPI_2INT': np.dtype([('v', '<i4'), ('l', '<i4')]),
    'MPI_LONG_INT': np.dtype([('v', '<i8'), ('l', '<i4'), ('p', '<i4')]),
    'MPI_SHORT_INT': np.dtype([('v', '<i2'), ('p', '<i2'), ('l', '<i4')]),
    'MPI_FLOAT_INT': np.dtype([('v', '<f4'), ('l', '<i4')]),
    'MPI_DOUBLE_INT': np.dtype([('v', '<f8'), ('l', '<i4'), ('p', '<i4')]),
    'MPI_LONG_DOUBLE_INT': np.dtype([('v', np.longdouble), ('l', '<i4'), ('p', 'V12')]),
    'MPI_2REAL': np.dtype([('v', '<f4'), ('l', '<f4')]),
    'MPI_2DOUBLE_PRECISION': np.dtype([('v', '<f8'), ('l', '<f8')]),
}

INT_NP = {
    'MPI_INT': '<i4', 'MPI_LONG': '<i8', 'MPI_SHORT': '<i2',
    'MPI_UNSIGNED_SHORT': '<u2', 'MPI_UNSIGNED': '<u4', 'MPI_UNSIGNED_LONG': '<u8',
    'MPI_UNSIGNED_CHAR': '<u1', 'MPI_INT8_T': '<i1', 'MPI_INT16_T': '<i2',
    'MPI_INT32_T': '<i4', 'MPI_INT64_T': '<i8', 'MPI_UINT8_T': '<u1',
    'MPI_UINT16_T': '<u2', 'MPI_UINT32_T': '<u4', 'MPI_UINT64_T': '<u8',
    'MPI_AINT': '<i8', 'MPI_OFFSET': '<i8', 'MPI_COUNT': '<i8',
}

cases = []
arrays = {}


def add(name, dtname, op, inputs, expected, source, rule, nan_equiv=False, cmp=None):
    """inputs: list of P numpy arrays (same dtype); expected: numpy array.
    cmp: 'bytes' (bit-exact, default), 'nan_equiv' (bit-exact except that any
    NaN matches any NaN: FP SUM/PROD payloads are unpinned), or 'fields'
    (compare the value/loc fields by value: x87 long double padding bytes
    are undefined)."""
    if cmp is None:
        cmp = 'nan_equiv' if nan_equiv else 'bytes'
    dt = expected.dtype
    layout = dt.descr if dt.fields else dt.str
    cid = 'c%04d' % len(cases)
    ins = np.stack([np.frombuffer(x.tobytes(), np.uint8) for x in inputs])
    out = np.frombuffer(expected.tobytes(), np.uint8).copy()
    assert ins.shape[1] == out.shape[0]
    arrays[cid + '_in'] = ins
    arrays[cid + '_out'] = out
    cases.append(dict(id=cid, name=name, datatype=DT[dtname], datatype_name=dtname,
                      op=OPS[op], op_name=op, nranks=len(inputs),
                      count=int(expected.shape[0]), nbytes=int(out.shape[0]),
                      source=source, rule=rule, cmp=cmp, layout=layout))


def int_cast(vals, npt):
    """C assignment of a long long to an integer of npt's width
    (allred.c:159-177 casts through the signed type of that size)."""
    bits = np.dtype(npt).itemsize * 8
    m = (1 << bits) - 1
    return np.array([int(v) & m for v in vals], dtype=np.dtype(npt).str.replace('i', 'u')).view(npt)


# ---------------------------------------------------------------------------
# 1. test/mpi/coll/allred.c -- closed forms of allred.c:451-593, run by
#    testlist.in:1-3 as (P=4,count=10), (P=7,count=10), (P=4,count=100).
# ---------------------------------------------------------------------------
ALLRED = 'test/mpi/coll/allred.c'


def allred_int_cases(dtname, npt, P, n, byte_only=False):
    i = np.arange(n)
    C = lambda v: int_cast(v, npt)          # noqa: E731
    const = lambda v: C([v] * n)            # noqa: E731
    src = lambda a, b: '%s:%d-%d (P=%d, count=%d)' % (ALLRED, a, b, P, n)  # noqa: E731
    if not byte_only:
        add('allred sum_test_1 %s' % dtname, dtname, 'SUM', [C(i)] * P, C(i * P),
            src(451, 457), 'in=i on every rank; sol=i*P')
        add('allred prod_test_1 %s' % dtname, dtname, 'PROD', [C(i)] * P, C(i ** P),
            src(459, 465), 'in=i; sol=i^P')
        add('allred max_test_1 %s' % dtname, dtname, 'MAX', [C(i + r) for r in range(P)],
            C(i + P - 1), src(467, 473), 'in=i+rank; sol=i+P-1')
        add('allred min_test_1 %s' % dtname, dtname, 'MIN', [C(i + r) for r in range(P)],
            C(i), src(475, 481), 'in=i+rank; sol=i')
        add('allred lor_test_1 %s' % dtname, dtname, 'LOR', [const(r & 1) for r in range(P)],
            const(int(P > 1)), src(490, 494), 'in=rank&1; sol=(P>1)')
        add('allred lor_test_2 %s' % dtname, dtname, 'LOR', [const(0)] * P, const(0),
            src(496, 500), 'in=0; sol=0')
        add('allred lxor_test_1 %s' % dtname, dtname, 'LXOR', [const(int(r == 1)) for r in range(P)],
            const(int(P > 1)), src(502, 506), 'in=(rank==1); sol=(P>1)')
        add('allred lxor_test_2 %s' % dtname, dtname, 'LXOR', [const(0)] * P, const(0),
            src(508, 512), 'in=0; sol=0')
        add('allred lxor_test_3 %s' % dtname, dtname, 'LXOR', [const(1)] * P, const(P & 1),
            src(514, 518), 'in=1; sol=P&1')
        add('allred land_test_1 %s' % dtname, dtname, 'LAND', [const(r & 1) for r in range(P)],
            const(0), src(520, 524), 'in=rank&1; sol=0')
        add('allred land_test_2 %s' % dtname, dtname, 'LAND', [const(1)] * P, const(1),
            src(526, 530), 'in=1; sol=1')
    add('allred bor_test_1 %s' % dtname, dtname, 'BOR', [const(r & 3) for r in range(P)],
        const(P - 1 if P < 3 else 3), src(532, 536), 'in=rank&3; sol=(P<3)?P-1:3')
    add('allred band_test_1 %s' % dtname, dtname, 'BAND',
        [C(i) if r == P - 1 else const(-1) for r in range(P)], C(i), src(556, 566),
        'last rank in=i, others ~0; sol=i')
    add('allred band_test_2 %s' % dtname, dtname, 'BAND',
        [C(i) if r == P - 1 else const(0) for r in range(P)], const(0), src(568, 578),
        'last rank in=i, others 0; sol=0')
    add('allred bxor_test_1 %s' % dtname, dtname, 'BXOR',
        [const(0xf0 * int(r == 1)) for r in range(P)], const(0xf0 * int(P > 1)),
        src(538, 542), 'in=(rank==1)*0xf0; sol=(P>1)*0xf0')
    add('allred bxor_test_2 %s' % dtname, dtname, 'BXOR', [const(0)] * P, const(0),
        src(544, 548), 'in=0; sol=0')
    add('allred bxor_test_3 %s' % dtname, dtname, 'BXOR', [const(-1)] * P,
        const(-1 if P & 1 else 0), src(550, 554), 'in=~0; sol=(P&1)?~0:0')


def allred_float_cases(dtname, npt, P, n):
    i = np.arange(n)
    F = lambda v: np.array(v, dtype=np.float64).astype(npt)  # noqa: E731
    src = lambda a, b: '%s:%d-%d (P=%d, count=%d)' % (ALLRED, a, b, P, n)  # noqa: E731
    add('allred sum_test_1 %s' % dtname, dtname, 'SUM', [F(i)] * P, F(i * P), src(451, 457),
        'in=i; sol=i*P')
    add('allred prod_test_1 %s' % dtname, dtname, 'PROD', [F(i)] * P,
        F([float(int(k) ** P) for k in i]), src(459, 465), 'in=i; sol=i^P')
    add('allred max_test_1 %s' % dtname, dtname, 'MAX', [F(i + r) for r in range(P)],
        F(i + P - 1), src(467, 473), 'in=i+rank; sol=i+P-1')
    add('allred min_test_1 %s' % dtname, dtname, 'MIN', [F(i + r) for r in range(P)], F(i),
        src(475, 481), 'in=i+rank; sol=i')


def allred_complex_cases(dtname, npt, P, n):
    i = np.arange(n)
    Z = lambda v: np.array(v, dtype=np.float64).astype(npt)  # noqa: E731
    note = (' (allred.c:648-657 iterates num_byte_types, so the reference only ever ran '
            'MPI_C_FLOAT_COMPLEX; the double case is the closed form it intended)'
            if 'DOUBLE' in dtname else '')
    add('allred sum_test_1 %s' % dtname, dtname, 'SUM', [Z(i)] * P, Z(i * P),
        '%s:451-457 (P=%d, count=%d)' % (ALLRED, P, n), 'in=(i,0); sol=(i*P,0)' + note)
    add('allred prod_test_1 %s' % dtname, dtname, 'PROD', [Z(i)] * P,
        Z([float(int(k) ** P) for k in i]), '%s:459-465 (P=%d, count=%d)' % (ALLRED, P, n),
        'in=(i,0); sol=(i^P,0)' + note)


def allred_pair_cases(dtname, P, n):
    dt = PAIR[dtname]
    i = np.arange(n)

    def mk(v, l):
        a = np.zeros(n, dt)
        a['v'] = v
        a['l'] = l
        return a
    add('allred maxloc_test %s' % dtname, dtname, 'MAXLOC', [mk(i + r, r) for r in range(P)],
        mk(i + P - 1, P - 1), '%s:580-586 (P=%d, count=%d)' % (ALLRED, P, n),
        'in=(i+rank, rank); sol=(i+P-1, P-1)')
    add('allred minloc_test %s' % dtname, dtname, 'MINLOC', [mk(i + r, r) for r in range(P)],
        mk(i, 0), '%s:588-593 (P=%d, count=%d)' % (ALLRED, P, n),
        'in=(i+rank, rank); sol=(i, 0)')


for P, n in ((4, 10), (7, 10), (4, 100)):
    for dtname, npt in INT_NP.items():
        allred_int_cases(dtname, npt, P, n)
    allred_int_cases('MPI_BYTE', '<u1', P, n, byte_only=True)
    for dtname, npt in (('MPI_FLOAT', np.float32), ('MPI_DOUBLE', np.float64)):
        allred_float_cases(dtname, npt, P, n)
    for dtname, npt in (('MPI_C_FLOAT_COMPLEX', np.complex64),
                        ('MPI_C_DOUBLE_COMPLEX', np.complex128)):
        allred_complex_cases(dtname, npt, P, n)
    # C_BOOL: the logical tests only (allred.c:660-672), bool stored as 1 byte
    i8 = lambda v: np.array([v] * n, np.uint8)  # noqa: E731
    for nm, op, ins, sol, lines in (
            ('lor_test_1', 'LOR', [i8(r & 1) for r in range(P)], i8(int(P > 1)), (490, 494)),
            ('lor_test_2', 'LOR', [i8(0)] * P, i8(0), (496, 500)),
            ('lxor_test_1', 'LXOR', [i8(int(r == 1)) for r in range(P)], i8(int(P > 1)), (502, 506)),
            ('lxor_test_2', 'LXOR', [i8(0)] * P, i8(0), (508, 512)),
            ('lxor_test_3', 'LXOR', [i8(1)] * P, i8(P & 1), (514, 518)),
            ('land_test_1', 'LAND', [i8(r & 1) for r in range(P)], i8(0), (520, 524)),
            ('land_test_2', 'LAND', [i8(1)] * P, i8(1), (526, 530))):
        add('allred %s MPI_C_BOOL' % nm, 'MPI_C_BOOL', op, ins, sol,
            '%s:%d-%d (P=%d, count=%d)' % (ALLRED, lines[0], lines[1], P, n), 'C_BOOL logical')
    for dtname in ('MPI_2INT', 'MPI_LONG_INT', 'MPI_SHORT_INT', 'MPI_FLOAT_INT', 'MPI_DOUBLE_INT'):
        allred_pair_cases(dtname, P, n)

# ---------------------------------------------------------------------------
# 2. test/mpi/coll/opmaxloc.c / opminloc.c -- 3-element KATs with ties:
#    equal values keep the MINIMUM loc (opmaxloc.c:20-23, the MPI-1 4.9.3 rule)
# ---------------------------------------------------------------------------
for P in (3, 4):
    for dtname, lines_max, lines_min in (
            ('MPI_2INT', (38, 78), (38, 70)), ('MPI_FLOAT_INT', (82, 122), (75, 107)),
            ('MPI_LONG_INT', (126, 166), (112, 144)), ('MPI_SHORT_INT', (170, 210), (149, 181)),
            ('MPI_DOUBLE_INT', (214, 260), (186, 218)),
            ('MPI_LONG_DOUBLE_INT', (264, 312), (222, 262))):
        dt = PAIR[dtname]
        ins = []
        for r in range(P):
            a = np.zeros(3, dt)
            a['v'] = [1, 0, r]
            a['l'] = r
            ins.append(a)
        sol = np.zeros(3, dt)
        sol['v'] = [1, 0, P - 1]
        sol['l'] = [0, 0, P - 1]
        add('opmaxloc %s' % dtname, dtname, 'MAXLOC', ins, sol,
            'test/mpi/coll/opmaxloc.c:%d-%d (P=%d)' % (lines_max[0], lines_max[1], P),
            'vals (1,0,rank) loc rank; ties -> loc 0; sol (1,0),(0,0),(P-1,P-1)',
            cmp='fields' if dtname == 'MPI_LONG_DOUBLE_INT' else None)
        ins = []
        for r in range(P):
            a = np.zeros(3, dt)
            a['v'] = [1, 0, r & 0x7f]
            a['l'] = r
            ins.append(a)
        sol = np.zeros(3, dt)
        sol['v'] = [1, 0, 0]
        sol['l'] = [0, 0, 0]
        add('opminloc %s' % dtname, dtname, 'MINLOC', ins, sol,
            'test/mpi/coll/opminloc.c:%d-%d (P=%d)' % (lines_min[0], lines_min[1], P),
            'vals (1,0,rank) loc rank; ties -> loc 0; sol (1,0),(0,0),(0,0)',
            cmp='fields' if dtname == 'MPI_LONG_DOUBLE_INT' else None)

# ---------------------------------------------------------------------------
# 3. test/mpi/coll/opsum.c:146-180 / opprod.c:147-210 -- MPI_DOUBLE_COMPLEX
# ---------------------------------------------------------------------------
for P in (2, 3, 4, 5):
    ins = [np.array([1 - 1j, 0j, complex(int(r > 0), -int(r > 0))], np.complex128)
           for r in range(P)]
    sol = np.array([complex(P, -P), 0j, complex(P - 1, 1 - P)], np.complex128)
    add('opsum MPI_DOUBLE_COMPLEX', 'MPI_DOUBLE_COMPLEX', 'SUM', ins, sol,
        'test/mpi/coll/opsum.c:146-180 (P=%d)' % P, 'sol (P,-P),(0,0),(P-1,1-P)')
    maxsize = min(P, 5)
    fact = [1, 1, 2, 6, 24, 120]
    ins = [np.array([complex(r if 0 < r < maxsize else 1, 0), 1j,
                     complex(int(r > 0), -int(r > 0))], np.complex128) for r in range(P)]
    rr, ii = {1: (0.0, 1.0), 2: (-1.0, 0.0), 3: (0.0, -1.0), 0: (1.0, 0.0)}[P % 4]
    closed = np.array([complex(fact[maxsize - 1], 0), complex(rr, ii), 0j], np.complex128)
    # The test compares with != (opprod.c:173-205), so -0 and +0 both pass;
    # the stored bits are those of the left fold with the plain finite-value
    # product (ac-bd, ad+bc), asserted equal in value to the closed form.
    sol = ins[0].copy()
    for r in range(1, P):
        x, y = sol, ins[r]
        sol = np.array([complex(x[k].real * y[k].real - x[k].imag * y[k].imag,
                                x[k].imag * y[k].real + x[k].real * y[k].imag)
                        for k in range(3)], np.complex128)
    assert np.all(sol == closed), (sol, closed)
    add('opprod MPI_DOUBLE_COMPLEX', 'MPI_DOUBLE_COMPLEX', 'PROD', ins, sol,
        'test/mpi/coll/opprod.c:147-210 (P=%d)' % P,
        'sol ((maxsize-1)!,0), i^P by P%4, (0,0)')

# ---------------------------------------------------------------------------
# 3b. test/mpi/coll/op{band,bor,bxor,land,lor,lxor,max,min,sum,prod}.c --
#     3-element KATs per type at the testlist sizes (testlist.in:113-127).
#     Inputs as the tests set them per rank; expected values are the tests'
#     own assertions (for the logical ops, which the tests only check for
#     truth, the exact 0/1 of op_fns.c:99-187).  MPI_LONG_DOUBLE legs are
#     left out: x87 arithmetic has no GPU path.
# ---------------------------------------------------------------------------
OPKAT_NP = {'MPI_CHAR': '<i1', 'MPI_SIGNED_CHAR': '<i1', 'MPI_UNSIGNED_CHAR': '<u1',
            'MPI_BYTE': '<u1', 'MPI_SHORT': '<i2', 'MPI_UNSIGNED_SHORT': '<u2',
            'MPI_UNSIGNED': '<u4', 'MPI_INT': '<i4', 'MPI_LONG': '<i8',
            'MPI_UNSIGNED_LONG': '<u8', 'MPI_LONG_LONG': '<i8'}


def opkat(test, line, op, dtname, per_rank, expected, Ps, rule):
    """per_rank(r, P) -> 3 values; expected(P) -> 3 values (C assignment
    semantics: values are cast to the type's width)"""
    npt = OPKAT_NP[dtname]
    for P in Ps:
        add('%s %s' % (test, dtname), dtname, op,
            [int_cast(per_rank(r, P), npt) for r in range(P)], int_cast(expected(P), npt),
            'test/mpi/coll/%s.c:%d (P=%d)' % (test, line, P), rule)


def pat(width, byte):
    """the tests' literal per width: 0xXX, 0xXXXX, or 0xXXXXXXXX for 4- and
    8-byte types (the 8-byte legs assign the same 32-bit literal)"""
    return int.from_bytes(bytes([byte]) * min(width, 4), 'little')


BITWISE_TYPES = {
    'opband': [('MPI_CHAR', 56), ('MPI_SIGNED_CHAR', 87), ('MPI_UNSIGNED_CHAR', 117),
               ('MPI_BYTE', 147), ('MPI_SHORT', 177), ('MPI_UNSIGNED_SHORT', 207),
               ('MPI_UNSIGNED', 237), ('MPI_LONG', 267), ('MPI_UNSIGNED_LONG', 297),
               ('MPI_LONG_LONG', 331)],
    'opbor': [('MPI_CHAR', 57), ('MPI_SIGNED_CHAR', 88), ('MPI_UNSIGNED_CHAR', 118),
              ('MPI_BYTE', 148), ('MPI_SHORT', 178), ('MPI_UNSIGNED_SHORT', 208),
              ('MPI_UNSIGNED', 238), ('MPI_INT', 268), ('MPI_LONG', 298),
              ('MPI_UNSIGNED_LONG', 328), ('MPI_LONG_LONG', 362)],
}
BITWISE_TYPES['opbxor'] = BITWISE_TYPES['opbor']
for dtname, line in BITWISE_TYPES['opband']:
    w = np.dtype(OPKAT_NP[dtname]).itemsize
    ones, f0 = pat(w, 0xff), pat(w, 0xf0)
    opkat('opband', line, 'BAND', dtname, lambda r, P: [ones, 0, ones if r > 0 else f0],
          lambda P: [ones, 0, f0], (4,), 'sol {ones, 0, 0xf0..}')
for dtname, line in BITWISE_TYPES['opbor']:
    w = np.dtype(OPKAT_NP[dtname]).itemsize
    ones, x3c, xc3 = pat(w, 0xff), pat(w, 0x3c), pat(w, 0xc3)
    opkat('opbor', line, 'BOR', dtname, lambda r, P: [ones, 0, x3c if r > 0 else xc3],
          lambda P: [ones, 0, ones], (4,), 'sol {ones, 0, ones}')
    opkat('opbxor', line, 'BXOR', dtname, lambda r, P: [ones, 0, x3c if r > 0 else xc3],
          lambda P: [ones if P % 2 else 0, 0, xc3 if P % 2 else ones], (4, 5),
          'sol {P%2 ? ones : 0, 0, P%2 ? 0xc3.. : ones}')

for test, op, lines, sol, Ps in (
        ('opland', 'LAND', (50, 81, 111, 145), lambda P: [1, 0, 0], (4,)),
        ('oplor', 'LOR', (67, 98, 128, 162), lambda P: [1, 0, 1], (4,)),
        ('oplxor', 'LXOR', (52, 83, 113, 147), lambda P: [P % 2, 0, (P - 1) % 2], (4, 5))):
    for dtname, line in zip(('MPI_CHAR', 'MPI_SIGNED_CHAR', 'MPI_UNSIGNED_CHAR', 'MPI_LONG_LONG'),
                            lines):
        opkat(test, line, op, dtname, lambda r, P: [1, 0, int(r > 0)], sol, Ps,
              'in {1, 0, rank>0}; 0/1 results (op_fns.c:99-187)')

for dtname, line in zip(('MPI_CHAR', 'MPI_SIGNED_CHAR', 'MPI_UNSIGNED_CHAR', 'MPI_LONG_LONG'),
                        (46, 72, 97, 158)):
    opkat('opmax', line, 'MAX', dtname, lambda r, P: [1, 0, r], lambda P: [1, 0, P - 1], (5,),
          'sol {1, 0, size-1}')
    opkat('opmin', line, 'MIN', dtname, lambda r, P: [1, 0, r & 0x7f], lambda P: [1, 0, 0], (4,),
          'sol {1, 0, 0}')

for dtname, line in zip(('MPI_CHAR', 'MPI_SIGNED_CHAR', 'MPI_UNSIGNED_CHAR', 'MPI_LONG_LONG'),
                        (70, 96, 121, 262)):
    opkat('opsum', line, 'SUM', dtname, lambda r, P: [1, 0, int(r > 0)],
          lambda P: [P, 0, P - 1], (4,), 'sol {size, 0, size-1}')

FACT = [1, 1, 2, 6, 24, 120]                                    # opprod.c:43
for dtname, line, gt in (('MPI_CHAR', 79, 1), ('MPI_SIGNED_CHAR', 106, 1),
                         ('MPI_UNSIGNED_CHAR', 132, 0), ('MPI_LONG_LONG', 314, 0)):
    opkat('opprod', line, 'PROD', dtname,
          lambda r, P: [r if 0 < r < min(P, 5) else 1, 0, int(r > gt)],
          lambda P: [FACT[min(P, 5) - 1], 0, 0], (5, 6), 'sol {(maxsize-1)!, 0, 0}')

# ---------------------------------------------------------------------------
# 4. test/mpi/impls/mpich/hip/stream_allred.hip:47-90 -- device buffers
# ---------------------------------------------------------------------------
P, N = 4, 10
add('stream_allred TEST 1 MPI_INT', 'MPI_INT', 'SUM', [np.full(N, r, '<i4') for r in range(P)],
    np.full(N, P * (P - 1) // 2, '<i4'), 'test/mpi/impls/mpich/hip/stream_allred.hip:47-70 (P=4)',
    'in=rank; sol=P(P-1)/2')
dt = PAIR['MPI_SHORT_INT']
ins = []
for r in range(P):
    a = np.zeros(N, dt)
    a['v'] = [0 if i % P == r else r + 1 for i in range(N)]
    a['l'] = r
    ins.append(a)
sol = np.zeros(N, dt)
sol['v'] = 0
sol['l'] = [i % P for i in range(N)]
add('stream_allred TEST 2 MPI_SHORT_INT', 'MPI_SHORT_INT', 'MINLOC', ins, sol,
    'test/mpi/impls/mpich/hip/stream_allred.hip:72-90 (P=4)', 'MINLOC result {0, i % size}')

# ---------------------------------------------------------------------------
# 5. Hand-derived two-operand edge vectors ("parity pinned by code reading
#    only": no reference test asserts these).  inputs = [a (inout), b (in)].
# ---------------------------------------------------------------------------
rng = np.random.default_rng(0x5EED0003)
f32 = np.float32
specials32 = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 1e-45, -1e-45,
                       3.4e38, -3.4e38, 1.17549435e-38], f32)
nanb = np.frombuffer(np.array([0x7fc00001, 0xffc12345], '<u4').tobytes(), f32)
sp = np.concatenate([specials32, nanb])
a = np.repeat(sp, len(sp))
b = np.tile(sp, len(sp))
with np.errstate(all='ignore'):
    add('edge MAX fp32 specials', 'MPI_FLOAT', 'MAX', [a, b], np.where(a > b, a, b),
        'src/mpi/coll/op/op_fns.c:257-271 + src/mpl/include/mpl_base.h:105',
        'MPL_MAX select (a>b)?a:b: any NaN -> b bit-exact; MAX(+0,-0)=-0, MAX(-0,+0)=+0')
    add('edge MIN fp32 specials', 'MPI_FLOAT', 'MIN', [a, b], np.where(a < b, a, b),
        'src/mpi/coll/op/op_fns.c:275-289 + mpl_base.h:106', 'MPL_MIN select (a<b)?a:b')
    add('edge SUM fp32 specials', 'MPI_FLOAT', 'SUM', [a, b], (a + b).astype(f32),
        'op_fns.c:19-55', 'IEEE fp32 add (NaN payload unpinned)', nan_equiv=True)
    add('edge PROD fp32 specials', 'MPI_FLOAT', 'PROD', [a, b], (a * b).astype(f32),
        'op_fns.c:61-91', 'IEEE fp32 mul (NaN payload unpinned)', nan_equiv=True)
    a64, b64 = a.astype(np.float64), b.astype(np.float64)
    add('edge MAX fp64 specials', 'MPI_DOUBLE', 'MAX', [a64, b64], np.where(a64 > b64, a64, b64),
        'op_fns.c:257-271', 'MPL_MAX select')
    add('edge MIN fp64 specials', 'MPI_DOUBLE', 'MIN', [a64, b64], np.where(a64 < b64, a64, b64),
        'op_fns.c:275-289', 'MPL_MIN select')
    # denormal arithmetic is kept (no flush) on the CPU path
    d = np.array([1e-45, 1e-40, -1e-39, 5.9e-39], f32)
    add('edge SUM fp32 denormals', 'MPI_FLOAT', 'SUM', [d, d[::-1].copy()], d + d[::-1],
        'op_fns.c:19-55', 'subnormal sums are not flushed')

# integer wraparound (mpir_op_util.h:51 casts the promoted result back)
add('edge SUM int32 wrap', 'MPI_INT', 'SUM',
    [np.array([2**31 - 1, -2**31, -1, 123], '<i4'), np.array([1, -1, 1, -124], '<i4')],
    np.array([-2**31, 2**31 - 1, 0, -1], '<i4'), 'mpir_op_util.h:46-53', 'two\'s complement wrap')
add('edge PROD int8 wrap', 'MPI_SIGNED_CHAR', 'PROD',
    [np.array([100, -128, 16, 7], '<i1'), np.array([3, -1, 16, -19], '<i1')],
    int_cast([300, 128, 256, -133], '<i1'), 'mpir_op_util.h:46-53', 'product mod 256')
add('edge PROD uint16 wrap', 'MPI_UNSIGNED_SHORT', 'PROD',
    [np.array([65535, 256, 3, 0], '<u2'), np.array([65535, 256, 21845, 9], '<u2')],
    int_cast([65535 * 65535, 65536, 65535, 0], '<u2'), 'mpir_op_util.h:46-53', 'product mod 65536')
add('edge SUM uint64 wrap', 'MPI_UINT64_T', 'SUM',
    [np.array([2**64 - 1, 2**63], '<u8'), np.array([2, 2**63], '<u8')],
    np.array([1, 0], '<u8'), 'mpir_op_util.h:46-53', 'sum mod 2^64')
la = np.array([0, 5, -1, 0, 7, 0], '<i4')
lb = np.array([0, 0, 3, 9, -2, 0], '<i4')
add('edge LAND int32 values', 'MPI_INT', 'LAND', [la, lb], ((la != 0) & (lb != 0)).astype('<i4'),
    'op_fns.c:95-119', 'a&&b yields 0/1')
add('edge LOR int32 values', 'MPI_INT', 'LOR', [la, lb], ((la != 0) | (lb != 0)).astype('<i4'),
    'op_fns.c:125-149', 'a||b yields 0/1')
add('edge LXOR int32 values', 'MPI_INT', 'LXOR', [la, lb], ((la != 0) ^ (lb != 0)).astype('<i4'),
    'op_fns.c:155-187', '(a&&!b)||(!a&&b) yields 0/1')
# Fortran LOGICAL (4 bytes) with the default .TRUE.=1/.FALSE.=0 (typeutil.c:502-510)
add('edge LXOR LOGICAL', 'MPI_LOGICAL', 'LXOR', [la, lb], ((la != 0) ^ (lb != 0)).astype('<i4'),
    'op_fns.c:155-187 + mpii_fortlogical.h:15,28', 'FROM_FLOG(x)=(x!=false); TO_FLOG')
for nm, op in (('BAND', np.bitwise_and), ('BOR', np.bitwise_or), ('BXOR', np.bitwise_xor)):
    x = rng.integers(-2**63, 2**63, 64, dtype=np.int64)
    y = rng.integers(-2**63, 2**63, 64, dtype=np.int64)
    add('edge %s long' % nm, 'MPI_LONG', nm, [x, y], op(x, y), 'op_fns.c:195-253', 'bitwise')
xs = rng.integers(-2**31, 2**31, 64, dtype=np.int64).astype('<i4')
ys = rng.integers(-2**31, 2**31, 64, dtype=np.int64).astype('<i4')
add('edge MAX int32 random', 'MPI_INT', 'MAX', [xs, ys], np.maximum(xs, ys), 'op_fns.c:257-271', 'max')
add('edge MIN uint32 random', 'MPI_UNSIGNED', 'MIN', [xs.view('<u4'), ys.view('<u4')],
    np.minimum(xs.view('<u4'), ys.view('<u4')), 'op_fns.c:275-289', 'unsigned compare')

# MAXLOC/MINLOC: NaN values leave inout unchanged; ties keep min loc
fi = PAIR['MPI_FLOAT_INT']
va = np.array([1.0, 2.0, np.nan, 3.0, np.nan, -0.0, 5.0], f32)
vb = np.array([2.0, 2.0, 1.0, np.nan, np.nan, 0.0, 5.0], f32)
A = np.zeros(7, fi)
B = np.zeros(7, fi)
A['v'], A['l'] = va, [7, 3, 1, 1, 1, 4, -5]
B['v'], B['l'] = vb, [9, 2, 2, 2, 2, 9, -6]
E = A.copy()
for k in range(7):
    if va[k] < vb[k]:
        E[k] = B[k]
    elif va[k] <= vb[k]:
        E['l'][k] = min(A['l'][k], B['l'][k])
add('edge MAXLOC FLOAT_INT nan/ties', 'MPI_FLOAT_INT', 'MAXLOC', [A, B], E,
    'op_fns.c:299-352', 'a<b take b; a<=b loc=min; NaN -> unchanged')
E = A.copy()
for k in range(7):
    if va[k] > vb[k]:
        E[k] = B[k]
    elif va[k] >= vb[k]:
        E['l'][k] = min(A['l'][k], B['l'][k])
add('edge MINLOC FLOAT_INT nan/ties', 'MPI_FLOAT_INT', 'MINLOC', [A, B], E,
    'op_fns.c:367-435', 'a>b take b; a>=b loc=min')
r2 = PAIR['MPI_2REAL']
A2 = np.zeros(5, r2)
B2 = np.zeros(5, r2)
A2['v'], A2['l'] = [1, 2, 3, 4, 5], [0.5, 2.0, 1.0, 1.0, 9.0]
B2['v'], B2['l'] = [1, 1, 4, 4, 5], [0.25, 7.0, 0.0, -1.0, np.nan]
E2 = A2.copy()
for k in range(5):
    if A2['v'][k] < B2['v'][k]:
        E2[k] = B2[k]
    elif A2['v'][k] <= B2['v'][k]:
        E2['l'][k] = A2['l'][k] if A2['l'][k] < B2['l'][k] else B2['l'][k]
add('edge MAXLOC 2REAL', 'MPI_2REAL', 'MAXLOC', [A2, B2], E2, 'op_fns.c:303-330',
    'builtin pair: loc is the value type, MPL_MIN select on loc')

# fp16 (MPIX_C_FLOAT16): native _Float16 semantics, each op correctly rounded
# (SURVEY.md Appendix A.5 -- unpinned by reference tests).  numpy's float16
# arithmetic is an independent correctly-rounded implementation.
h = np.array([0.0, -0.0, 1.0, -2.5, 65504.0, 6.1e-5, 5.96e-8, np.inf, 1.0009765625,
              0.33325195, 1024.0, -7.0], np.float16)
ha = np.repeat(h, len(h))
hb = np.tile(h, len(h))
with np.errstate(all='ignore'):
    add('edge SUM fp16', 'MPIX_C_FLOAT16', 'SUM', [ha, hb], (ha + hb).astype(np.float16),
        'mpir_op_util.h:211-217 (FLOAT16 in FLOATING_POINT with _Float16)', 'RNE fp16 add',
        nan_equiv=True)
    add('edge PROD fp16', 'MPIX_C_FLOAT16', 'PROD', [ha, hb], (ha * hb).astype(np.float16),
        'mpir_op_util.h:211-217', 'RNE fp16 mul', nan_equiv=True)
    add('edge MAX fp16', 'MPIX_C_FLOAT16', 'MAX', [ha, hb], np.where(ha > hb, ha, hb),
        'op_fns.c:257-271', 'select')

# bf16 SUM: fp32 add then (u>>16) + ((u & 0x8000) ? 1 : 0)   (op_fns.c:459-493)
bfa = rng.integers(0, 1 << 16, 256, dtype=np.uint32).astype('<u2')
bfb = rng.integers(0, 1 << 16, 256, dtype=np.uint32).astype('<u2')
fa = (bfa.astype(np.uint32) << 16).view(np.float32)
fb = (bfb.astype(np.uint32) << 16).view(np.float32)
keep = ~(np.isnan(fa) | np.isnan(fb))
bfa, bfb, fa, fb = bfa[keep], bfb[keep], fa[keep], fb[keep]
with np.errstate(all='ignore'):
    s = (fa + fb).astype(np.float32).view(np.uint32)
bfo = (((s >> 16) + ((s & 0x8000) != 0)) & 0xffff).astype('<u2')
okay = ~np.isnan((s & 0xffffffff).view(np.float32))
add('edge SUM bf16 ties-away', 'MPIX_BFLOAT16', 'SUM', [bfa[okay], bfb[okay]], bfo[okay],
    'src/mpi/coll/op/op_fns.c:459-493', 'fp32 add, store rounds half away on the magnitude bits')

# C99 Annex G complex multiply (float _Complex, C-native group, op_fns.c:61-71)


def mulsc3(a, b, c, d, T):
    """restated from C99 Annex G.5.1 / libgcc __mulXc3: (a+ib)(c+id)"""
    a, b, c, d = T(a), T(b), T(c), T(d)
    with np.errstate(all='ignore'):
        ac, bd, ad, bc = T(a * c), T(b * d), T(a * d), T(b * c)
        x, y = T(ac - bd), T(ad + bc)
        if np.isnan(x) and np.isnan(y):
            recalc = False
            if np.isinf(a) or np.isinf(b):
                a = T(np.copysign(1.0 if np.isinf(a) else 0.0, a))
                b = T(np.copysign(1.0 if np.isinf(b) else 0.0, b))
                if np.isnan(c):
                    c = T(np.copysign(0.0, c))
                if np.isnan(d):
                    d = T(np.copysign(0.0, d))
                recalc = True
            if np.isinf(c) or np.isinf(d):
                c = T(np.copysign(1.0 if np.isinf(c) else 0.0, c))
                d = T(np.copysign(1.0 if np.isinf(d) else 0.0, d))
                if np.isnan(a):
                    a = T(np.copysign(0.0, a))
                if np.isnan(b):
                    b = T(np.copysign(0.0, b))
                recalc = True
            if not recalc and (np.isinf(ac) or np.isinf(bd) or np.isinf(ad) or np.isinf(bc)):
                if np.isnan(a):
                    a = T(np.copysign(0.0, a))
                if np.isnan(b):
                    b = T(np.copysign(0.0, b))
                if np.isnan(c):
                    c = T(np.copysign(0.0, c))
                if np.isnan(d):
                    d = T(np.copysign(0.0, d))
                recalc = True
            if recalc:
                x = T(T(np.inf) * T(T(a * c) - T(b * d)))
                y = T(T(np.inf) * T(T(a * d) + T(b * c)))
    return x, y


cz = [(1.5, -2.0), (np.inf, np.nan), (np.nan, np.inf), (np.inf, 0.0), (0.0, np.inf),
      (np.nan, np.nan), (3e38, 3e38), (-0.0, 0.0), (1e-30, 1e30), (2.0, 0.5)]
for T, cdt, dtn in ((np.float32, np.complex64, 'MPI_C_FLOAT_COMPLEX'),
                    (np.float64, np.complex128, 'MPI_C_DOUBLE_COMPLEX')):
    za, zb, ze = [], [], []
    for (ar, ai) in cz:
        for (br, bi) in cz:
            x, y = mulsc3(ar, ai, br, bi, T)
            za.append(complex(ar, ai))
            zb.append(complex(br, bi))
            ze.append((x, y))
    A = np.array(za, cdt)
    B = np.array(zb, cdt)
    Eo = np.zeros(len(ze), cdt)
    Eo.real = [e[0] for e in ze]
    Eo.imag = [e[1] for e in ze]
    add('edge PROD %s Annex G' % dtn, dtn, 'PROD', [A, B], Eo, 'op_fns.c:61-71 (C-native complex *)',
        'C99 Annex G multiply incl. NaN recovery; a = inout, b = in', nan_equiv=True)

# REPLACE / NO_OP (op_fns.c:439-457)
ra = np.arange(8, dtype='<i4')
rb = np.arange(100, 108, dtype='<i4')
add('edge REPLACE int', 'MPI_INT', 'REPLACE', [ra, rb], rb, 'op_fns.c:445-457', 'inout = in')
add('edge NO_OP int', 'MPI_INT', 'NO_OP', [ra, rb], ra, 'op_fns.c:439-443', 'inout unchanged')

# MPIX_EQUAL (src/mpi/coll/op/opequal.c:20-35): MPI_BYTE buffers led by a
# uint64 is_equal flag; inout's flag drops to 0 unless both flags are 1 and
# the payloads match byte for byte.  (Reached only through
# MPIR_Reduce_equal / MPIR_Allreduce_equal, opequal.c:37-102.)
def eq_buf(flag, payload):
    return np.concatenate([np.array([flag], '<u8').view(np.uint8), np.array(payload, np.uint8)])


for nm, a_, b_, e_ in (
        ('equal payloads', eq_buf(1, [1, 2, 3, 4, 5]), eq_buf(1, [1, 2, 3, 4, 5]), 1),
        ('one byte differs', eq_buf(1, [1, 2, 3, 4, 5]), eq_buf(1, [1, 2, 3, 9, 5]), 0),
        ('in flag 0', eq_buf(1, [7] * 20), eq_buf(0, [7] * 20), 0),
        ('inout flag 0', eq_buf(0, [7] * 20), eq_buf(1, [7] * 20), 0),
        ('flag 2 is not 1', eq_buf(1, [7] * 3), eq_buf(2, [7] * 3), 0),
        ('header only', eq_buf(1, []), eq_buf(1, []), 1)):
    exp = a_.copy()
    exp[:8] = np.array([e_], '<u8').view(np.uint8)
    add('edge EQUAL %s' % nm, 'MPI_BYTE', 'EQUAL', [a_, b_], exp, 'src/mpi/coll/op/opequal.c:20-35',
        'is_equal = (in.flag == 1 && inout.flag == 1 && payloads equal) ? inout.flag : 0')

# ---------------------------------------------------------------------------
# Rule-based KATs too large to store as bytes: the tests build the arrays
# from these rules (cited) and check the stated closed form.
# ---------------------------------------------------------------------------
rule_kats = [
    dict(name='reduce_local MPI_INT SUM', source='test/mpi/coll/reduce_local.c:55-67',
         rule='counts 0,1,2,4,...,32768; in[i]=inout[i]=i; expect inout[i]=2i. The reference '
              'nests the inout check under the in check (:62-65) so a wrong sum is never '
              'detected; this port checks inout unconditionally.'),
    dict(name='redscatblk3 MPI_INT SUM', source='test/mpi/coll/redscatblk3.c:36-78',
         rule='mycount=(1024*1024)/P; rank r block i holds r+i; rank r result = P*r + P(P-1)/2'),
    dict(name='allred_float association', source='test/mpi/coll/allred_float.c:21-90',
         rule='every rank must get bit-identical results (memcmp); checked by running the same '
              'schedule on every rank'),
]

with open(os.path.join(HERE, 'kat_manifest.json'), 'w') as f:
    json.dump(dict(generator='tests/golden/make_golden.py', cases=cases, rule_kats=rule_kats),
              f, indent=1)
np.savez_compressed(os.path.join(HERE, 'kat_vectors.npz'), **arrays)
print('wrote %d cases (%d bytes of vectors)' % (len(cases), sum(v.nbytes for v in arrays.values())))
