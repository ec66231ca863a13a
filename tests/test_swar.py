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
