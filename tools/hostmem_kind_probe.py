#!/usr/bin/env python3
"""Zero-copy combine rate by the kind of page-locked host memory: 1 GiB fp32
SUM operands allocated with hipHostMalloc flags Default / Coherent /
NonCoherent, and `in` write-combined (the CPU only writes it, the GPU only
reads it); one synchronous MPIX_Reduce_local over the whole buffers and the
same bytes as 16 / 64 MiB calls.  Also the host memcpy rate into each kind
(what the pageable path's copy-in pays) and out of it (its copy-out).
usage: hostmem_kind_probe.py OUT.json"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime: torch's)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

hip = ctypes.CDLL('libamdhip64.so')
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]
KINDS = {'default': 0x0, 'coherent': 0x40000000, 'noncoherent': 0x80000000,
         'writecombined': 0x4}


def alloc(nbytes, flags):
    p = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(p), nbytes, flags)
    if rc:
        return None
    return p.value


def as_np(p, n):
    return np.ctypeslib.as_array((ctypes.c_float * n).from_address(p))


def calls(pin, pio, n):
    L = redop.lib()
    f, s = H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM)
    out = {}
    for mib in (0, 16, 64):
        chunk = n if mib == 0 else (mib << 20) // 4
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            for off in range(0, n, chunk):
                rc = L.MPIX_Reduce_local(pin + 4 * off, pio + 4 * off, min(chunk, n - off), f, s)
                assert rc == 0, rc
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        out['one_call_ms' if mib == 0 else 'chunks_%dMiB_ms' % mib] = round(best * 1e3, 2)
    return out


def memcpy_rate(dst, src):
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        np.copyto(dst, src)
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return round(dst.nbytes / best / 1e9, 2)


def main():
    n = 1 << 28
    src = np.random.default_rng(3).random(n, dtype=np.float32)
    res = {}
    for kin, kio in (('default', 'default'), ('coherent', 'coherent'),
                     ('noncoherent', 'noncoherent'), ('writecombined', 'default'),
                     ('writecombined', 'noncoherent')):
        pi, po = alloc(4 * n, KINDS[kin]), alloc(4 * n, KINDS[kio])
        if not pi or not po:
            res['%s/%s' % (kin, kio)] = 'alloc failed'
            continue
        ai, ao = as_np(pi, n), as_np(po, n)
        r = dict(memcpy_into_in_GBs=memcpy_rate(ai, src), memcpy_into_inout_GBs=memcpy_rate(ao, src))
        r['memcpy_out_of_inout_GBs'] = memcpy_rate(src.copy(), ao)
        r.update(calls(pi, po, n))
        res['%s/%s' % (kin, kio)] = r
        hip.hipHostFree(pi)
        hip.hipHostFree(po)
        print(kin, kio, r, flush=True)
    print(json.dumps(res))
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
