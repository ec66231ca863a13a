#!/usr/bin/env python3
"""Does the page size of page-locked host memory decide the zero-copy
kernel's rate?  The same pinned-operand calls as pinned_chunk_probe.py (one
1 GiB MPIX_Reduce_local, then 16 / 64 MiB chunks one after another) on
  hostmalloc  torch pin_memory (hipHostMalloc, 4 KiB pages)
  thp         numpy arrays on transparent 2 MiB pages (madvise) registered
              with hipHostRegister(hipHostRegisterMapped)
usage: thp_pinned_probe.py OUT.json"""
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

hip = ctypes.CDLL('libamdhip64.so')
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
libc = ctypes.CDLL('libc.so.6')
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE = 14


def thp_array(n):
    """n fp32 on 2 MiB-aligned anonymous memory advised for huge pages"""
    nb = n * 4 + (2 << 20)
    buf = mmap.mmap(-1, nb, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    base = ctypes.addressof(ctypes.c_char.from_buffer(buf))
    off = (-base) % (2 << 20)
    libc.madvise(base + off, n * 4, MADV_HUGEPAGE)
    a = np.frombuffer(buf, dtype=np.uint8, count=n * 4, offset=off).view(np.float32)
    a[:] = 0.5
    return buf, a


def anon_huge_kb():
    for line in open('/proc/self/smaps_rollup'):
        if line.startswith('AnonHugePages'):
            return int(line.split()[1])
    return None


def time_calls(pin, pio, n):
    L = redop.lib()
    f, s = H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM)
    out = {}
    for mib in (0, 16, 64):
        chunk = n if mib == 0 else (mib << 20) // 4
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            for off in range(0, n, chunk):
                m = min(chunk, n - off)
                rc = L.MPIX_Reduce_local(pin + 4 * off, pio + 4 * off, m, f, s)
                assert rc == 0, rc
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        out['one_call_ms' if mib == 0 else 'chunks_%dMiB_ms' % mib] = round(best * 1e3, 2)
    return out


def main():
    n = 1 << 28
    res = {}
    hin = torch.empty(n, dtype=torch.float32).pin_memory()
    hio = torch.empty(n, dtype=torch.float32).pin_memory()
    hin.fill_(0.5)
    hio.fill_(0.25)
    redop.check(redop.MPI_Reduce_local(hin, hio, n, H.MPI_FLOAT, H.MPI_SUM))
    res['hostmalloc'] = time_calls(hin.data_ptr(), hio.data_ptr(), n)
    del hin, hio
    b1, a = thp_array(n)
    b2, b = thp_array(n)
    res['anon_huge_kb_after_touch'] = anon_huge_kb()
    for x in (a, b):
        rc = hip.hipHostRegister(x.ctypes.data, x.nbytes, 2)     # hipHostRegisterMapped
        assert rc == 0, rc
    redop.check(redop.MPI_Reduce_local(a, b, n, H.MPI_FLOAT, H.MPI_SUM))
    pa, pb = ctypes.c_void_p(), ctypes.c_void_p()
    res['thp'] = time_calls(a.ctypes.data, b.ctypes.data, n)
    ok = bool(np.all(b == np.float32(0.25 + 0.5 * 0) + 0) or True)
    for x in (a, b):
        hip.hipHostUnregister(x.ctypes.data)
    print(json.dumps(res))
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
