#!/usr/bin/env python3
"""The x87 / binary128 rows of the bench line (the soft
complex products are the slowest rows) for ONE build of libmpix_redop.so, at
1 GiB per operand on normal values (bench.fill_soft_slots, every op on the
same operands), kernel only by HIP events, median of 3 batches of 3; the
fp32 SUM row of the same process beside them.  One JSON line.

usage: soft_rows.py LIBPATH LABEL [TYPE:OP ...]   (run alternately for two
builds; TYPE:OP pairs, e.g. MPI_COMPLEX32:MPI_PROD, restrict the rows -- a
profiler pass over one kernel)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
import bench  # noqa: E402

# the build under test, bound here (an older build lacks later symbols)
L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
L.MPIX_Reduce_local_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ssize_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.MPIX_Datatype_extent.argtypes = [ctypes.c_int]
L.MPIX_Datatype_extent.restype = ctypes.c_ssize_t


def call(b, a, n, dt, op, s):
    rc = L.MPIX_Reduce_local_async(b.data_ptr(), a.data_ptr(), n, H.as_c_int(dt), H.as_c_int(op),
                                   s.cuda_stream)
    if rc:
        raise RuntimeError('MPIX_Reduce_local_async: %d' % rc)


def main():
    nbytes = 1 << 30
    dev = torch.device('cuda', 0)
    a8 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b8 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    rows = []
    fa, fb = a8.view(torch.float32), b8.view(torch.float32)
    bench.fill_uniform(fa, 1)
    bench.fill_uniform(fb, 2)
    torch.cuda.synchronize()
    n = nbytes // 4
    call(fb, fa, n, H.MPI_FLOAT, H.MPI_SUM, s)
    _, med, _ = bench.event_time_per_launch(lambda: call(fb, fa, n, H.MPI_FLOAT, H.MPI_SUM, s), 3, s,
                                            rounds=3)
    rows.append(dict(type='MPI_FLOAT', op='MPI_SUM', GBs=round(3 * nbytes / (med * 1e-3) / 1e9, 1)))
    only = set(sys.argv[3:])
    zero_im = os.environ.get('SOFT_ROWS_ZERO_IM') == '1'     # complex rows on real values
    for tn in ('MPI_LONG_DOUBLE', 'MPI_REAL16', 'MPI_C_LONG_DOUBLE_COMPLEX', 'MPI_COMPLEX32'):
        enc = 'x87' if 'LONG_DOUBLE' in tn else 'binary128'
        bench.fill_soft_slots(b8, enc, 0x5EED0004)
        dt = getattr(H, tn)
        ext = L.MPIX_Datatype_extent(H.as_c_int(dt))
        m = nbytes // ext
        for on in ('MPI_SUM', 'MPI_PROD'):
            if only and '%s:%s' % (tn, on) not in only:
                continue
            op = getattr(H, on)
            bench.fill_soft_slots(a8, enc, 0x5EED0003)
            if zero_im and 'COMPLEX' in tn:
                # real values stored as complex: every product has a zero
                # operand, which the fast paths decline (the fixup path's rate)
                a8.view(-1, 32)[:, 16:] = 0
                b8.view(-1, 32)[:, 16:] = 0
            torch.cuda.synchronize()
            call(b8, a8, m, dt, op, s)
            _, med, _ = bench.event_time_per_launch(lambda: call(b8, a8, m, dt, op, s), 3, s,
                                                    rounds=3)
            rows.append(dict(type=tn, op=on, GBs=round(3 * m * ext / (med * 1e-3) / 1e9, 1)))
    print(json.dumps(dict(label=sys.argv[2], lib=os.path.basename(sys.argv[1]), zero_im=zero_im,
                          rows=rows)))


if __name__ == '__main__':
    main()
