#!/usr/bin/env python3
"""Per-process kernel-time split probe.

One process = one sample.  In it, on 1 GiB fp32 operands:
  contig  the shipped MPIX_Reduce_local_async kernel (inout += in)
  triad   the STREAM triad of libmpix_bench on three 1 GiB arrays
  slab    the shipped kernel on both operands carved from ONE 2 GiB hipMalloc
each timed with HIP events on the launch stream (median of `batches`
batches of `reps` launches).  If a slow process is slow on the triad too, the
split is a property of the process's memory / device state, not of the
combine kernel.  One JSON line per process on stdout.
"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

N = 1 << 28


def timed(fn, s, reps=20, batches=5):
    for _ in range(3):
        fn()
    out = []
    for _ in range(batches):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        b.synchronize()
        out.append(a.elapsed_time(b) / reps)
    out.sort()
    return round(out[len(out) // 2], 4), round(out[0], 4)


def offsets(B, s):
    """both operands (and the triad's three arrays) carved from ONE 3 GiB
    allocation: inout at 0, in at 1 GiB + off"""
    slab = torch.empty(3 * N + (1 << 28) // 4, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    torch.cuda.synchronize()
    out = {}
    for off in (0, 4096, 65536, 2 << 20, (2 << 20) + 4096, (96 << 20) + 12288,
                (512 << 20) + 4096):
        e = N + off // 4
        out['slab_in_at_1GiB+%d' % off], _ = timed(
            lambda: redop.check(redop.reduce_local_async(slab[e:e + N], slab[:N], N, H.MPI_FLOAT,
                                                         H.MPI_SUM, s)), s, reps=10, batches=3)
    out['slab_triad'], _ = timed(
        lambda: B.mpix_bench_triad(slab.data_ptr(), slab[N:].data_ptr(), slab[2 * N:].data_ptr(),
                                   ctypes.c_float(0.5), N, s.cuda_stream), s, reps=10, batches=3)
    del slab
    torch.cuda.empty_cache()
    x = torch.empty(N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    y = torch.empty(N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    z = torch.empty(N, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    out['separate_contig'], _ = timed(
        lambda: redop.check(redop.reduce_local_async(y, x, N, H.MPI_FLOAT, H.MPI_SUM, s)), s,
        reps=10, batches=3)
    out['separate_triad'], _ = timed(
        lambda: B.mpix_bench_triad(z.data_ptr(), x.data_ptr(), y.data_ptr(), ctypes.c_float(0.5),
                                   N, s.cuda_stream), s, reps=10, batches=3)
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else ''
    assert redop.lib().MPIX_Redop_init() == 0
    B = ctypes.CDLL(os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so'))
    B.mpix_bench_triad.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p]
    s = torch.cuda.current_stream()
    if tag.startswith('offsets'):
        print(json.dumps(dict(tag=tag, pid=os.getpid(), **offsets(B, s))), flush=True)
        return
    t0 = time.time()
    x = torch.empty(N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    y = torch.empty(N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    z = torch.empty(N, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    rec = dict(tag=tag, pid=os.getpid())
    rec['contig_ms'], rec['contig_min_ms'] = timed(
        lambda: redop.check(redop.reduce_local_async(y, x, N, H.MPI_FLOAT, H.MPI_SUM, s)), s)
    rec['triad_ms'], rec['triad_min_ms'] = timed(
        lambda: B.mpix_bench_triad(z.data_ptr(), x.data_ptr(), y.data_ptr(), ctypes.c_float(0.5),
                                   N, s.cuda_stream), s)
    rec['contig2_ms'], _ = timed(
        lambda: redop.check(redop.reduce_local_async(y, x, N, H.MPI_FLOAT, H.MPI_SUM, s)), s)
    del x, y, z
    torch.cuda.empty_cache()
    slab = torch.empty(2 * N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    torch.cuda.synchronize()
    rec['slab_ms'], _ = timed(
        lambda: redop.check(redop.reduce_local_async(slab[N:], slab[:N], N, H.MPI_FLOAT,
                                                     H.MPI_SUM, s)), s)
    rec['GBs_contig'] = round(3 * N * 4 / (rec['contig_ms'] * 1e6), 1)
    rec['GBs_triad'] = round(3 * N * 4 / (rec['triad_ms'] * 1e6), 1)
    rec['ratio'] = round(rec['triad_ms'] / rec['contig_ms'], 4)
    rec['wall_s'] = round(time.time() - t0, 2)
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
