#!/usr/bin/env python3
"""Placement probe for the 1 GiB fp32 SUM kernel: is the 0.50 / 0.52 ms split
a property of where the two operands sit?  (a) fresh pairs of separate 1 GiB
allocations, (b) both operands inside one allocation at several relative
byte offsets.  Kernel time per launch from HIP events; JSON lines to stdout."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

N = 1 << 28


def kernel_ms(inb, io, reps=30):
    s = torch.cuda.current_stream()
    for _ in range(3):
        redop.check(redop.reduce_local_async(inb, io, N, H.MPI_FLOAT, H.MPI_SUM, s))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        redop.check(redop.reduce_local_async(inb, io, N, H.MPI_FLOAT, H.MPI_SUM, s))
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    assert redop.lib().MPIX_Redop_init() == 0
    for k in range(6):
        x = torch.zeros(N, dtype=torch.float32, device='cuda')
        y = torch.zeros(N, dtype=torch.float32, device='cuda')
        torch.cuda.synchronize()
        print(json.dumps(dict(kind='separate', trial=k, delta=y.data_ptr() - x.data_ptr(),
                              ms=round(kernel_ms(y, x), 4))), flush=True)
        del x, y
        torch.cuda.empty_cache()
    pad = 1 << 30
    big = torch.zeros(2 * N + pad // 4, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    for off in (0, 256, 4096, 65536, 1 << 20, 2 << 20, 3 << 20, 64 << 20, 256 << 20, 512 << 20):
        e = N + off // 4
        print(json.dumps(dict(kind='one_alloc', offset_bytes=off,
                              ms=round(kernel_ms(big[e:e + N], big[:N]), 4))), flush=True)


if __name__ == '__main__':
    main()
