#!/usr/bin/env python3
"""Per-call latency of the synchronous MPIX_Reduce_local (fp32 SUM) by size,
for device-resident and host-resident (pinned / pageable) operands.
Host wall time per call, median over repetitions.  JSON to stdout."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402


def timeit(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device('cuda', 0)
    out = dict(device=[], pinned=[], pageable=[], chunk=os.environ.get('MPIX_REDOP_STAGE_CHUNK'),
               sync=os.environ.get('MPIX_REDOP_SYNC', 'spin'))
    counts = os.environ.get('PERF_COUNTS')
    counts = [int(x) for x in counts.split(',')] if counts else \
        (1, 16, 256, 4096, 4097, 16384, 65536, 262144, 1 << 20, 1 << 24, 1 << 28)
    out.update(small_bytes=os.environ.get('MPIX_REDOP_SMALL_BYTES'),
               bounce_bytes=os.environ.get('MPIX_REDOP_BOUNCE_BYTES'))
    for n in counts:
        a = torch.zeros(n, dtype=torch.float32, device=dev)
        b = torch.zeros(n, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        reps = 200 if n <= (1 << 20) else 20
        t = timeit(lambda: redop.check(redop.MPI_Reduce_local(b, a, n, H.MPI_FLOAT, H.MPI_SUM)), reps)
        out['device'].append(dict(count=n, us=round(t * 1e6, 2), GiBs=round(12 * n / t / 2**30, 2)))
        del a, b
        for kind in ('pinned', 'pageable'):
            if kind == 'pinned':
                ha = torch.zeros(n, dtype=torch.float32).pin_memory()
                hb = torch.zeros(n, dtype=torch.float32).pin_memory()
            else:
                ha = np.zeros(n, np.float32)
                hb = np.zeros(n, np.float32)
            reps = 100 if n <= (1 << 20) else 5
            t = timeit(lambda: redop.check(redop.MPI_Reduce_local(hb, ha, n, H.MPI_FLOAT,
                                                                  H.MPI_SUM)), reps)
            out[kind].append(dict(count=n, us=round(t * 1e6, 2), GiBs=round(12 * n / t / 2**30, 2)))
    torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
