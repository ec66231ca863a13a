#!/usr/bin/env python3
"""Reduce-scatter-block schedules of libmpix_coll.so on the local device
transport, P ranks as threads on cuda:0 (fp32 SUM, BYTES per rank).  On one
GPU the "exchange" is a device-to-device copy sharing HBM with the combine,
so this only bounds the schedules' own overhead (chunking, stream hand-offs);
link-level gains need the multi-GPU run.  JSON to stdout."""
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import ccl  # noqa: E402
from mpich_amd import handles as H  # noqa: E402


def main():
    P = int(os.environ.get('P', '4'))
    nbytes = int(os.environ.get('BYTES', str(1 << 30)))
    reps = int(os.environ.get('REPS', '5'))
    recvcount = nbytes // 4 // P
    sends = [torch.rand(recvcount * P, device='cuda') for _ in range(P)]
    recvs = [torch.empty(recvcount, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    out = dict(P=P, bytes_per_rank=recvcount * P * 4, transport='local device, one GPU')
    for algo in ('pairwise', 'pairwise_pipelined', 'recursive_halving', 'pairwise_sequential'):
        comms = ccl.comm_create_local(P, [0] * P)
        times = []
        for rep in range(reps + 1):
            barrier = threading.Barrier(P)
            res = [None] * P

            def body(r):
                barrier.wait()
                res[r] = ccl.reduce_scatter_block(sends[r], recvs[r], recvcount, H.MPI_FLOAT,
                                                  H.MPI_SUM, comms[r], algo)
            ths = [threading.Thread(target=body, args=(r,)) for r in range(P)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join(120)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            assert res == [0] * P, res
            if rep:
                times.append(dt)
        for c in comms:
            c.free()
        times.sort()
        out[algo] = dict(ms_median=round(times[len(times) // 2] * 1e3, 3),
                         ms_min=round(times[0] * 1e3, 3))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
