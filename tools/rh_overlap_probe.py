#!/usr/bin/env python3
"""Recursive-halving reduce-scatter with the combine overlap off and on, P
ranks as threads of one process sharing device 0 (local communicator: the
exchange is a device copy, so transfer and combine compete for the same HBM
and the overlap can only show its cost, not its gain over xGMI).  fp32 SUM,
S bytes per rank, wall time of the whole collective (all ranks, synchronised),
the two settings alternating; each result checked equal between settings.
One JSON line.  usage: python3 tools/rh_overlap_probe.py [--p 4] [--mib 256]
"""
import argparse
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
from mpich_amd import redop  # noqa: E402


def run_ranks(comms, fn):
    out = [None] * len(comms)

    def body(r):
        out[r] = fn(r, comms[r])
    ths = [threading.Thread(target=body, args=(r,)) for r in range(len(comms))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--p', type=int, default=4)
    ap.add_argument('--mib', type=int, default=256)
    ap.add_argument('--reps', type=int, default=6)
    a = ap.parse_args()
    P = a.p
    total = (a.mib << 20) // 4 // P * P
    rc = total // P
    dev = torch.device('cuda', 0)
    sends = [torch.empty(total, dtype=torch.float32, device=dev).uniform_(-1, 1) for _ in range(P)]
    recvs = {m: [torch.empty(rc, dtype=torch.float32, device=dev) for _ in range(P)]
             for m in ('0', 'default')}
    comms = ccl.comm_create_local(P, [0] * P)
    times = {'0': [], 'default': []}

    def once(mode):
        if mode == '0':
            os.environ['MPIX_COLL_RH_OVERLAP'] = '0'
        else:
            os.environ.pop('MPIX_COLL_RH_OVERLAP', None)
        torch.cuda.synchronize()
        t = time.perf_counter()
        rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
            sends[r], recvs[mode][r], rc, H.MPI_FLOAT, H.MPI_SUM, c, 'recursive_halving'))
        torch.cuda.synchronize()
        assert rcs == [0] * P, rcs
        return time.perf_counter() - t

    for mode in ('0', 'default'):
        once(mode)          # scratch, streams
    for _ in range(a.reps):
        for mode in ('0', 'default'):
            times[mode].append(once(mode))
    same = all(torch.equal(recvs['0'][r].view(torch.int32), recvs['default'][r].view(torch.int32))
               for r in range(P))
    for c in comms:
        redop.check(c.free())
    med = {m: sorted(v)[len(v) // 2] * 1e3 for m, v in times.items()}
    print(json.dumps(dict(
        what='recursive-halving MPI_Reduce_scatter_block (fp32 SUM, %d MiB per rank), %d ranks as '
             'threads sharing device 0, local (device-copy) exchange; median wall ms of %d calls '
             'per setting, alternating' % (a.mib, P, a.reps),
        overlap_off_ms=round(med['0'], 3), overlap_default_ms=round(med['default'], 3),
        ratio=round(med['default'] / med['0'], 4), bit_identical=same,
        all_ms={m: [round(1e3 * t, 3) for t in v] for m, v in times.items()})), flush=True)


if __name__ == '__main__':
    main()
