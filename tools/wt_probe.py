#!/usr/bin/env python3
"""Write-through store patterns of the contiguous kernel (MPIX_Redop_set_store_policy):
blocks b with b % every == phase store write-through (sc0 sc1) instead of
non-temporally.  One process; 1 GiB fp32 SUM launches timed with HIP events
on their stream (median of batches), patterns interleaved round by round, for
several operand placements: two separate 1 GiB allocations, and both carved
from one slab with `in` at 1 GiB + offset (the placements that split the
kernel's time in round 2, profiles/r02_split_rootcause.json); plus sizes.

run: wt_probe.py OUT.json   (one JSON object)
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

N = 1 << 28
# (xcd_mask, every, phase)
PATTERNS = [(0, 0, 0), (0, 4, 3), (0x88, 0, 0), (0x22, 0, 0), (0x11, 0, 0), (0x03, 0, 0),
            (0x0c, 0, 0), (0x80, 0, 0), (0x81, 0, 0), (0xaa, 0, 0), (0x8c, 0, 0)]
OFFSETS = [0, 65536, (2 << 20) + 4096]


def timed(fn, s, reps=10, batches=3):
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
    return out[len(out) // 2]


def main(path):
    s = torch.cuda.Stream()
    sep_in = torch.empty(N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    sep_io = torch.empty(N, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    slab = torch.empty(2 * N + (128 << 20) // 4, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    torch.cuda.synchronize()
    places = {'separate': (sep_in, sep_io)}
    for off in OFFSETS:
        e = N + off // 4
        places['slab_in_at_1GiB+%d' % off] = (slab[e:e + N], slab[:N])
    key = lambda pat: '0x%x:%d:%d' % pat
    res = {p: {key(pat): [] for pat in PATTERNS} for p in places}
    for _ in range(3):
        for pname, (xin, xio) in places.items():
            for pat in PATTERNS:
                redop.check(redop.set_store_policy(*pat))
                ms = timed(lambda: redop.check(redop.reduce_local_async(
                    xin, xio, N, H.MPI_FLOAT, H.MPI_SUM, s)), s)
                res[pname][key(pat)].append(ms)
    out = {'what': 'median kernel ms of 1 GiB fp32 SUM per store pattern (xcd_mask:every:phase) '
                   'and placement, three interleaved rounds', 'kernel_ms': {}, 'vs_none': {}}
    for pname, d in res.items():
        med = {k: round(sorted(v)[1], 4) for k, v in d.items()}
        out['kernel_ms'][pname] = med
        out['vs_none'][pname] = {k: round(med['0x0:0:0'] / v, 4) for k, v in med.items()}
    sizes = {}
    for mib in (16, 64, 256, 1024):
        m = mib * (1 << 20) // 4
        row = {}
        for pat in ((0, 0, 0), (0x88, 0, 0)):
            redop.check(redop.set_store_policy(*pat))
            row[key(pat)] = round(timed(lambda: redop.check(redop.reduce_local_async(
                sep_in, sep_io, m, H.MPI_FLOAT, H.MPI_SUM, s)), s, reps=20), 4)
        sizes['%dMiB' % mib] = row
    out['sizes_separate_kernel_ms'] = sizes
    redop.check(redop.set_store_policy(0, 0, 0, 0))
    json.dump(out, open(path, 'w'), indent=1)
    print(json.dumps(out['vs_none']))


if __name__ == '__main__':
    main(sys.argv[1])
