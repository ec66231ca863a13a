#!/usr/bin/env python3
"""Zero-copy (page-locked host) MPIX_Reduce_local against the grid size.

At 1 GiB the zero-copy kernel runs at 0.94 of the PCIe floor, at 4 MiB at about
0.66: one tile per block means every block loads its whole tile (PCIe
host-to-device) before it stores anything (device-to-host), and at a few
hundred blocks the grid is one round, so the two link directions take turns
instead of overlapping.  A capped grid makes every block loop over tiles, so
some blocks store while others load.  This probe times the synchronous call
(median of C-timed calls, fp32 SUM, both operands page-locked) per operand
size and grid cap (MPIX_Redop_set_launch max_grid; 0 = one tile per block),
the caps interleaved within each size.  One JSON line.
usage: python3 tools/pinned_grid.py [--sizes-mib 1,4,16,64,256,1024] [--caps 0,1024,512,256,128,64]
                                     [--blocks 256]
Run it with MPIX_REDOP_ZC_GRID=0, else the library's own zero-copy cap (32)
applies under every --caps value.  --blocks: threads per block to cross with
the caps (round 5, one packet per lane: a 1024-thread block moves the tile a
256 x 4 block moved before).
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes-mib', default='1,4,16,64,256,1024')
    ap.add_argument('--caps', default='0,1024,512,256,128,64')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--blocks', default='')
    a = ap.parse_args()
    sizes = [int(x) << 20 for x in a.sizes_mib.split(',')]
    old = redop.get_launch()
    blocks = [int(x) for x in a.blocks.split(',')] if a.blocks else [old['block']]
    caps = [(b, int(x)) for b in blocks for x in a.caps.split(',')]
    B = bench.bench_lib()
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local, ctypes.c_void_p).value
    top = max(sizes) // 4
    inb = torch.empty(top, dtype=torch.float32).pin_memory()
    io = torch.empty(top, dtype=torch.float32).pin_memory()
    inb.uniform_(-1, 1)
    io.uniform_(-1, 1)
    rows = []
    try:
        for s in sizes:
            n = s // 4
            reps = max(5, min(400, (64 << 20) // s))
            t = {c: [] for c in caps}
            for _ in range(a.rounds):
                for c in caps:
                    redop.check(redop.set_launch(c[0], c[1]))
                    t[c].append(bench.c_call_median_us(B, fn, inb.data_ptr(), io.data_ptr(), n,
                                                       reps))
            for c in caps:
                us = sorted(t[c])[len(t[c]) // 2]
                rows.append(dict(bytes=s, block=c[0], max_grid=c[1], us=round(us, 2),
                                 GBs_pcie_bytes=round(3 * s / (us * 1e-6) / 1e9, 2)))
            print(json.dumps(dict(progress=s)), file=sys.stderr, flush=True)
    finally:
        redop.set_launch(old['block'], old['max_grid'])
    print(json.dumps(dict(what='synchronous zero-copy MPIX_Reduce_local (fp32 SUM, both operands '
                                'page-locked) per operand size, block and grid cap, median of %d '
                                'interleaved rounds of C-timed medians' % a.rounds,
                           zc_grid_env=os.environ.get('MPIX_REDOP_ZC_GRID'), rows=rows)),
          flush=True)


if __name__ == '__main__':
    main()
