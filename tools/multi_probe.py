#!/usr/bin/env python3
"""Multi-input and tree combines (the pairwise reduce-scatter's fold and the
pulls' tree), kernel time by HIP events: fp32 SUM, S bytes per operand,
MPIX_Reduce_local_multi_async with k inputs ((k + 2) x S moved) and
MPIX_Reduce_local_tree_async with k slots into a separate output ((k + 1) x S).
The plain STREAM triad of the same process is printed beside them.  One JSON
line.  usage: python3 tools/multi_probe.py [--mib 256] [--ks 1,2,3,4,7,15]
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
    ap.add_argument('--mib', type=int, default=256)
    ap.add_argument('--ks', default='1,2,3,4,7,15')
    ap.add_argument('--tree-ks', default='2,4,8,16')
    ap.add_argument('--tree-inplace', action='store_true',
                    help='tree folds write slot 0 in place instead of a separate output')
    ap.add_argument('--skew', type=int, default=0,
                    help='operand q starts q * SKEW bytes into its allocation (placement probe)')
    a = ap.parse_args()
    S = a.mib << 20
    n = S // 4
    ks = [int(x) for x in a.ks.split(',')]
    tks = [int(x) for x in a.tree_ks.split(',')]
    top = max(ks + tks)
    dev = torch.device('cuda', 0)
    sk = a.skew // 4
    bufs = [torch.empty(n + q * sk, dtype=torch.float32, device=dev)[q * sk:].uniform_(-1, 1)
            for q in range(top + 1)]
    out = torch.empty(n, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    B = bench.bench_lib()
    tri, _, _ = bench.event_time_per_launch(
        lambda: B.mpix_bench_triad(out.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(),
                                   ctypes.c_float(0.5), n, s.cuda_stream), 10, s)
    rows = [dict(kind='triad', GBs=round(3 * S / (tri * 1e-3) / 1e9, 1))]
    for k in ks:
        ins = bufs[1:1 + k]
        f = lambda: redop.check(redop.reduce_local_multi_async(ins, bufs[0], n, H.MPI_FLOAT,  # noqa
                                                                H.MPI_SUM, s))
        f()
        ms, _, _ = bench.event_time_per_launch(f, 10, s)
        rows.append(dict(kind='multi', k=k, ms=round(ms, 4),
                         GBs=round((k + 2) * S / (ms * 1e-3) / 1e9, 1)))
    for k in tks:
        ins = bufs[:k]
        dst = ins[0] if a.tree_inplace else out
        f = lambda: redop.check(redop.reduce_local_tree_async(ins, dst, n, H.MPI_FLOAT,  # noqa
                                                               H.MPI_SUM, s))
        f()
        ms, _, _ = bench.event_time_per_launch(f, 10, s)
        rows.append(dict(kind='tree', k=k, ms=round(ms, 4),
                         GBs=round((k + 1) * S / (ms * 1e-3) / 1e9, 1)))
    print(json.dumps(dict(skew=a.skew, tree_inplace=a.tree_inplace, env={k: v for k, v in os.environ.items()
                                            if k.startswith('MPIX_REDOP_')}, what='fp32 SUM multi-input and tree combines, %d MiB per operand, HIP '
                               'events (average of 3 batches of 10 launches)' % a.mib, rows=rows)),
          flush=True)


if __name__ == '__main__':
    main()
