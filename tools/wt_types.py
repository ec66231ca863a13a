#!/usr/bin/env python3
"""Every config-3 (op, type) row at 1 GiB per operand, kernel only (HIP
events), with the contiguous kernel's store policy off and on in the same
process, row by row (MPIX_Redop_set_store_policy; POLICY = xcd_mask,every,phase).

usage: wt_types.py OUT.json [POLICY]   (default 0x88,0,0)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402
from bench import event_time_per_launch  # noqa: E402

TYPES = ('MPI_INT8_T', 'MPI_UINT8_T', 'MPI_INT16_T', 'MPI_INT32_T', 'MPI_INT64_T', 'MPI_INTEGER16',
         'MPIX_C_FLOAT16', 'MPIX_BFLOAT16', 'MPI_FLOAT', 'MPI_DOUBLE', 'MPI_COMPLEX4',
         'MPI_C_FLOAT_COMPLEX', 'MPI_C_DOUBLE_COMPLEX', 'MPI_C_BOOL', 'MPI_LOGICAL', 'MPI_BYTE',
         'MPI_2INT', 'MPI_FLOAT_INT', 'MPI_DOUBLE_INT', 'MPI_SHORT_INT')   # as tools/ab_types.py


def main(path, policy):
    nbytes = 1 << 30
    dev = torch.device('cuda', 0)
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.view(torch.int8).random_(0, 3)
    b.view(torch.int8).random_(0, 3)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()

    def one(dt, op, n, pol):
        redop.check(redop.set_store_policy(*pol))
        redop.check(redop.reduce_local_async(b, a, n, dt, op, s))
        avg, _, _ = event_time_per_launch(
            lambda: redop.check(redop.reduce_local_async(b, a, n, dt, op, s)), 5, s, rounds=2)
        return avg

    off = (0, 0, 0, 0)
    rows = []
    for tn in TYPES:
        dt = getattr(H, tn, None)
        if dt is None:
            continue
        ext = redop.datatype_extent(dt)
        n = nbytes // ext
        for on, op in H.OPS.items():
            if op in (H.MPI_REPLACE, H.MPI_NO_OP) or not redop.is_supported(op, dt):
                continue
            t0 = one(dt, op, n, off)
            t1 = one(dt, op, n, policy)
            t2 = one(dt, op, n, off)
            t3 = one(dt, op, n, policy)
            toff, ton = (t0 + t2) / 2, (t1 + t3) / 2
            rows.append(dict(type=tn, op=on, off_ms=round(toff, 4), on_ms=round(ton, 4),
                             speedup=round(toff / ton, 4)))
    redop.check(redop.set_store_policy(*off))
    rows.sort(key=lambda r: r['speedup'])
    sp = [r['speedup'] for r in rows]
    res = dict(policy=list(policy), rows=len(rows), min_speedup=sp[0], max_speedup=sp[-1],
               median_speedup=sp[len(sp) // 2], slower=[r for r in rows if r['speedup'] < 1.0],
               all=rows)
    json.dump(res, open(path, 'w'), indent=1)
    print(json.dumps({k: res[k] for k in ('policy', 'rows', 'min_speedup', 'median_speedup',
                                          'max_speedup')}))


if __name__ == '__main__':
    pol = tuple(int(x, 0) for x in (sys.argv[2] if len(sys.argv) > 2 else '0x88,0,0').split(','))
    main(sys.argv[1], pol + (0,) * (4 - len(pol)))
