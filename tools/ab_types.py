#!/usr/bin/env python3
"""Config-3 rows (every supported (op, type) at 1 GiB per operand, kernel only,
HIP events) for ONE build of libmpix_redop.so, each row also as a fraction of
the fp32 SUM row measured in the same process (the placement-independent
figure VERDICT r02 item 5 asks for: every row within 2 % of fp32 SUM).

usage: ab_types.py LIBPATH LABEL   (run alternately for two builds)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import redop  # noqa: E402

redop.LIB_PATH = os.path.abspath(sys.argv[1])
from mpich_amd import handles as H  # noqa: E402
from bench import event_time_per_launch  # noqa: E402

TYPES = ('MPI_INT8_T', 'MPI_UINT8_T', 'MPI_INT16_T', 'MPI_INT32_T', 'MPI_INT64_T', 'MPI_INTEGER16',
         'MPIX_C_FLOAT16', 'MPIX_BFLOAT16', 'MPI_FLOAT', 'MPI_DOUBLE', 'MPI_COMPLEX4',
         'MPI_C_FLOAT_COMPLEX', 'MPI_C_DOUBLE_COMPLEX', 'MPI_C_BOOL', 'MPI_LOGICAL', 'MPI_BYTE',
         'MPI_2INT', 'MPI_FLOAT_INT', 'MPI_DOUBLE_INT', 'MPI_SHORT_INT')


def main():
    nbytes = 1 << 30
    dev = torch.device('cuda', 0)
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.view(torch.int8).random_(0, 3)
    b.view(torch.int8).random_(0, 3)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    rows = []

    def one(dt, op, n):
        redop.check(redop.reduce_local_async(b, a, n, dt, op, s))
        avg, _, _ = event_time_per_launch(
            lambda: redop.check(redop.reduce_local_async(b, a, n, dt, op, s)), 5, s, rounds=2)
        return avg

    ref = []
    for tn in TYPES:
        dt = getattr(H, tn, None)
        if dt is None:
            continue
        ext = redop.datatype_extent(dt)
        n = nbytes // ext
        for on, op in H.OPS.items():
            if op in (H.MPI_REPLACE, H.MPI_NO_OP) or not redop.is_supported(op, dt):
                continue
            # fp32 SUM timed right before and after each row (drift-free ratio)
            r0 = one(H.MPI_FLOAT, H.MPI_SUM, nbytes // 4)
            t = one(dt, op, n)
            r1 = one(H.MPI_FLOAT, H.MPI_SUM, nbytes // 4)
            ref += [r0, r1]
            rows.append(dict(type=tn, op=on, ms=round(t, 4), GBs=round(3 * n * ext / t / 1e6, 1),
                             vs_fp32_sum=round((r0 + r1) / 2 / t, 4)))
    t_ref = sum(ref) / len(ref)
    ref = [min(ref), max(ref)]
    rows.sort(key=lambda r: r['vs_fp32_sum'])
    print(json.dumps(dict(label=sys.argv[2], build=redop.build_info(), fp32_sum_ms=round(t_ref, 4),
                          fp32_sum_ms_range=[round(x, 4) for x in ref],
                          min_vs_fp32_sum=rows[0]['vs_fp32_sum'],
                          within_2pct=sum(r['vs_fp32_sum'] >= 0.98 for r in rows), rows=len(rows),
                          slowest=rows[:12], all=rows)))


if __name__ == '__main__':
    main()
