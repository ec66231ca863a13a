#!/usr/bin/env python3
"""NaN payloads of floating-point SUM / PROD: on every
pair of NaN-bearing operands, does gfx950's v_add / v_mul return the payload
the reference's CPU loop returns?  The reference loop (op_fns.c:19-91,
`a[i] = a[i] + b[i]`) compiled for x86-64 returns the first NaN operand,
quieted (SSE addss/mulss keep src1 = inout); the oracle is that loop built by
gcc on this host, so its bits are the x86 rule.  Records, does not assert.

usage: nan_payload_probe.py [out.json]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import redop  # noqa: E402
from oracle import oracle as orc  # noqa: E402

MPI_FLOAT, MPI_DOUBLE, MPIX_C_FLOAT16 = 0x4c00040a, 0x4c00080b, 0x4c000246
MPI_SUM, MPI_PROD = 0x58000003, 0x58000004

SPECIALS = {
    'float32': (np.uint32, MPI_FLOAT, [0x7fc00000, 0x7fc12345, 0xffc54321, 0x7f800001,
                                       0xff812345, 0x3f800000, 0x7f800000, 0x00000000]),
    'float64': (np.uint64, MPI_DOUBLE, [0x7ff8000000000000, 0x7ff8000012345678,
                                        0xfff8000087654321, 0x7ff0000000000001,
                                        0xfff0000012345678, 0x3ff0000000000000,
                                        0x7ff0000000000000, 0x0]),
    'float16': (np.uint16, MPIX_C_FLOAT16, [0x7e00, 0x7e15, 0xfe2a, 0x7c01, 0xfc15, 0x3c00,
                                            0x7c00, 0x0000]),
}


def is_nan(bits, width):
    if width == 16:
        return (bits & 0x7c00) == 0x7c00 and (bits & 0x3ff) != 0
    if width == 32:
        return (bits & 0x7f800000) == 0x7f800000 and (bits & 0x7fffff) != 0
    return (bits & 0x7ff0000000000000) == 0x7ff0000000000000 and (bits & 0xfffffffffffff) != 0


def main():
    orc.build()
    out = {}
    for name, (ut, dt, vals) in SPECIALS.items():
        width = np.dtype(ut).itemsize * 8
        a = np.array([x for x in vals for _ in vals], dtype=ut)      # inout
        b = np.array([y for _ in vals for y in vals], dtype=ut)      # in
        for opn, op in (('SUM', MPI_SUM), ('PROD', MPI_PROD)):
            da, db = torch.from_numpy(a.copy()).cuda(), torch.from_numpy(b.copy()).cuda()
            torch.cuda.synchronize()
            redop.check(redop.MPI_Reduce_local(db, da, a.size, dt, op))
            gpu = da.cpu().numpy()
            cpu = a.copy()
            orc.reduce_local(b, cpu, a.size, dt, op)
            rows, same, nan_rows = [], 0, 0
            for i in range(a.size):
                if not (is_nan(int(a[i]), width) or is_nan(int(b[i]), width)):
                    continue
                nan_rows += 1
                g, c = int(gpu[i]), int(cpu[i])
                same += g == c
                rows.append(dict(inout=hex(int(a[i])), in_=hex(int(b[i])), gpu=hex(g), x86=hex(c),
                                 gpu_is_nan=is_nan(g, width)))
            out['%s_%s' % (name, opn)] = dict(nan_pairs=nan_rows, identical_to_x86=same,
                                              all_gpu_results_nan=all(r['gpu_is_nan'] for r in rows),
                                              rows=rows)
    summary = {k: dict(nan_pairs=v['nan_pairs'], identical_to_x86=v['identical_to_x86'],
                       all_gpu_results_nan=v['all_gpu_results_nan']) for k, v in out.items()}
    res = dict(summary=summary, cases=out, build=redop.build_info())
    if len(sys.argv) > 1:
        with open(sys.argv[1], 'w') as f:
            json.dump(res, f, indent=1)
    print(json.dumps(summary))


if __name__ == '__main__':
    main()
