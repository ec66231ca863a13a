#!/usr/bin/env python3
"""Per-(op, type) kernel throughput (BASELINE config 3: 256 MiB per operand)
and the vector-target path (config 5: vector(67108864, 1, 2, MPI_DOUBLE)).
Kernel time from HIP events on the launch stream, batch-averaged;
GB/s = algorithmic bytes (3 x payload) / time.  Writes JSON to stdout."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402
from bench import event_time_per_launch  # noqa: E402

TYPES = ['MPI_INT8_T', 'MPI_INT16_T', 'MPI_INT32_T', 'MPI_INT64_T', 'MPI_UINT32_T', 'MPI_INTEGER16',
         'MPIX_C_FLOAT16', 'MPIX_BFLOAT16', 'MPI_FLOAT', 'MPI_DOUBLE', 'MPI_COMPLEX4',
         'MPI_C_FLOAT_COMPLEX', 'MPI_C_DOUBLE_COMPLEX', 'MPI_LOGICAL', 'MPI_C_BOOL', 'MPI_BYTE',
         'MPI_2INT', 'MPI_FLOAT_INT', 'MPI_DOUBLE_INT', 'MPI_LONG_INT', 'MPI_SHORT_INT',
         'MPI_2DOUBLE_PRECISION']


def main():
    nbytes = int(os.environ.get('PERF_BYTES', 256 << 20))
    dev = torch.device('cuda', 0)
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    # small non-negative values: no NaN/Inf traffic effects, no data-dependent branches
    a.view(torch.int8).random_(0, 3)
    b.view(torch.int8).random_(0, 3)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    out = []
    for tn in TYPES:
        dt = getattr(H, tn)
        ext = redop.datatype_extent(dt)
        n = nbytes // ext
        for on, op in H.OPS.items():
            if op in (H.MPI_REPLACE, H.MPI_NO_OP) or not redop.is_supported(op, dt):
                continue
            redop.check(redop.reduce_local_async(b, a, n, dt, op, s))   # lazy module load
            s.synchronize()
            avg, med, mn = event_time_per_launch(
                lambda: redop.check(redop.reduce_local_async(b, a, n, dt, op, s)), 10, s)
            out.append(dict(type=tn, op=on, bytes=n * ext, ms=round(avg, 4),
                            GBs=round(3 * n * ext / (avg * 1e-3) / 1e9, 1)))
    # relatively misaligned operands (in at +4 bytes: packet kernel with
    # unaligned loads of `in`, default cache policy for them), next to the
    # aligned launch, both at 256 MiB and at 1 GiB per operand -- at 256 MiB
    # the default-policy `in` stream can stay in the 256 MB MALL across
    # back-to-back launches of the same buffers, at 1 GiB it cannot
    misaligned = []
    for mb in (nbytes, 1 << 30):
        if mb == nbytes:
            x, y = a, b
        else:
            x = torch.empty(mb, dtype=torch.uint8, device=dev)
            y = torch.empty(mb, dtype=torch.uint8, device=dev)
            x.view(torch.int8).random_(0, 3)
            y.view(torch.int8).random_(0, 3)
        n = mb // 4 - 4
        row = dict(bytes=mb)
        for tag, shift in (('aligned', 0), ('in_plus_4B', 4)):
            redop.check(redop.reduce_local_async(y.data_ptr() + shift, x, n, H.MPI_FLOAT,
                                                 H.MPI_SUM, s))
            avg, med, mn = event_time_per_launch(
                lambda: redop.check(redop.reduce_local_async(y.data_ptr() + shift, x, n,
                                                             H.MPI_FLOAT, H.MPI_SUM, s)), 10, s)
            row[tag] = dict(ms=round(avg, 4), GBs=round(12 * n / (avg * 1e-3) / 1e9, 1))
        misaligned.append(row)
        if mb != nbytes:
            del x, y
    # fused multi-input combine (pairwise reduce-scatter epilogue): 7 received
    # 64 MiB blocks folded into the result in one pass vs 7 sequential calls
    blk = 64 << 20
    m = blk // 4
    ins = [torch.empty(m, dtype=torch.float32, device=dev).uniform_(-1, 1) for _ in range(7)]
    acc = torch.empty(m, dtype=torch.float32, device=dev).uniform_(-1, 1)
    torch.cuda.synchronize()
    redop.check(redop.reduce_local_multi_async(ins, acc, m, H.MPI_FLOAT, H.MPI_SUM, s))
    t_multi, _, _ = event_time_per_launch(
        lambda: redop.check(redop.reduce_local_multi_async(ins, acc, m, H.MPI_FLOAT, H.MPI_SUM,
                                                           s)), 10, s)

    def seq():
        for x in ins:
            redop.check(redop.reduce_local_async(x, acc, m, H.MPI_FLOAT, H.MPI_SUM, s))
    t_seq, _, _ = event_time_per_launch(seq, 10, s)
    multi = dict(case='7 x 64 MiB fp32 blocks folded into a 64 MiB result',
                 fused_ms=round(t_multi, 4), sequential_ms=round(t_seq, 4),
                 fused_GBs=round(9 * blk / (t_multi * 1e-3) / 1e9, 1),
                 sequential_GBs_algorithmic=round(21 * blk / (t_seq * 1e-3) / 1e9, 1),
                 speedup=round(t_seq / t_multi, 2))
    del ins, acc
    del a, b
    torch.cuda.empty_cache()
    # config 5: vector(67108864, 1, 2, MPI_DOUBLE), 512 MiB payload, 1 GiB span
    cnt = 67108864
    src = torch.zeros(cnt, dtype=torch.float64, device=dev)
    dst = torch.zeros(2 * cnt, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    redop.check(redop.reduce_local_vector(src, dst, cnt, 1, 2, H.MPI_DOUBLE, H.MPI_SUM, s))
    avg, med, mn = event_time_per_launch(
        lambda: redop.check(redop.reduce_local_vector(src, dst, cnt, 1, 2, H.MPI_DOUBLE, H.MPI_SUM,
                                                      s)), 10, s)
    vec = dict(config='vector(67108864,1,2,MPI_DOUBLE) SUM', ms=round(avg, 4),
               GBs_algorithmic=round(3 * cnt * 8 / (avg * 1e-3) / 1e9, 1),
               frac_of_8TBs=round(3 * cnt * 8 / (avg * 1e-3) / 8e12, 4))
    print(json.dumps(dict(per_type=out, vector=vec, misaligned=misaligned, multi=multi,
                          build=redop.build_info())))


if __name__ == '__main__':
    main()
