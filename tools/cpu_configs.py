#!/usr/bin/env python3
"""CPU side of BASELINE.md's per-config comparison table, timed on the host
cores of the box it runs on (no GPU used).  The baseline is the oracle --
the clean-room C restatement of MPICH's op loop (oracle/redop_oracle.c;
running reference code is denied) -- with the same loop
shape as MPIR_OP_TYPE_REDUCE_CASE (mpir_op_util.h:46-53), one element per
iteration, one thread per rank.

  C2: fp32 SUM at 16..1024 MiB per operand (x2), 1 core and all cores
  C3: every (op, type) the GPU path runs, 256 MiB per operand, 1 core
  C4: one rank's combine steps of the recursive-halving reduce-scatter-block
      schedule, P = 2, 4, 8, 4 GiB per rank, 1 core (the CPU cap on MPICH's
      RSB throughput with an infinitely fast network)
  C5: vector(67108864, 1, 2, MPI_DOUBLE) SUM target, packed source, 1 core

Writes one JSON object to stdout.  Usage: cpu_configs.py [--quick]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from oracle import oracle as orc  # noqa: E402

GIB = float(1 << 30)
TYPES = ['MPI_INT8_T', 'MPI_INT16_T', 'MPI_INT32_T', 'MPI_INT64_T', 'MPI_UINT32_T', 'MPI_INTEGER16',
         'MPIX_C_FLOAT16', 'MPIX_BFLOAT16', 'MPI_FLOAT', 'MPI_DOUBLE', 'MPI_COMPLEX4',
         'MPI_C_FLOAT_COMPLEX', 'MPI_C_DOUBLE_COMPLEX', 'MPI_LOGICAL', 'MPI_C_BOOL', 'MPI_BYTE',
         'MPI_2INT', 'MPI_FLOAT_INT', 'MPI_DOUBLE_INT', 'MPI_LONG_INT', 'MPI_SHORT_INT',
         'MPI_2DOUBLE_PRECISION']


def timed(fn, min_reps=2, budget=0.5):
    """median wall seconds of fn() over >= min_reps calls (after one warm call)"""
    fn()
    ts = []
    t_end = time.perf_counter() + budget
    while len(ts) < min_reps or time.perf_counter() < t_end:
        t0 = orc.wtime()
        fn()
        ts.append(orc.wtime() - t0)
    ts.sort()
    return ts[len(ts) // 2], len(ts)


def progress(msg):
    print('[cpu_configs %.0fs] %s' % (time.perf_counter() - T0, msg), file=sys.stderr, flush=True)


T0 = time.perf_counter()


def operand(rng, dt, nbytes):
    """bytes of `dt` elements with normal floating values (uniform [-1, 1)
    per float component: no denormal assists on the host) and random bits
    for everything else"""
    it = orc.internal(dt)
    kind = (it >> 16) & 0xf if (it >> 24) == 0x4c else 0
    size = (it >> 8) & 0xff
    comp = size // 2 if kind == 4 else size
    if kind in (3, 4, 5) and comp in (2, 4, 8):
        n = nbytes // comp
        if kind == 5:                                   # bf16: upper half of fp32
            x = (rng.uniform(-1, 1, n).astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
        else:
            x = rng.uniform(-1, 1, n).astype({2: np.float16, 4: np.float32, 8: np.float64}[comp])
        return x.view(np.uint8)
    return rng.integers(0, 256, nbytes, dtype=np.uint8)


def main():
    quick = '--quick' in sys.argv
    orc.build()
    from mpich_amd import redop
    ncores = len(os.sched_getaffinity(0))
    threads_all = max(1, min(16, ncores))
    rng = np.random.default_rng(0x5EED0002)
    out = dict(host_cpu='', nproc=os.cpu_count(), affinity_cpus=ncores, threads_all=threads_all,
               baseline='oracle/redop_oracle.c (clean-room restatement of op_fns.c), kind "port"')
    for line in open('/proc/cpuinfo'):
        if line.startswith('model name'):
            out['host_cpu'] = line.split(':', 1)[1].strip()
            break

    # C2: fp32 SUM size sweep
    sizes = (16, 64, 256) if quick else (16, 32, 64, 128, 256, 512, 1024)
    big = max(sizes) << 20
    a = rng.uniform(-1, 1, big // 4).astype(np.float32)
    b = rng.uniform(-1, 1, big // 4).astype(np.float32)
    c2 = []
    for mib in sizes:
        n = (mib << 20) // 4
        row = dict(mib=mib)
        for tag, nth in (('1core', 1), ('allcores', threads_all)):
            t, reps = timed(lambda: orc.reduce_local(b, a, n, H.MPI_FLOAT, H.MPI_SUM,
                                                     nthreads=nth))
            row[tag] = dict(GiBs=round(12 * n / t / GIB, 2), ms=round(t * 1e3, 3), reps=reps)
        c2.append(row)
    out['c2_fp32_sum_sweep'] = c2
    progress('c2 done')
    del a, b

    # C3: per (op, type), 256 MiB per operand, 1 core
    nbytes = (64 if quick else 256) << 20
    c3 = []
    for tn in TYPES:
        dt = getattr(H, tn)
        ext = orc.extent(dt)
        n = nbytes // ext
        x = operand(rng, dt, n * ext)
        y = operand(rng, dt, n * ext)
        for on, op in H.OPS.items():
            if op in (H.MPI_REPLACE, H.MPI_NO_OP) or not redop.is_supported(op, dt):
                continue
            x0 = x.copy()       # every op starts from the same operands
            t, reps = timed(lambda: orc.reduce_local(y, x0, n, dt, op), budget=0.2)
            c3.append(dict(type=tn, op=on, bytes=n * ext, ms=round(t * 1e3, 3),
                           GiBs_1core=round(3 * n * ext / t / GIB, 2)))
        del x, y
        progress('c3 ' + tn)
    out['c3_per_type_1core'] = c3

    # C4: the combine work one rank of the recursive-halving schedule does
    # (…recursive_halving.c:164-229: step k reduces total / 2^(k+1) received
    # elements into tmp_results), on one core with preallocated buffers --
    # the CPU-side cap on MPICH's RSB even with an infinitely fast network
    per_rank = (256 << 20) if quick else (4 << 30)
    total = per_rank // 4
    x = np.random.default_rng(0x5EED0100).random(total // 2, dtype=np.float32)
    y = np.random.default_rng(0x5EED0101).random(total // 2, dtype=np.float32)
    c4 = []
    for P in (2, 4, 8):
        steps = []
        k = total // 2
        while k >= total // P:
            steps.append(k)
            k //= 2

        def schedule():
            for m in steps:
                orc.reduce_local(x, y, m, H.MPI_FLOAT, H.MPI_SUM)
        t, reps = timed(schedule, min_reps=2, budget=1.0)
        c4.append(dict(P=P, bytes_per_rank=per_rank, combined_elements=sum(steps),
                       combine_s=round(t, 4), reps=reps,
                       busbw_cap_GBs=round((P - 1) / P * per_rank / t / 1e9, 2),
                       note='one rank\'s combine steps only (no network): the CPU cap on '
                            '(P-1)/P x bytes / t'))
    del x, y
    out['c4_rsb_combine_1core'] = c4
    progress('c4 done')

    # C5: vector(67108864, 1, 2, MPI_DOUBLE) SUM target, 1 core
    cnt = (1 << 24) if quick else 67108864
    src = rng.uniform(-1, 1, cnt)
    dst = rng.uniform(-1, 1, 2 * cnt)
    t, reps = timed(lambda: orc.reduce_local_vector(src, dst, cnt, 1, 2, H.MPI_DOUBLE,
                                                    H.MPI_SUM))
    out['c5_vector_1core'] = dict(count=cnt, ms=round(t * 1e3, 3), reps=reps,
                                  GiBs_algorithmic=round(3 * cnt * 8 / t / GIB, 2))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
