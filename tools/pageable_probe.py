#!/usr/bin/env python3
"""The pageable end-to-end path: MPIX_Reduce_local on 1 GiB
pageable (numpy) operands through the library's host workers, one
configuration per process (the workers' knobs are read from the environment
at first use):

  W      MPIX_REDOP_PAGEABLE_THREADS   workers (the caller is worker 0)
  chunk  MPIX_REDOP_PAGEABLE_CHUNK     bytes per chunk
  db     MPIX_REDOP_PAGEABLE_DB        1: copy the next chunk during the kernel
  aff    MPIX_REDOP_PAGEABLE_AFFINITY  none | gpu (CPUs of the GPU's NUMA node)
  nt     MPIX_REDOP_PAGEABLE_NT        1: non-temporal stores into the pinned buffers
  mode   MPIX_REDOP_PAGEABLE_MODE      worker (own chunks) | wave (all on one chunk)

Beside each: the host memcpy rate of one thread and of W threads (numpy
copyto on disjoint 16 MiB slices, pageable -> page-locked), and the PCIe
floor of the call's traffic (max(2 GiB / H2D, 1 GiB / D2H), hipMemcpy from
page-locked memory).  Checked against the oracle's result on a slice.

usage: pageable_probe.py sweep OUT.jsonl      (spawns one process per config)
       pageable_probe.py one                  (the current environment)"""
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [(8, 16, 0, 'none'), (8, 16, 1, 'none'), (8, 8, 1, 'none'), (8, 16, 1, 'gpu'),
           (8, 8, 1, 'gpu'), (12, 8, 1, 'gpu'), (15, 8, 1, 'gpu'), (15, 16, 1, 'gpu'),
           (12, 16, 0, 'gpu')]
if os.environ.get('PAGEABLE_CONFIGS'):      # "W:chunkMiB:db:aff[:nt[:mode]],..."
    CONFIGS = [tuple(int(x) if i in (0, 1, 2, 4) else x for i, x in enumerate(c.split(':')))
               for c in os.environ['PAGEABLE_CONFIGS'].split(',')]


def trace_summary(stderr):
    """the library's MPIX_REDOP_PIPE_TRACE line of the last call: per chunk
    copy-in, wait for the kernel, copy-out (ms summed over chunks) and the
    call's span"""
    line = [ln for ln in stderr.splitlines() if ln.startswith('{"pipe_trace"')]
    if not line:
        return None
    t = json.loads(line[-1])['pipe_trace']
    ns = t['ns']
    k = len(ns) // 5
    cin = sum(ns[5 * i + 1] - ns[5 * i] for i in range(k)) / 1e6
    wait = sum(ns[5 * i + 3] - ns[5 * i + 2] for i in range(k)) / 1e6
    cout = sum(ns[5 * i + 4] - ns[5 * i + 3] for i in range(k)) / 1e6
    span = max(ns) / 1e6
    first_wait = min(ns[5 * i + 2] for i in range(k)) / 1e6
    return dict(chunks=k, W=t['W'], nbuf=t['nbuf'], span_ms=round(span, 2),
                copy_in_ms_sum=round(cin, 2), wait_ms_sum=round(wait, 2),
                copy_out_ms_sum=round(cout, 2), first_wait_at_ms=round(first_wait, 2),
                worker_busy_frac=round((cin + cout) / (t['W'] * span), 3))


def memcpy_rate(src, dst, threads, chunk=16 << 20):
    """GB/s of host memcpy from pageable src into page-locked dst, `threads`
    threads on disjoint chunks (numpy releases the GIL inside copyto)"""
    import numpy as np
    n = src.nbytes
    s8, d8 = src.view(np.uint8), dst

    def part(t):
        for off in range(t * chunk, n, threads * chunk):
            np.copyto(d8[off:off + chunk], s8[off:off + chunk])
    best = None
    for _ in range(3):
        ths = [threading.Thread(target=part, args=(t,)) for t in range(threads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return round(n / best / 1e9, 2)


def one():
    import numpy as np
    import torch
    from mpich_amd import handles as H
    from mpich_amd import redop
    from oracle import oracle as orc
    n = int(os.environ.get('PAGEABLE_BYTES', 1 << 30)) // 4
    a = np.random.default_rng(1).random(n, dtype=np.float32)
    b = np.random.default_rng(2).random(n, dtype=np.float32)
    ref = a.copy()
    orc.build()
    orc.reduce_local(b, ref, n, H.MPI_FLOAT, H.MPI_SUM)
    redop.check(redop.MPI_Reduce_local(b, a, n, H.MPI_FLOAT, H.MPI_SUM))
    ok = a.tobytes() == ref.tobytes()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        redop.check(redop.MPI_Reduce_local(b, a, n, H.MPI_FLOAT, H.MPI_SUM))
        ts.append(time.perf_counter() - t0)
    ts.sort()
    pg = redop.get_pageable()
    pinned = torch.empty(n * 4, dtype=torch.uint8).pin_memory().numpy()
    # the pinned zero-copy call on the same bytes (the target: >= 0.9 x its rate)
    pa = torch.from_numpy(pinned).view(torch.float32)
    pb = torch.empty(n, dtype=torch.float32).pin_memory()
    redop.check(redop.MPI_Reduce_local(pb, pa, n, H.MPI_FLOAT, H.MPI_SUM))
    tp = []
    for _ in range(3):
        t0 = time.perf_counter()
        redop.check(redop.MPI_Reduce_local(pb, pa, n, H.MPI_FLOAT, H.MPI_SUM))
        tp.append(time.perf_counter() - t0)
    pinned_ms = min(tp) * 1e3
    del pb
    W = pg['threads']
    out = dict(bytes=4 * n, W=W, chunk_MiB=pg['chunk_bytes'] >> 20, db=os.environ.get('MPIX_REDOP_PAGEABLE_DB', '1'),
               aff=os.environ.get('MPIX_REDOP_PAGEABLE_AFFINITY', 'none'),
               nt=os.environ.get('MPIX_REDOP_PAGEABLE_NT', '1'),
               mode=os.environ.get('MPIX_REDOP_PAGEABLE_MODE', 'worker'),
               ms=round(ts[len(ts) // 2] * 1e3, 2), best_ms=round(ts[0] * 1e3, 2),
               GiBs=round(3 * n * 4 / ts[len(ts) // 2] / (1 << 30), 2), checked=ok,
               memcpy_1thread_GBs=memcpy_rate(b, pinned, 1),
               memcpy_W_GBs=memcpy_rate(b, pinned, W))
    # PCIe floor of the call's traffic
    d = torch.empty(n, dtype=torch.float32, device='cuda')
    h = torch.from_numpy(pinned).view(torch.float32)
    torch.cuda.synchronize()
    rates = {}
    for name, fn in (('h2d', lambda: d.copy_(h, non_blocking=True)),
                     ('d2h', lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        rates[name] = (time.perf_counter() - t0) / 3
    floor = max(2 * rates['h2d'], rates['d2h'])
    out.update(pcie_floor_ms=round(floor * 1e3, 2), frac_of_pcie=round(floor / (out['ms'] / 1e3), 4),
               pinned_call_ms=round(pinned_ms, 2), vs_pinned=round(pinned_ms / out['ms'], 4))
    print(json.dumps(out), flush=True)


def sweep(path):
    with open(path, 'w') as f:
        for cfg in CONFIGS:
            W, ck, db, aff = cfg[:4]
            nt = cfg[4] if len(cfg) > 4 else 1
            mode = cfg[5] if len(cfg) > 5 else 'worker'
            env = dict(os.environ, MPIX_REDOP_PAGEABLE_THREADS=str(W), MPIX_REDOP_PAGEABLE_MODE=mode,
                       MPIX_REDOP_PAGEABLE_CHUNK=str(ck << 20), MPIX_REDOP_PAGEABLE_DB=str(db),
                       MPIX_REDOP_PAGEABLE_AFFINITY=aff, MPIX_REDOP_PAGEABLE_NT=str(nt),
                       MPIX_REDOP_PIPE_TRACE='1')
            p = subprocess.run([sys.executable, __file__, 'one'], env=env, capture_output=True,
                               text=True, timeout=300)
            if p.returncode == 0 and p.stdout.strip():
                d = json.loads(p.stdout.strip().splitlines()[-1])
                d['trace_last_call'] = trace_summary(p.stderr)
                line = json.dumps(d)
            else:
                line = json.dumps(dict(W=W, chunk_MiB=ck, db=db, aff=aff, error=p.stderr[-500:]))
            f.write(line + '\n')
            f.flush()
            print(line, flush=True)


if __name__ == '__main__':
    if sys.argv[1] == 'one':
        one()
    else:
        sweep(sys.argv[2])
