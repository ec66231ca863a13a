#!/usr/bin/env python3
"""Is the pageable workers' GPU side slower than the one-kernel pinned call
because of the chunking itself?  On PINNED 1 GiB operands (no host memcpy at
all): one synchronous MPIX_Reduce_local over the whole buffers, then the same
bytes as 16 MiB chunks issued by T threads concurrently (each a synchronous
call on its own slice, as a pageable worker does after its copy-in).  Also
where the memory sits: the NUMA nodes of the numpy (pageable) and torch
(pinned) buffers from /proc/self/numa_maps, and the GPU's own NUMA node.

usage: pinned_chunk_probe.py OUT.json"""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402


def numa_of(addr):
    """{node: pages} of the VMA containing addr"""
    for line in open('/proc/self/numa_maps'):
        parts = line.split()
        start = int(parts[0], 16)
        # numa_maps has no end address: take the page count fields and check
        # the range with /proc/self/maps
        for m in open('/proc/self/maps'):
            a, b = m.split()[0].split('-')
            if int(a, 16) == start:
                if start <= addr < int(b, 16):
                    return {p.split('=')[0]: int(p.split('=')[1]) for p in parts
                            if p.startswith('N') and '=' in p}
                break
    return None


def gpu_numa():
    p = torch.cuda.get_device_properties(0)
    bus = '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    try:
        return bus, int(open('/sys/bus/pci/devices/%s/numa_node' % bus).read()), \
            open('/sys/bus/pci/devices/%s/local_cpulist' % bus).read().strip()
    except OSError as e:
        return bus, None, str(e)


def main():
    n = 1 << 28
    out = dict(gpu=gpu_numa())
    hin = torch.empty(n, dtype=torch.float32).pin_memory()
    hio = torch.empty(n, dtype=torch.float32).pin_memory()
    hin.uniform_(-1, 1)
    hio.uniform_(-1, 1)
    pg = np.random.default_rng(1).random(n, dtype=np.float32)
    out['numa_pinned'] = numa_of(hin.data_ptr())
    out['numa_pageable'] = numa_of(pg.ctypes.data)
    redop.check(redop.MPI_Reduce_local(hin, hio, n, H.MPI_FLOAT, H.MPI_SUM))
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        redop.check(redop.MPI_Reduce_local(hin, hio, n, H.MPI_FLOAT, H.MPI_SUM))
        ts.append(time.perf_counter() - t0)
    out['pinned_one_call_ms'] = round(min(ts) * 1e3, 2)
    L = redop.lib()
    sizes = [int(x) for x in os.environ.get('CHUNK_MIB', '16').split(',')]
    threads = [int(x) for x in os.environ.get('CHUNK_T', '1,2,4,8').split(',')]
    for mib, T in [(m, t) for m in sizes for t in threads]:
        chunk = (mib << 20) // 4
        def work(t):
            for off in range(t * chunk, n, T * chunk):
                m = min(chunk, n - off)
                L.MPIX_Reduce_local(hin.data_ptr() + 4 * off, hio.data_ptr() + 4 * off, m,
                                    H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM))
        best = None
        for _ in range(3):
            ths = [threading.Thread(target=work, args=(t,)) for t in range(T)]
            t0 = time.perf_counter()
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        out['pinned_%dMiB_chunks_T%d_ms' % (mib, T)] = round(best * 1e3, 2)
    print(json.dumps(out))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
