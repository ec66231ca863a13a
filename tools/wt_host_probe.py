#!/usr/bin/env python3
"""Host-resident 1 GiB fp32 SUM calls (page-locked zero-copy, and pageable
through the wave form) under store policies (XCD masks) set in one process,
interleaved: does the contiguous kernel's store policy matter when the
stores go to host memory over PCIe?

usage: wt_host_probe.py OUT.json"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402


def main(path):
    n = 1 << 28
    hin = torch.empty(n, dtype=torch.float32).pin_memory().uniform_(-1, 1)
    hio = torch.empty(n, dtype=torch.float32).pin_memory().uniform_(-1, 1)
    pin = np.random.default_rng(7).random(n, dtype=np.float32)
    pio = np.random.default_rng(8).random(n, dtype=np.float32)
    redop.check(redop.MPI_Reduce_local(hin, hio, n, H.MPI_FLOAT, H.MPI_SUM))
    redop.check(redop.MPI_Reduce_local(pin, pio, n, H.MPI_FLOAT, H.MPI_SUM))
    masks = (0, 0x88, 0xff)
    res = {('%#x' % m): {'pinned_ms': [], 'pageable_ms': []} for m in masks}
    for _ in range(3):
        for m in masks:
            redop.check(redop.set_store_policy(m, 0, 0, 0))
            for key, (a, b) in (('pinned_ms', (hin, hio)), ('pageable_ms', (pin, pio))):
                t0 = time.perf_counter()
                for _ in range(2):
                    redop.check(redop.MPI_Reduce_local(a, b, n, H.MPI_FLOAT, H.MPI_SUM))
                res['%#x' % m][key].append((time.perf_counter() - t0) / 2 * 1e3)
    redop.check(redop.set_store_policy(0x88, 0, 0, 0))
    out = {m: {k: round(sorted(v)[1], 2) for k, v in d.items()} for m, d in res.items()}
    json.dump(dict(what='host-resident 1 GiB fp32 SUM per call (median of 3 rounds x 2 calls) by store policy',
                   ms=out), open(path, 'w'), indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main(sys.argv[1])
