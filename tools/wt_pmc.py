#!/usr/bin/env python3
"""A short command to profile: 8 launches of the 1 GiB fp32 SUM contiguous
kernel (MPIX_Reduce_local_async) under the store policy given as an XCD mask
(MPIX_Redop_set_store_policy), for rocprofv3 --pmc passes comparing the
policy's memory-side counters (tools/gpu_wt_pmc.sh).

usage: wt_pmc.py XCD_MASK"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402


def main(mask):
    n = 1 << 28
    a = torch.empty(n, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    b = torch.empty(n, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    torch.cuda.synchronize()
    redop.check(redop.set_store_policy(mask, 0, 0, 0))
    s = torch.cuda.current_stream()
    for _ in range(8):
        redop.check(redop.reduce_local_async(b, a, n, H.MPI_FLOAT, H.MPI_SUM, s))
    torch.cuda.synchronize()


if __name__ == '__main__':
    main(int(sys.argv[1], 0))
