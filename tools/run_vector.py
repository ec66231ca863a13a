#!/usr/bin/env python3
"""Five launches of the config-5 vector-target kernel
(vector(67108864, 1, 2, MPI_DOUBLE) SUM) -- a short command to profile."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

cnt = 67108864
src = torch.rand(cnt, dtype=torch.float64, device='cuda')
dst = torch.rand(2 * cnt, dtype=torch.float64, device='cuda')
torch.cuda.synchronize()
for _ in range(5):
    redop.check(redop.reduce_local_vector(src, dst, cnt, 1, 2, H.MPI_DOUBLE, H.MPI_SUM))
torch.cuda.synchronize()
print('ok')
