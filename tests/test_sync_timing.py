"""MPIX_Redop_sync_timing: the kernel timing bench.py's roofline figure is
read from -- a HIP event pair the library records around the launch of each
of the next n synchronous calls on its own stream.  The CPU part checks the
arguments (rejected before any HIP call); the GPU part that exactly n calls
are recorded, that the durations are a kernel's, and that the recording
changes neither the result nor the calls after it."""
import ctypes

import numpy as np
import pytest
import torch

from mpich_amd import redop
from mpich_amd import handles as H


def test_sync_timing_arguments():
    L = redop.lib()
    got = ctypes.c_int(-7)
    buf = (ctypes.c_float * 4)()
    assert L.MPIX_Redop_sync_timing(-1, 4) != 0
    assert L.MPIX_Redop_sync_timing(64, 4) != 0
    assert L.MPIX_Redop_sync_timing(0, -1) != 0
    assert L.MPIX_Redop_sync_timing(0, (1 << 16) + 1) != 0
    assert L.MPIX_Redop_sync_timing_read(-1, buf, 4, ctypes.byref(got)) != 0
    assert L.MPIX_Redop_sync_timing_read(0, buf, 4, None) != 0
    assert L.MPIX_Redop_sync_timing_read(0, None, 4, ctypes.byref(got)) != 0
    assert L.MPIX_Redop_sync_timing_read(0, buf, -1, ctypes.byref(got)) != 0
    assert got.value == -7


@pytest.mark.gpu
def test_sync_timing_records_exactly_n_calls():
    dev = torch.device('cuda:0')
    n = (1 << 22) + 5
    g = torch.Generator(device=dev)
    g.manual_seed(0x7117)
    a = torch.rand(n, device=dev, generator=g)
    b0 = torch.rand(n, device=dev, generator=g)
    b = b0.clone()
    redop.sync_timing(0, 3)
    for _ in range(5):
        redop.check(redop.MPI_Reduce_local(a, b, n, H.MPI_FLOAT, H.MPI_SUM))
    ms = redop.sync_timing_read(0)
    assert len(ms) == 3
    # a 48 MiB pass: tens of microseconds, not the host's seconds
    assert all(0.0 < t < 50.0 for t in ms), ms
    # the result: five in-order sums, the recording changed nothing
    ref = b0.cpu().numpy().copy()
    an = a.cpu().numpy()
    for _ in range(5):
        ref = (ref + an).astype(np.float32)
    assert np.array_equal(b.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    # stopped: nothing more is recorded
    redop.check(redop.MPI_Reduce_local(a, b, n, H.MPI_FLOAT, H.MPI_SUM))
    assert redop.sync_timing_read(0) == []
    # 0 stops a recording before its calls
    redop.sync_timing(0, 4)
    redop.sync_timing(0, 0)
    redop.check(redop.MPI_Reduce_local(a, b, n, H.MPI_FLOAT, H.MPI_SUM))
    assert redop.sync_timing_read(0) == []
