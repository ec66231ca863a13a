"""Property-based schedule parity for libmpix_coll.so (hypothesis,
derandomised): random world sizes, ragged and empty counts, roots, types
(including the MPI_2INT MAXLOC pair) and algorithms, the C++ schedules on the
host transport with the oracle as the combine, against the oracle's
single-process simulations of the reference schedules
(reduce_scatter_intra_{recursive_halving,pairwise}.c,
allreduce_intra_{reduce_scatter_allgather,recursive_doubling,ring}.c,
reduce_intra_{binomial,reduce_scatter_gather}.c,
{scan,exscan}_intra_recursive_doubling.c).  Bit-for-bit: any index or
ordering slip in a schedule changes the fp association or the MAXLOC winner.

GPU: the same properties on the device transport with the HIP combine, P
ranks as threads on cuda:0, counts large enough for the packet kernels.
"""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tests.test_coll_c import MPI_2INT, MPI_DOUBLE, MPI_FLOAT, MPI_INT, MPI_BXOR, MPI_MAX, \
    MPI_MAXLOC, MPI_SUM, _dev_comms, free_all, host_comms, run_ranks

CASES = [(MPI_FLOAT, MPI_SUM, 4), (MPI_DOUBLE, MPI_MAX, 8), (MPI_INT, MPI_BXOR, 4),
         (MPI_2INT, MPI_MAXLOC, 8)]

SETTINGS = settings(max_examples=100, derandomize=True, deadline=None,
                    suppress_health_check=[HealthCheck.function_scoped_fixture,
                                           HealthCheck.too_slow])


def _inputs(P, n, case, seed):
    """P operands of n elements as bytes; doubles carry NaN / +-0, pairs
    carry value ties"""
    dt, op, ext = case
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(P):
        if dt == MPI_FLOAT:
            a = rng.uniform(-1, 1, n).astype(np.float32)
        elif dt == MPI_DOUBLE:
            a = rng.uniform(-1, 1, n)
            k = rng.random(n)
            a[k < 0.05] = np.nan
            a[(k >= 0.05) & (k < 0.1)] = 0.0
            a[(k >= 0.1) & (k < 0.15)] = -0.0
        elif dt == MPI_INT:
            a = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        else:
            a = np.stack([rng.integers(0, 4, n), rng.integers(-50, 50, n)], 1).astype(np.int32)
        out.append(np.ascontiguousarray(a).view(np.uint8).reshape(-1))
    return out


@SETTINGS
@given(P=st.integers(1, 12), case=st.sampled_from(CASES),
       algo=st.sampled_from(['recursive_halving', 'pairwise', 'pairwise_sequential',
                             'pairwise_pipelined', 'pull', 'recursive_halving_pull']),
       in_place=st.booleans(), data=st.data(), seed=st.integers(0, 2**31))
def test_reduce_scatter_random(oracle, P, case, algo, in_place, data, seed):
    from mpich_amd import ccl
    dt, op, ext = case
    counts = data.draw(st.lists(st.integers(0, 90), min_size=P, max_size=P))
    total = sum(counts)
    sends = _inputs(P, total, case, seed)
    sim = 'recursive_halving' if algo.startswith('recursive_halving') else 'pairwise'
    exp = oracle.rs_schedule(sends, counts, dt, op, sim)
    comms = host_comms(P, oracle)
    bufs = [s.copy() if in_place else np.zeros(max(1, counts[r]) * ext, np.uint8)
            for r, s in enumerate(sends)]
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(
        None if in_place else sends[r], bufs[r], counts, dt, op, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert bufs[r][:counts[r] * ext].tobytes() == exp[r].tobytes(), r


@SETTINGS
@given(P=st.integers(1, 12), case=st.sampled_from(CASES),
       algo=st.sampled_from(['reduce_scatter_allgather', 'rsag_rd_allgather',
                             'recursive_doubling', 'ring', 'rsag_multipath', 'pull']),
       count=st.integers(1, 200), seed=st.integers(0, 2**31))
def test_allreduce_random(oracle, P, case, algo, count, seed):
    from mpich_amd import ccl
    dt, op, ext = case
    pof2 = 1 << (P.bit_length() - 1)
    if (algo.startswith('r') or algo == 'pull') and algo != 'recursive_doubling' and \
            count < pof2:
        count = pof2            # the reference asserts count >= pof2 there
    sends = _inputs(P, count, case, seed)
    sim = algo if algo in ('recursive_doubling', 'ring') else 'reduce_scatter_allgather'
    exp = oracle.allreduce_rabenseifner(sends, count, dt, op, algorithm=sim)
    comms = host_comms(P, oracle)
    outs = [np.zeros(count * ext, np.uint8) for _ in range(P)]
    rcs = run_ranks(comms, lambda r, c: ccl.allreduce(sends[r], outs[r], count, dt, op, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert outs[r].tobytes() == exp[r].tobytes(), r


@SETTINGS
@given(P=st.integers(1, 12), case=st.sampled_from(CASES),
       algo=st.sampled_from(['binomial', 'reduce_scatter_gather']),
       count=st.integers(1, 200), data=st.data(), in_place=st.booleans(),
       seed=st.integers(0, 2**31))
def test_reduce_random(oracle, P, case, algo, count, data, in_place, seed):
    from mpich_amd import ccl
    dt, op, ext = case
    pof2 = 1 << (P.bit_length() - 1)
    if algo == 'reduce_scatter_gather' and count < pof2:
        count = pof2
    root = data.draw(st.integers(0, P - 1))
    sends = _inputs(P, count, case, seed)
    exp = oracle.reduce_schedule(sends, count, dt, op, root, algo)
    comms = host_comms(P, oracle)
    out = sends[root].copy() if in_place else np.zeros(count * ext, np.uint8)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce(
        None if (in_place and r == root) else sends[r], out if r == root else None,
        count, dt, op, root, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    assert out.tobytes() == exp.tobytes()


@SETTINGS
@given(P=st.integers(1, 12), case=st.sampled_from(CASES), exclusive=st.booleans(),
       count=st.integers(1, 200), in_place=st.booleans(), seed=st.integers(0, 2**31))
def test_scan_random(oracle, P, case, exclusive, count, in_place, seed):
    from mpich_amd import ccl
    dt, op, ext = case
    sends = _inputs(P, count, case, seed)
    prior = [np.full(count * ext, 7, np.uint8) for _ in range(P)]
    outs = [s.copy() if in_place else p.copy() for s, p in zip(sends, prior)]
    exp = [o.copy() for o in outs]
    oracle.scan_schedule(sends, exp, count, dt, op, exclusive)
    comms = host_comms(P, oracle)
    rcs = run_ranks(comms, lambda r, c: ccl.scan(None if in_place else sends[r], outs[r], count,
                                                 dt, op, c, exclusive))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert outs[r].tobytes() == exp[r].tobytes(), r


GPU_SETTINGS = settings(max_examples=int(os.environ.get('MPIX_FUZZ_EXAMPLES_COLL', 25)),
                        derandomize=not os.environ.get('MPIX_FUZZ_RANDOM'), deadline=None,
                        suppress_health_check=[HealthCheck.function_scoped_fixture,
                                               HealthCheck.too_slow])


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.gpu
@GPU_SETTINGS
@given(P=st.integers(2, 8), case=st.sampled_from(CASES),
       algo=st.sampled_from(['recursive_halving', 'pairwise', 'pairwise_sequential',
                             'pairwise_pipelined', 'pull', 'recursive_halving_pull']),
       in_place=st.booleans(), data=st.data(), seed=st.integers(0, 2**31))
def test_reduce_scatter_random_device(oracle, P, case, algo, in_place, data, seed):
    import torch
    from mpich_amd import ccl
    dt, op, ext = case
    counts = data.draw(st.lists(st.integers(0, 6000), min_size=P, max_size=P))
    sends = _inputs(P, sum(counts), case, seed)
    sim = 'recursive_halving' if algo.startswith('recursive_halving') else 'pairwise'
    exp = oracle.rs_schedule(sends, counts, dt, op, sim)
    dsend = [_dev(s) for s in sends]
    bufs = [_dev(s) if in_place else torch.zeros(max(1, counts[r]) * ext, dtype=torch.uint8,
                                                  device='cuda') for r, s in enumerate(sends)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(
        None if in_place else dsend[r], bufs[r], counts, dt, op, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert bufs[r][:counts[r] * ext].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@GPU_SETTINGS
@given(P=st.integers(2, 8), case=st.sampled_from(CASES),
       algo=st.sampled_from(['reduce_scatter_allgather', 'rsag_rd_allgather',
                             'recursive_doubling', 'ring', 'rsag_multipath', 'pull']),
       count=st.integers(1, 20000), seed=st.integers(0, 2**31))
def test_allreduce_random_device(oracle, P, case, algo, count, seed):
    import torch
    from mpich_amd import ccl
    dt, op, ext = case
    pof2 = 1 << (P.bit_length() - 1)
    if (algo.startswith('r') or algo == 'pull') and algo != 'recursive_doubling' and \
            count < pof2:
        count = pof2
    sends = _inputs(P, count, case, seed)
    sim = algo if algo in ('recursive_doubling', 'ring') else 'reduce_scatter_allgather'
    exp = oracle.allreduce_rabenseifner(sends, count, dt, op, algorithm=sim)
    dsend = [_dev(s) for s in sends]
    outs = [torch.zeros(count * ext, dtype=torch.uint8, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.allreduce(dsend[r], outs[r], count, dt, op, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert outs[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@GPU_SETTINGS
@given(P=st.integers(2, 8), case=st.sampled_from(CASES),
       algo=st.sampled_from(['binomial', 'reduce_scatter_gather']),
       count=st.integers(1, 20000), data=st.data(), seed=st.integers(0, 2**31))
def test_reduce_random_device(oracle, P, case, algo, count, data, seed):
    import torch
    from mpich_amd import ccl
    dt, op, ext = case
    pof2 = 1 << (P.bit_length() - 1)
    if algo == 'reduce_scatter_gather' and count < pof2:
        count = pof2
    root = data.draw(st.integers(0, P - 1))
    sends = _inputs(P, count, case, seed)
    exp = oracle.reduce_schedule(sends, count, dt, op, root, algo)
    dsend = [_dev(s) for s in sends]
    out = torch.zeros(count * ext, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce(dsend[r], out if r == root else None, count,
                                                   dt, op, root, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    assert out.cpu().numpy().tobytes() == exp.tobytes()


@pytest.mark.gpu
@GPU_SETTINGS
@given(P=st.integers(2, 8), case=st.sampled_from(CASES), exclusive=st.booleans(),
       count=st.integers(1, 20000), seed=st.integers(0, 2**31))
def test_scan_random_device(oracle, P, case, exclusive, count, seed):
    import torch
    from mpich_amd import ccl
    dt, op, ext = case
    sends = _inputs(P, count, case, seed)
    exp = [np.full(count * ext, 7, np.uint8) for _ in range(P)]
    oracle.scan_schedule(sends, exp, count, dt, op, exclusive)
    dsend = [_dev(s) for s in sends]
    outs = [torch.full((count * ext,), 7, dtype=torch.uint8, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.scan(dsend[r], outs[r], count, dt, op, c, exclusive))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert outs[r].cpu().numpy().tobytes() == exp[r].tobytes(), r
