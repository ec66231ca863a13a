"""libmpix_coll.so -- the C++ restatement of MPICH's reduce-scatter,
allreduce, reduce and scan schedules (include/mpix_coll.h) -- driven with P
in-process ranks, one thread each.

CPU: the host-memory transport with the oracle installed as the combine
(the product has no CPU compute path), checked bit-for-bit against the
oracle's single-process simulation of the reference schedules
(reduce_scatter_block_intra_recursive_halving.c:38-260, …_pairwise.c:42-104,
allreduce_intra_reduce_scatter_allgather.c:41-277,
allreduce_intra_recursive_doubling.c:24-150), against the redscatblk3.c
closed form and against every allred.c KAT generated for that world size.

GPU: the device transport (stream-ordered device-to-device copies with event
hand-offs) and the HIP combine, all ranks on cuda:0 -- the same schedules
with the product kernels, bit-identical to the oracle's simulation.
"""
import ctypes
import os
import threading

import numpy as np
import pytest

from tests import golden_util as gu

MPI_FLOAT, MPI_DOUBLE, MPI_INT = 0x4c00040a, 0x4c00080b, 0x4c000405
MPI_2INT = 0x4c000816
MPI_MIN = 0x58000002
MPI_SUM, MPI_PROD, MPI_MAX, MPI_BXOR, MPI_MAXLOC = 0x58000003, 0x58000004, 0x58000001, \
    0x5800000a, 0x5800000c


def run_ranks(comms, fn, timeout=120):
    """fn(rank, comm) on one thread per rank (ctypes drops the GIL inside the
    C calls, so the ranks really run concurrently); returns fn's results"""
    out = [None] * len(comms)

    def body(r):
        try:
            out[r] = fn(r, comms[r])
        except BaseException as e:      # noqa: B902 -- reported below
            out[r] = e
    # daemon threads: a rank stuck in a C call must not keep the process alive
    ths = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(len(comms))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
        assert not t.is_alive(), 'rank thread hung'
    for r, x in enumerate(out):
        if isinstance(x, BaseException):
            raise AssertionError('rank %d: %r' % (r, x))
    return out


def host_comms(P, oracle):
    from mpich_amd import ccl
    comms = ccl.comm_create_local(P)
    for c in comms:
        c.set_combine(oracle.combine_fn_address())
    return comms


def free_all(comms):
    for c in comms:
        assert c.free() == 0


def float_sends(P, n, seed=0x5EED0100):
    return [np.random.default_rng(seed + r).uniform(-1, 1, n).astype(np.float32)
            for r in range(P)]


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential'])
@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 7, 8, 13, 16])
def test_rsb_host_matches_oracle_schedule(oracle, P, algo):
    from mpich_amd import ccl
    recvcount = 1001
    sends = float_sends(P, P * recvcount)
    recvs = [np.zeros(recvcount, np.float32) for _ in range(P)]
    comms = host_comms(P, oracle)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(sends[r], recvs[r], recvcount,
                                                                  MPI_FLOAT, MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    sim = oracle.rsb_pairwise if algo.startswith('pairwise') else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('recvcount', [1, 7, 1001, (1 << 24) // 4 + 5])
@pytest.mark.parametrize('P', [2, 3, 4, 8, 16])
def test_rsb_multipath_host_matches_recursive_halving(oracle, P, recvcount):
    """MPIX_RSB_RECURSIVE_HALVING_MULTIPATH: the recursive-halving schedule
    with every step's half spread over all links through relays (P a power of
    two >= 4; other P fall back to plain recursive halving) -- bit-identical
    to the oracle's recursive-halving simulation, also with blocks large
    enough for the relay hops to be pipelined in several chunks"""
    from mpich_amd import ccl
    if recvcount > 100000 and P > 8:
        pytest.skip('large blocks at P = 2..8 only (memory)')
    sends = float_sends(P, P * recvcount, seed=0x5EED0E00)
    recvs = [np.zeros(recvcount, np.float32) for _ in range(P)]
    comms = host_comms(P, oracle)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
        sends[r], recvs[r], recvcount, MPI_FLOAT, MPI_SUM, c, 'recursive_halving_multipath'))
    free_all(comms)
    assert rcs == [0] * P
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT,
                                       MPI_SUM)
    for r in range(P):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'auto',
                                  'recursive_halving_multipath', 'recursive_halving_pull'])
@pytest.mark.parametrize('P', [2, 3, 4, 6, 8])
def test_rsb_host_redscatblk3(oracle, P, algo):
    """redscatblk3.c:43-56: block i of rank r holds r + i; the result on rank
    r is P*r + P*(P-1)/2 everywhere"""
    from mpich_amd import ccl
    recvcount = (1 << 20) // P // 64
    sends = [np.concatenate([np.full(recvcount, r + i, np.int32) for i in range(P)])
             for r in range(P)]
    recvs = [np.zeros(recvcount, np.int32) for _ in range(P)]
    comms = host_comms(P, oracle)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(sends[r], recvs[r], recvcount,
                                                                  MPI_INT, MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    for r in range(P):
        assert np.all(recvs[r] == P * r + P * (P - 1) // 2), r


@pytest.mark.parametrize('algo', ['reduce_scatter_allgather', 'rsag_rd_allgather',
                                  'recursive_doubling', 'ring', 'rsag_multipath', 'pull'])
@pytest.mark.parametrize('P', [1, 2, 3, 4, 7, 8, 12, 16])
def test_allreduce_host_matches_oracle_and_kats(oracle, P, algo):
    from mpich_amd import ccl
    count = 1037
    sends = float_sends(P, count, 0x5EED0200)
    recvs = [np.zeros(count, np.float32) for _ in range(P)]
    comms = host_comms(P, oracle)
    rcs = run_ranks(comms, lambda r, c: ccl.allreduce(sends[r], recvs[r], count, MPI_FLOAT,
                                                       MPI_SUM, c, algo))
    assert rcs == [0] * P
    exp = oracle.allreduce_rabenseifner(
        [s.view(np.uint8) for s in sends], count, MPI_FLOAT, MPI_SUM,
        algorithm=algo if algo in ('recursive_doubling', 'ring') else 'reduce_scatter_allgather')
    for r in range(P):
        assert recvs[r].tobytes() == exp[r].tobytes(), r
    # the allred.c KATs generated for this world size, every op and type
    pof2 = 1 << (P.bit_length() - 1)
    ncase = 0
    for case in gu.load_cases():
        if case['nranks'] != P or not case['name'].startswith('allred '):
            continue
        if algo not in ('recursive_doubling', 'ring') and case['count'] < pof2:
            continue
        ext = len(case['expected']) // case['count']
        outs = [np.zeros(case['count'] * ext, np.uint8) for _ in range(P)]
        ins = [np.ascontiguousarray(case['inputs'][r]) for r in range(P)]
        rcs = run_ranks(comms, lambda r, c: ccl.allreduce(ins[r], outs[r], case['count'],
                                                           case['datatype'], case['op'], c, algo))
        assert rcs == [0] * P, case['id']
        for r in range(P):
            assert not gu.mismatches(case, outs[r]), (case['id'], r)
        ncase += 1
    free_all(comms)
    if P in (4, 7):
        assert ncase > 0


@pytest.mark.parametrize('P', [2, 3, 5, 8])
def test_allreduce_ring_ragged_and_auto_rule(oracle, P):
    """the ring with counts that leave short and empty blocks (fp64 MAX over
    NaN / +-0: every step's operand order shows), and the generic.json:114-117
    rule: up to 8 bytes the auto choice is recursive doubling even at
    count >= pof2"""
    from mpich_amd import ccl
    comms = host_comms(P, oracle)
    for count in (1, P - 1, P + 1, 3 * P - 2, 1000):
        sends = _special_doubles(P, count, count)
        outs = [np.zeros(count) for _ in range(P)]
        rcs = run_ranks(comms, lambda r, c: ccl.allreduce(sends[r], outs[r], count, MPI_DOUBLE,
                                                           MPI_MAX, c, 'ring'))
        assert rcs == [0] * P
        exp = oracle.allreduce_rabenseifner([s.view(np.uint8) for s in sends], count, MPI_DOUBLE,
                                            MPI_MAX, algorithm='ring')
        for r in range(P):
            assert outs[r].view(np.uint8).tobytes() == exp[r].tobytes(), (count, r)
    pof2 = 1 << (P.bit_length() - 1)
    for count in (max(1, 8 // 8), pof2):        # 8 bytes -> recursive doubling; > 8 -> RSAG
        sends = _special_doubles(P, count, 77 + count)
        outs = [np.zeros(count) for _ in range(P)]
        rcs = run_ranks(comms, lambda r, c: ccl.allreduce(sends[r], outs[r], count, MPI_DOUBLE,
                                                           MPI_MAX, c, 'auto'))
        assert rcs == [0] * P
        algo = 'recursive_doubling' if count * 8 <= 8 or count < pof2 else \
            'reduce_scatter_allgather'
        exp = oracle.allreduce_rabenseifner([s.view(np.uint8) for s in sends], count, MPI_DOUBLE,
                                            MPI_MAX, algorithm=algo)
        for r in range(P):
            assert outs[r].view(np.uint8).tobytes() == exp[r].tobytes(), (count, r)
    free_all(comms)


@pytest.mark.parametrize('P,count', [(4, 4096), (8, 4096), (16, 4096), (8, 1 << 22),
                                     (4, 4098), (8, 8), (6, 4096)])
def test_allreduce_rsag_multipath_matches_oracle(oracle, P, count):
    """MPIX_ALLREDUCE_RSAG_MULTIPATH: every reduce-scatter step spread over all
    links through relays when P is a power of two >= 4 and count a multiple
    of P (chunked relay hops at 16 MiB); ragged counts, tiny counts and
    non-power-of-two P run the plain steps -- same bits in every case"""
    from mpich_amd import ccl
    sends = float_sends(P, count, 0x5EED0A00 + count)
    outs = [np.zeros(count, np.float32) for _ in range(P)]
    comms = host_comms(P, oracle)
    rcs = run_ranks(comms, lambda r, c: ccl.allreduce(sends[r], outs[r], count, MPI_FLOAT,
                                                       MPI_SUM, c, 'rsag_multipath'))
    free_all(comms)
    assert rcs == [0] * P
    exp = oracle.allreduce_rabenseifner([s.view(np.uint8) for s in sends], count, MPI_FLOAT,
                                        MPI_SUM, algorithm='reduce_scatter_allgather')
    for r in range(P):
        assert outs[r].tobytes() == exp[r].tobytes(), r


def test_allreduce_rsag_multipath_uses_every_link(oracle):
    """the exchange trace (MPIX_COLL_TRACE) of rank 0 at P = 8: the multipath
    reduce-scatter steps post to all 7 peers, the plain ones to one partner"""
    import subprocess
    import sys
    code = r'''
import threading, numpy as np
from mpich_amd import ccl, handles as H
from oracle import oracle as O
import sys
P, count, algo = 8, 4096, sys.argv[1]
comms = ccl.comm_create_local(P)
for c in comms:
    c.set_combine(O.combine_fn_address())
sends = [np.full(count, r, np.float32) for r in range(P)]
outs = [np.zeros(count, np.float32) for _ in range(P)]
ts = [threading.Thread(target=lambda r=r: ccl.allreduce(sends[r], outs[r], count, H.MPI_FLOAT,
                                                         H.MPI_SUM, comms[r], algo))
      for r in range(P)]
[t.start() for t in ts]
[t.join() for t in ts]
assert all(np.all(o == 28) for o in outs)
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    peers = {}
    for algo in ('reduce_scatter_allgather', 'rsag_multipath'):
        p = subprocess.run([sys.executable, '-c', code, algo], capture_output=True, text=True,
                           cwd=root, env=dict(os.environ, MPIX_COLL_TRACE='1'), timeout=120)
        assert p.returncode == 0, p.stderr[-3000:]
        lines = [ln for ln in p.stderr.splitlines() if ln.startswith('[mpix_coll rank 0/8]')]
        steps = [{int(t[1:].split(':')[0]) for t in ln.split(']')[1].split()} for ln in lines]
        peers[algo] = steps
    # plain: 3 reduce-scatter steps with one partner each, one allgather group to all
    assert [len(s) for s in peers['reduce_scatter_allgather']] == [1, 1, 1, 7]
    # multipath (one chunk at this size): per step, the partner and the 3
    # relays first, then the 3 relayed second hops -- all 7 links per step
    rs = peers['rsag_multipath'][:-1]
    assert len(rs) == 6, peers['rsag_multipath']
    for k in range(3):
        assert len(rs[2 * k]) == 4 and len(rs[2 * k + 1]) == 3
        assert len(rs[2 * k] | rs[2 * k + 1]) == 7
    assert len(peers['rsag_multipath'][-1]) == 7


def test_in_place_allreduce_and_workspace(oracle):
    """MPI_IN_PLACE (sendbuf None) and a caller-provided workspace"""
    import torch
    from mpich_amd import ccl
    P, count = 4, 4099
    sends = float_sends(P, count, 7)
    bufs = [s.copy() for s in sends]
    comms = host_comms(P, oracle)
    need = ccl.allreduce_workspace_bytes(count, MPI_FLOAT, comms[0])
    assert need >= count * 4
    wss = [torch.zeros(need, dtype=torch.uint8) for _ in range(P)]
    rcs = run_ranks(comms, lambda r, c: ccl.allreduce(None, bufs[r], count, MPI_FLOAT, MPI_SUM, c,
                                                       workspace=wss[r]))
    assert rcs == [0] * P
    exp = oracle.allreduce_rabenseifner([s.view(np.uint8) for s in sends], count, MPI_FLOAT,
                                        MPI_SUM)
    for r in range(P):
        assert bufs[r].tobytes() == exp[r].tobytes()
    # a too-small workspace is an argument error, detected before any exchange
    small = torch.zeros(16, dtype=torch.uint8)
    assert ccl.allreduce(None, bufs[0], count, MPI_FLOAT, MPI_SUM, comms[0], workspace=small) == 12
    free_all(comms)


@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential'])
@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 8])
def test_rsb_host_in_place(oracle, P, algo):
    """MPI_IN_PLACE (sendbuf NULL): recvbuf holds the P*recvcount inputs and
    gets the result in its first block.  red_scat_block.c:33-70 (recvcount 1,
    block i of rank r = r + i, sum P*r + P(P-1)/2) with and without IN_PLACE,
    and bit-identity with the oracle's simulation on floats"""
    from mpich_amd import ccl
    comms = host_comms(P, oracle)
    for in_place in (False, True):
        sends = [np.arange(r, r + P, dtype=np.int32) for r in range(P)]
        bufs = [s.copy() if in_place else np.zeros(1, np.int32) for s in sends]
        rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
            None if in_place else sends[r], bufs[r], 1, MPI_INT, MPI_SUM, c, algo))
        assert rcs == [0] * P
        for r in range(P):
            assert bufs[r][0] == P * r + P * (P - 1) // 2, (in_place, r)
    recvcount = 333
    sends = float_sends(P, P * recvcount, 11)
    bufs = [s.copy() for s in sends]
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(None, bufs[r], recvcount,
                                                                  MPI_FLOAT, MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    sim = oracle.rsb_pairwise if algo.startswith('pairwise') else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert bufs[r][:recvcount].tobytes() == exp[r].tobytes(), r


def _ragged_counts(P, seed):
    """per-rank recvcounts with zeros and uneven sizes"""
    rng = np.random.default_rng(seed)
    c = [int(x) for x in rng.integers(0, 700, P)]
    if P > 2:
        c[1] = 0
    return c


@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential',
                                  'pairwise_pipelined', 'auto'])
@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 6, 7, 8, 11, 16])
def test_reduce_scatter_host_matches_oracle(oracle, P, algo):
    """MPI_Reduce_scatter with ragged recvcounts (zeros included) against the
    oracle's simulation of reduce_scatter_intra_{recursive_halving,pairwise}.c,
    plain and MPI_IN_PLACE"""
    from mpich_amd import ccl
    counts = _ragged_counts(P, 100 + P)
    total = sum(counts)
    sends = float_sends(P, total, 0x5EED0400)
    comms = host_comms(P, oracle)
    sim_algo = 'recursive_halving' if algo in ('recursive_halving', 'auto') and \
        total * 4 < (512 << 10) else 'pairwise'
    exp = oracle.rs_schedule([s.view(np.uint8) for s in sends], counts, MPI_FLOAT, MPI_SUM,
                             sim_algo)
    for in_place in (False, True):
        bufs = [s.copy() if in_place else np.zeros(max(1, counts[r]), np.float32)
                for r, s in enumerate(sends)]
        rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(
            None if in_place else sends[r], bufs[r], counts, MPI_FLOAT, MPI_SUM, c, algo))
        assert rcs == [0] * P
        for r in range(P):
            assert bufs[r][:counts[r]].tobytes() == exp[r].tobytes(), (in_place, r)
    free_all(comms)


@pytest.mark.parametrize('P', [4, 6, 8])
def test_reduce_scatter_redscat_kats(oracle, P):
    """redscat.c:40-55 (recvcounts 1) and redscat3.c:51-100 (1 Mi / P ints per
    rank, then MPI_IN_PLACE): block i of rank r holds r + i, result P*r +
    P(P-1)/2; the two simulations of the reference schedules agree on ragged
    integer counts too (exact arithmetic: association-free)"""
    from mpich_amd import ccl
    comms = host_comms(P, oracle)
    for mycount in (1, (1 << 20) // P):
        counts = [mycount] * P
        sends = [np.concatenate([np.full(mycount, r + i, np.int32) for i in range(P)])
                 for r in range(P)]
        for algo in ('recursive_halving', 'pairwise'):
            outs = [np.full(mycount, -1, np.int32) for _ in range(P)]
            rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(sends[r], outs[r], counts,
                                                                   MPI_INT, MPI_SUM, c, algo))
            assert rcs == [0] * P
            for r in range(P):
                assert np.all(outs[r] == P * r + P * (P - 1) // 2), (mycount, algo, r)
        bufs = [s.copy() for s in sends]
        rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(None, bufs[r], counts, MPI_INT,
                                                               MPI_SUM, c))
        assert rcs == [0] * P
        for r in range(P):
            assert np.all(bufs[r][:mycount] == P * r + P * (P - 1) // 2)
    free_all(comms)
    counts = _ragged_counts(P, 7)
    rng = np.random.default_rng(3)
    ints = [rng.integers(-1000, 1000, sum(counts)).astype(np.int32) for _ in range(P)]
    rh = oracle.rs_schedule([x.view(np.uint8) for x in ints], counts, MPI_INT, MPI_SUM)
    pw = oracle.rs_schedule([x.view(np.uint8) for x in ints], counts, MPI_INT, MPI_SUM, 'pairwise')
    offs = np.concatenate([[0], np.cumsum(counts)])
    for r in range(P):
        closed = sum(x[offs[r]:offs[r + 1]] for x in ints).astype(np.int32)
        assert rh[r].tobytes() == pw[r].tobytes() == closed.tobytes(), r


def test_argument_errors(oracle):
    from mpich_amd import ccl
    from mpich_amd import handles as H
    comms = host_comms(2, oracle)
    a = np.zeros(8, np.float32)
    b = np.zeros(4, np.float32)
    c0 = comms[0]
    assert ccl.reduce_scatter_block(a, b, -1, MPI_FLOAT, MPI_SUM, c0) == H.MPI_ERR_COUNT
    assert ccl.reduce_scatter_block(a, b, 4, MPI_FLOAT, MPI_BXOR, c0) == H.MPI_ERR_OP
    assert ccl.reduce_scatter_block(a, None, 4, MPI_FLOAT, MPI_SUM, c0) == H.MPI_ERR_BUFFER
    assert ccl.reduce_scatter_block(a, b, 4, MPI_FLOAT, MPI_SUM, c0, 9) == H.MPI_ERR_ARG
    assert ccl.reduce_scatter_block(a, b, 0, MPI_FLOAT, MPI_SUM, c0) == 0
    # the reduce-scatter+allgather allreduce needs count >= pof2 (:127)
    assert ccl.allreduce(a, a, 1, MPI_FLOAT, MPI_SUM, c0, 'reduce_scatter_allgather') == \
        H.MPI_ERR_COUNT
    assert ccl.allreduce(a, a, 8, MPI_FLOAT, MPI_SUM, c0, 7) == H.MPI_ERR_ARG
    free_all(comms)


def test_custom_transport_and_symbols(oracle):
    """MPIX_Comm_create_custom with a caller exchange function (here a
    1-rank loop that must never be called) and the exported symbol set"""
    from mpich_amd import ccl
    L = ccl.lib()
    calls = []
    XFN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_void_p)
    fn = XFN(lambda ctx, rank, ops, nops, stream: calls.append(nops) or 0)
    h = ctypes.c_void_p()
    assert L.MPIX_Comm_create_custom(0, 1, ctypes.cast(fn, ctypes.c_void_p), None, 1,
                                     ctypes.byref(h)) == 0
    c = ccl.Comm(h.value)
    c.set_combine(oracle.combine_fn_address())
    x = np.arange(10, dtype=np.float32)
    y = np.zeros(10, np.float32)
    assert ccl.reduce_scatter_block(x, y, 10, MPI_FLOAT, MPI_SUM, c) == 0
    assert np.array_equal(x, y) and calls == []
    assert c.free() == 0


@pytest.mark.parametrize('P', [1, 2, 5])
def test_barrier_and_custom_memory_kinds(oracle, P):
    """MPIX_Comm_barrier: every rank leaves only after every rank entered (host
    transport); MPIX_Comm_create_custom rejects an unknown memory kind; the
    step timer is inert on host communicators"""
    from mpich_amd import ccl
    import time
    comms = host_comms(P, oracle)
    entered = [None] * P

    def body(r, c):
        time.sleep(0.05 * r)            # arrive in turn
        entered[r] = time.monotonic()
        c.barrier()
        left = time.monotonic()
        c.set_step_timing(True)
        assert ccl.reduce_scatter_block(np.zeros(P, np.float32), np.zeros(1, np.float32), 1,
                                        MPI_FLOAT, MPI_SUM, c, 'recursive_halving') == 0
        c.set_step_timing(False)
        return left, c.step_times()
    out = run_ranks(comms, body)
    assert all(left >= max(entered) for left, _ in out)
    assert all(st == [] for _, st in out)
    free_all(comms)
    L = ccl.lib()
    h = ctypes.c_void_p()
    XFN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_void_p)
    fn = XFN(lambda *a: 0)
    assert L.MPIX_Comm_create_custom(0, 1, ctypes.cast(fn, ctypes.c_void_p), None, 3,
                                     ctypes.byref(h)) == 12     # MPI_ERR_ARG


def test_shared_memory_argument_errors(oracle):
    """MPIX_Comm_alloc_shared is for device communicators (a host one gets
    MPI_ERR_ARG and no memory); MPIX_Comm_free_shared of an address it did not
    hand out is MPI_ERR_BUFFER"""
    from mpich_amd import ccl
    L = ccl.lib()
    comms = host_comms(1, oracle)
    p = ctypes.c_void_p(1)
    assert L.MPIX_Comm_alloc_shared(comms[0].h, 4096, ctypes.byref(p)) == 12
    assert not p.value
    assert L.MPIX_Comm_alloc_shared(comms[0].h, 4096, None) == 12
    assert L.MPIX_Comm_free_shared(comms[0].h, 4096) == 1
    free_all(comms)


@pytest.mark.gpu
def test_shared_memory_local_communicator(oracle):
    """threads of one process: MPIX_Comm_alloc_shared is plain device memory
    (the pulls read peers' buffers directly anyway); a pull over it matches
    the oracle, and free_shared / free release it"""
    import torch
    from mpich_amd import ccl
    P, n = 4, 4099
    comms = _dev_comms(P)
    sh = [c.shared_tensor(P * n, torch.float32) for c in comms]
    sends = float_sends(P, P * n, 0x5EED0900)
    for t, x in zip(sh, sends):
        t.copy_(torch.from_numpy(x))
    out = [torch.zeros(n, dtype=torch.float32, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
        sh[r], out[r], n, MPI_FLOAT, MPI_SUM, c, 'recursive_halving_pull'))
    assert rcs == [0] * P
    exp = oracle.rsb_recursive_halving([x.view(np.uint8) for x in sends], n, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert out[r].cpu().numpy().tobytes() == exp[r].tobytes(), r
    run_ranks(comms, lambda r, c: c.free_shared(sh[r].data_ptr()))
    free_all(comms)


# ------------------------------------------------------------------ GPU
def _dev_comms(P):
    from mpich_amd import ccl
    return ccl.comm_create_local(P, [0] * P)


@pytest.mark.gpu
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential',
                                  'recursive_halving_multipath', 'recursive_halving_pull'])
@pytest.mark.parametrize('P', [2, 3, 4, 8])
def test_rsb_device_local_matches_oracle(oracle, P, algo):
    import torch
    from mpich_amd import ccl
    recvcount = (1 << 18) + 13
    sends = float_sends(P, P * recvcount)
    dsend = [torch.from_numpy(s).cuda() for s in sends]
    drecv = [torch.zeros(recvcount, dtype=torch.float32, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(dsend[r], drecv[r], recvcount,
                                                                  MPI_FLOAT, MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    sim = oracle.rsb_pairwise if algo.startswith('pairwise') else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert drecv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('in_place', [False, True])
@pytest.mark.parametrize('dt,op', [(MPI_FLOAT, MPI_SUM), (MPI_DOUBLE, MPI_MAX),
                                   (MPI_DOUBLE, MPI_MIN), (MPI_2INT, MPI_MAXLOC)])
@pytest.mark.parametrize('P', [2, 3, 4, 6, 7, 8, 12, 16])
def test_rsb_recursive_halving_pull_matches_oracle(oracle, P, dt, op, in_place):
    """MPIX_RSB_RECURSIVE_HALVING_PULL: one tree kernel per rank reading its
    block of all P ranks through the mappings, bit-identical to the oracle's
    recursive-halving simulation -- NaN payloads, +-0 and MAXLOC ties show the
    operand roles of every level; odd recvcount puts the blocks off the
    16-byte grid (element path); MPI_IN_PLACE lands the block at recvbuf[0]"""
    import torch
    from mpich_amd import ccl
    recvcount = 40961 if P <= 8 else 4099
    ext = oracle.extent(dt)
    rng = np.random.default_rng(0x5EED0700 + P)
    if dt == MPI_2INT:
        sends = [rng.integers(0, 3, (P * recvcount, 2)).astype(np.int32) for _ in range(P)]
    elif dt == MPI_DOUBLE:
        sends = _special_doubles(P, P * recvcount, P)
    else:
        sends = float_sends(P, P * recvcount, 0x5EED0701)
    raw = [np.ascontiguousarray(s).view(np.uint8).reshape(-1) for s in sends]
    dsend = [torch.from_numpy(r.copy()).cuda() for r in raw]
    drecv = dsend if in_place else [torch.zeros(recvcount * ext, dtype=torch.uint8, device='cuda')
                                    for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
        None if in_place else dsend[r], drecv[r], recvcount, dt, op, c, 'recursive_halving_pull'))
    free_all(comms)
    assert rcs == [0] * P
    exp = oracle.rsb_recursive_halving(raw, recvcount, dt, op)
    for r in range(P):
        got = drecv[r].cpu().numpy()[:recvcount * ext]
        assert got.tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('overlap', ['1', '0', 'default', str(1 << 20)])
@pytest.mark.parametrize('in_place', [False, True])
@pytest.mark.parametrize('dt,op', [(MPI_FLOAT, MPI_SUM), (MPI_DOUBLE, MPI_MAX),
                                   (MPI_2INT, MPI_MAXLOC)])
@pytest.mark.parametrize('P', [4, 8, 16])
def test_rsb_recursive_halving_overlap_matches_oracle(oracle, monkeypatch, P, dt, op, in_place,
                                                      overlap):
    """recursive halving with each step's kept half combined on the second
    stream under the next exchange (MPIX_COLL_RH_OVERLAP=1: every half-step
    splits; 2^20: half-steps of >= 1 MiB, the RCCL communicators' default; 0
    and the default of these local communicators: none) is bit-identical to
    the oracle's simulation of reduce_scatter_block_intra_recursive_halving.c
    -- NaN payloads and +-0 (double MAX) and MAXLOC ties show the operand
    roles; the step labels show which combines ran split"""
    import torch
    from mpich_amd import ccl
    if overlap == 'default':
        monkeypatch.delenv('MPIX_COLL_RH_OVERLAP', raising=False)
    else:
        monkeypatch.setenv('MPIX_COLL_RH_OVERLAP', overlap)
    recvcount = 4099
    if overlap == str(1 << 20):
        recvcount = (1 << 20) // oracle.extent(dt) + 5      # one block > 1 MiB
        if P == 16:
            recvcount //= 4
    ext = oracle.extent(dt)
    rng = np.random.default_rng(0x5EED0900 + P)
    if dt == MPI_2INT:
        sends = [rng.integers(0, 3, (P * recvcount, 2)).astype(np.int32) for _ in range(P)]
    elif dt == MPI_DOUBLE:
        sends = _special_doubles(P, P * recvcount, P)
    else:
        sends = float_sends(P, P * recvcount, 0x5EED0901)
    raw = [np.ascontiguousarray(s).view(np.uint8).reshape(-1) for s in sends]
    dsend = [torch.from_numpy(r.copy()).cuda() for r in raw]
    drecv = dsend if in_place else [torch.zeros(recvcount * ext, dtype=torch.uint8, device='cuda')
                                    for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)

    def body(r, c):
        c.set_step_timing(True)
        rc = ccl.reduce_scatter_block(None if in_place else dsend[r], drecv[r], recvcount, dt, op,
                                      c, 'recursive_halving')
        c.set_step_timing(False)
        torch.cuda.synchronize()
        return rc, [s['phase'] for s in c.step_times()]
    out = run_ranks(comms, body)
    free_all(comms)
    assert [o[0] for o in out] == [0] * P, out
    steps = P.bit_length() - 1
    for rc, phases in out:
        split = phases.count('combine (sent half)')
        assert split + phases.count('combine') == steps, phases
        if overlap in ('0', 'default'):
            assert split == 0, phases
        elif overlap == '1':
            assert split == steps - 1, phases
        else:       # the first step's kept quarter is >= 1 MiB: at least it splits
            assert split >= 1, phases
    exp = oracle.rsb_recursive_halving(raw, recvcount, dt, op)
    for r in range(P):
        got = drecv[r].cpu().numpy()[:recvcount * ext]
        assert got.tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('dt,op', [(MPI_INT, MPI_PROD), (MPI_DOUBLE, MPI_MAX),
                                   (MPI_INT, MPI_BXOR), (MPI_2INT, MPI_MAXLOC)])
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise'])
def test_rsb_device_local_types(oracle, dt, op, algo):
    import torch
    from mpich_amd import ccl
    P, recvcount = 5, 4097
    ext = oracle.extent(dt)
    rng = np.random.default_rng(0x5EED0003)
    if dt == MPI_2INT:      # values in 0..3 force ties (loc = min)
        sends = [rng.integers(0, 4, (P * recvcount, 2)).astype(np.int32) for _ in range(P)]
    elif dt == MPI_DOUBLE:
        sends = [rng.uniform(-1, 1, P * recvcount) for _ in range(P)]
    else:
        sends = [rng.integers(-2**31, 2**31, P * recvcount).astype(np.int32) for _ in range(P)]
    dsend = [torch.from_numpy(np.ascontiguousarray(s).view(np.uint8).reshape(-1)).cuda()
             for s in sends]
    drecv = [torch.zeros(recvcount * ext, dtype=torch.uint8, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(dsend[r], drecv[r], recvcount,
                                                                  dt, op, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    sim = oracle.rsb_pairwise if algo == 'pairwise' else oracle.rsb_recursive_halving
    exp = sim([np.ascontiguousarray(s).view(np.uint8).reshape(-1) for s in sends], recvcount,
              dt, op)
    for r in range(P):
        assert drecv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('algo', ['reduce_scatter_allgather', 'rsag_rd_allgather',
                                  'recursive_doubling', 'ring', 'rsag_multipath', 'pull'])
@pytest.mark.parametrize('P', [2, 3, 4, 7, 8])
def test_allreduce_device_local_matches_oracle(oracle, P, algo):
    import torch
    from mpich_amd import ccl
    count = (1 << 18) + 37
    sends = float_sends(P, count, 0x5EED0200)
    dsend = [torch.from_numpy(s).cuda() for s in sends]
    drecv = [torch.zeros(count, dtype=torch.float32, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    for rep in range(2):        # the second call reuses the communicators' scratch
        rcs = run_ranks(comms, lambda r, c: ccl.allreduce(dsend[r], drecv[r], count, MPI_FLOAT,
                                                           MPI_SUM, c, algo))
        assert rcs == [0] * P
    free_all(comms)
    exp = oracle.allreduce_rabenseifner(
        [s.view(np.uint8) for s in sends], count, MPI_FLOAT, MPI_SUM,
        algorithm=algo if algo in ('recursive_doubling', 'ring') else 'reduce_scatter_allgather')
    for r in range(P):
        assert drecv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('in_place', [False, True])
@pytest.mark.parametrize('dt,op', [(MPI_FLOAT, MPI_SUM), (MPI_DOUBLE, MPI_MAX),
                                   (MPI_2INT, MPI_MAXLOC)])
@pytest.mark.parametrize('P', [2, 3, 4, 5, 7, 8, 12, 16])
def test_allreduce_pull_matches_oracle(oracle, P, dt, op, in_place):
    """MPIX_ALLREDUCE_PULL: a tree kernel per rank over every rank's input
    (rank r owns block bitrev(r)), then one copy kernel gathering the peers'
    blocks -- the bits of the Rabenseifner schedule, with NaN/+-0 and MAXLOC
    ties showing every operand role; ragged blocks (count % P != 0) and
    MPI_IN_PLACE"""
    import torch
    from mpich_amd import ccl
    count = 30011 if P <= 8 else 4103
    ext = oracle.extent(dt)
    rng = np.random.default_rng(0x5EED0800 + P)
    if dt == MPI_2INT:
        sends = [rng.integers(0, 3, (count, 2)).astype(np.int32) for _ in range(P)]
    elif dt == MPI_DOUBLE:
        sends = _special_doubles(P, count, 3 * P)
    else:
        sends = float_sends(P, count, 0x5EED0801)
    raw = [np.ascontiguousarray(s).view(np.uint8).reshape(-1) for s in sends]
    dsend = [torch.from_numpy(r.copy()).cuda() for r in raw]
    drecv = dsend if in_place else [torch.zeros(count * ext, dtype=torch.uint8, device='cuda')
                                    for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.allreduce(None if in_place else dsend[r], drecv[r],
                                                       count, dt, op, c, 'pull'))
    free_all(comms)
    assert rcs == [0] * P
    exp = oracle.allreduce_rabenseifner(raw, count, dt, op, algorithm='reduce_scatter_allgather')
    for r in range(P):
        assert drecv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
def test_copy_multi():
    """MPIX_Copy_multi_async: up to 16 independent copies in one launch,
    16-byte-phase-matched and mismatched pairs, empty entries skipped"""
    import torch
    from mpich_amd import redop
    L = redop.lib()
    src = torch.randint(0, 256, (1 << 22,), dtype=torch.uint8, device='cuda')
    dst = torch.zeros(1 << 22, dtype=torch.uint8, device='cuda')
    segs = [(0, 0, 1000003), (1000003 + 16, 1100000, 65536), (1300001, 1300001, 5),
            (2000000, 2000003, 77777), (3000000, 3000000, 0)] + \
        [(3100000 + 40000 * i, 3100000 + 40000 * i + (i % 3), 30000 + i) for i in range(11)]
    assert len(segs) == 16
    torch.cuda.synchronize()
    vp = ctypes.c_void_p
    srcs = (vp * 16)(*[src.data_ptr() + a for a, _, _ in segs])
    dsts = (vp * 16)(*[dst.data_ptr() + b for _, b, _ in segs])
    nb = (ctypes.c_ssize_t * 16)(*[n for _, _, n in segs])
    L.MPIX_Copy_multi_async.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                        ctypes.POINTER(ctypes.c_ssize_t), ctypes.c_int, vp]
    assert L.MPIX_Copy_multi_async(srcs, dsts, nb, 16, None) == 0
    torch.cuda.synchronize()
    s, d = src.cpu().numpy(), dst.cpu().numpy()
    exp = np.zeros_like(d)
    for a, b, n in segs:
        exp[b:b + n] = s[a:a + n]
    assert np.array_equal(d, exp)


@pytest.mark.gpu
def test_async_on_caller_streams_back_to_back(oracle):
    """stream-ordered form on each rank's own torch stream, three collectives
    queued back to back without host synchronisation in between: the event
    hand-offs alone must order the copies against the combines"""
    import torch
    from mpich_amd import ccl
    P, recvcount = 4, 100003
    sends = float_sends(P, P * recvcount, 99)
    dsend = [torch.from_numpy(s).cuda() for s in sends]
    outs = [[torch.zeros(recvcount, dtype=torch.float32, device='cuda') for _ in range(3)]
            for _ in range(P)]
    streams = [torch.cuda.Stream() for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)

    def body(r, c):
        rc = []
        for k, algo in enumerate(['recursive_halving', 'pairwise', 'recursive_halving']):
            rc.append(ccl.reduce_scatter_block(dsend[r], outs[r][k], recvcount, MPI_FLOAT,
                                               MPI_SUM, c, algo, stream=streams[r],
                                               blocking=False))
        streams[r].synchronize()
        return rc
    rcs = run_ranks(comms, body)
    free_all(comms)
    assert rcs == [[0, 0, 0]] * P
    rh = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT,
                                      MPI_SUM)
    pw = oracle.rsb_pairwise([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert outs[r][0].cpu().numpy().tobytes() == rh[r].tobytes()
        assert outs[r][1].cpu().numpy().tobytes() == pw[r].tobytes()
        assert outs[r][2].cpu().numpy().tobytes() == rh[r].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential'])
@pytest.mark.parametrize('P', [3, 4, 7])
def test_reduce_scatter_device_ragged(oracle, P, algo):
    """MPI_Reduce_scatter on device buffers with ragged recvcounts (zeros
    included), HIP combine, bit-identical to the oracle's simulation"""
    import torch
    from mpich_amd import ccl
    counts = [c * 37 for c in _ragged_counts(P, 200 + P)]
    sends = float_sends(P, sum(counts), 0x5EED0500)
    dsend = [torch.from_numpy(s).cuda() for s in sends]
    drecv = [torch.zeros(max(1, c), dtype=torch.float32, device='cuda') for c in counts]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(dsend[r], drecv[r], counts, MPI_FLOAT,
                                                           MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    exp = oracle.rs_schedule([s.view(np.uint8) for s in sends], counts, MPI_FLOAT, MPI_SUM,
                             'pairwise' if algo.startswith('pairwise') else 'recursive_halving')
    for r in range(P):
        assert drecv[r][:counts[r]].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('P', [2, 3, 4])
def test_reduce_scatter_device_pipelined(oracle, P):
    """MPIX_RSB_PAIRWISE_PIPELINED with blocks large enough to be cut into
    chunks (>= 4 MiB each, up to 8): chunk k's combine runs on the
    communicator's second stream while chunk k+1 moves.  Bit-identical to the
    pairwise simulation: equal blocks, ragged blocks (one below the 4 MiB
    cut, one empty), MPI_IN_PLACE, and two collectives back to back on one
    communicator (the hand-off events are reused)."""
    import torch
    from mpich_amd import ccl
    big = (3 << 20) + 7                     # 12 MiB fp32 blocks -> 3 chunks
    for counts in ([big] * P, [big + 5 * r for r in range(P)][:-1] + [1000],
                   [0] + [(9 << 20) + 3] * (P - 1)):
        total = sum(counts)
        sends = float_sends(P, total, 0x5EED0900 + len(counts))
        exp = oracle.rs_schedule([s.view(np.uint8) for s in sends], counts, MPI_FLOAT, MPI_SUM,
                                 'pairwise')
        comms = _dev_comms(P)
        for in_place in (False, True):
            dsend = [torch.from_numpy(s).cuda() for s in sends]
            bufs = [d.clone() if in_place else torch.zeros(max(1, counts[r]), device='cuda')
                    for r, d in enumerate(dsend)]
            torch.cuda.synchronize()
            for rep in range(2):
                if rep and in_place:
                    for b, d in zip(bufs, dsend):
                        b.copy_(d)
                    torch.cuda.synchronize()
                rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(
                    None if in_place else dsend[r], bufs[r], counts, MPI_FLOAT, MPI_SUM, c,
                    'pairwise_pipelined'))
                assert rcs == [0] * P
                for r in range(P):
                    got = bufs[r][:counts[r]].cpu().numpy()
                    assert got.tobytes() == exp[r].tobytes(), (counts[r], in_place, rep, r)
        free_all(comms)


@pytest.mark.gpu
@pytest.mark.parametrize('counts', [[1, 4000, 3, 9000], [1, 4000], [4000, 1], [5, 5]])
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential'])
def test_reduce_scatter_device_in_place_overlap(oracle, algo, counts):
    """MPI_IN_PLACE with uneven counts where a rank's own block overlaps the
    front of recvbuf (counts [1, 4000, 3, 9000]: rank 1's block at offset 1
    is moved to offset 0), device buffers.  P = 2 recursive halving: the
    first step is also the last and reads recvbuf's second block while the
    result goes to its front -- [1, 4000] overlaps."""
    import torch
    from mpich_amd import ccl
    P = len(counts)
    sends = float_sends(P, sum(counts), 0x5EED0900)
    bufs = [torch.from_numpy(s.copy()).cuda() for s in sends]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter(None, bufs[r], counts, MPI_FLOAT,
                                                           MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    exp = oracle.rs_schedule([s.view(np.uint8) for s in sends], counts, MPI_FLOAT, MPI_SUM,
                             'pairwise' if algo.startswith('pairwise') else 'recursive_halving')
    for r in range(P):
        assert bufs[r][:counts[r]].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise', 'pairwise_sequential'])
def test_rsb_device_in_place(oracle, algo):
    """MPI_IN_PLACE on device buffers: inputs in recvbuf, result in its
    first block, bit-identical to the oracle's simulation"""
    import torch
    from mpich_amd import ccl
    P, recvcount = 5, 20011
    sends = float_sends(P, P * recvcount, 31)
    bufs = [torch.from_numpy(s.copy()).cuda() for s in sends]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(None, bufs[r], recvcount,
                                                                  MPI_FLOAT, MPI_SUM, c, algo))
    free_all(comms)
    assert rcs == [0] * P
    sim = oracle.rsb_pairwise if algo.startswith('pairwise') else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], recvcount, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert bufs[r][:recvcount].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
def test_async_scratch_shared_across_streams(oracle):
    """back-to-back async collectives of one rank on TWO streams, no
    workspace given: they share the communicator's scratch (the third call
    needs a bigger one, so it also grows), and the scratch event must order
    each user behind the previous one"""
    import torch
    from mpich_amd import ccl
    P = 4
    counts = (50021, 50021, 200003)
    sends = [float_sends(P, P * m, 7 + k) for k, m in enumerate(counts)]
    dsend = [[torch.from_numpy(s[r]).cuda() for r in range(P)] for s in sends]
    outs = [[torch.zeros(m, dtype=torch.float32, device='cuda') for m in counts]
            for _ in range(P)]
    streams = [(torch.cuda.Stream(), torch.cuda.Stream()) for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)

    def body(r, c):
        rc = [ccl.reduce_scatter_block(dsend[k][r], outs[r][k], m, MPI_FLOAT, MPI_SUM, c,
                                       'recursive_halving', stream=streams[r][k & 1],
                                       blocking=False)
              for k, m in enumerate(counts)]
        for s in streams[r]:
            s.synchronize()
        return rc
    rcs = run_ranks(comms, body)
    free_all(comms)
    assert rcs == [[0, 0, 0]] * P
    for k, m in enumerate(counts):
        exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends[k]], m, MPI_FLOAT,
                                           MPI_SUM)
        for r in range(P):
            assert outs[r][k].cpu().numpy().tobytes() == exp[r].tobytes(), (k, r)


@pytest.mark.gpu
def test_rccl_communicator_single_rank():
    """MPIX_Comm_create_ccl (MPIR_RCCLcomm_init, rccl.c:21-52) on the test
    box's one GPU: unique id, ncclCommInitRank with one rank, the P = 1
    collectives (a local copy, coll_api.txt:402-411) and MPIX_Comm_free.
    The P > 1 RCCL exchanges run in the driver's multi-GPU bench, which checks
    the redscatblk3.c closed form on every rank first."""
    import torch
    from mpich_amd import ccl
    uid = ccl.get_unique_id()
    assert len(uid) == ccl.UNIQUE_ID_BYTES and any(uid)
    c = ccl.comm_create_ccl(0, 1, uid)
    assert (c.rank, c.size) == (0, 1)
    x = torch.arange(1000, dtype=torch.float32, device='cuda')
    y = torch.zeros_like(x)
    torch.cuda.synchronize()
    assert ccl.reduce_scatter_block(x, y, 1000, MPI_FLOAT, MPI_SUM, c) == 0
    assert torch.equal(x, y)
    z = torch.zeros_like(x)
    assert ccl.allreduce(x, z, 1000, MPI_FLOAT, MPI_SUM, c) == 0
    assert torch.equal(x, z)
    assert c.free() == 0


# ------------------------------------------------------------ MPI_Reduce
def _special_doubles(P, n, seed):
    """values with ties, NaN and +-0 so that the operand order of every
    MPIR_Reduce_local of the schedule shows in MAX's bits"""
    rng = np.random.default_rng(seed)
    out = []
    for r in range(P):
        x = rng.integers(-3, 4, n).astype(np.float64)
        k = rng.random(n)
        x[k < 0.05] = np.nan
        x[(k >= 0.05) & (k < 0.15)] = -0.0
        x[(k >= 0.15) & (k < 0.25)] = 0.0
        out.append(x)
    return out


@pytest.mark.parametrize('algo', ['binomial', 'reduce_scatter_gather', 'auto'])
@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 6, 7, 8, 11, 16])
def test_reduce_host_matches_oracle(oracle, P, algo):
    """MPI_Reduce with every root: fp32 SUM and fp64 MAX (NaN / +-0 operand
    order) bit-identical to the oracle's simulation of
    reduce_intra_{binomial,reduce_scatter_gather}.c, plus MPI_IN_PLACE at the root"""
    from mpich_amd import ccl
    count = 1031
    comms = host_comms(P, oracle)
    for dt, op, sends in ((MPI_FLOAT, MPI_SUM, float_sends(P, count, 0x5EED0600)),
                          (MPI_DOUBLE, MPI_MAX, _special_doubles(P, count, 5))):
        ext = sends[0].itemsize
        sim_algo = 'binomial' if algo == 'binomial' or (algo == 'auto' and count * ext <= 2048) \
            else 'reduce_scatter_gather'
        for root in range(P):
            exp = oracle.reduce_schedule([s.view(np.uint8) for s in sends], count, dt, op, root,
                                         sim_algo)
            for in_place in (False, True):
                out = sends[root].copy() if in_place else np.zeros_like(sends[root])
                rcs = run_ranks(comms, lambda r, c: ccl.reduce(
                    None if (in_place and r == root) else sends[r], out if r == root else None,
                    count, dt, op, root, c, algo))
                assert rcs == [0] * P
                assert out.view(np.uint8).tobytes() == exp.tobytes(), (dt, root, in_place)
    free_all(comms)


@pytest.mark.parametrize('P', [3, 5, 8])
def test_reduce_kat(oracle, P):
    """reduce.c:17-110 (testlist sizes 3, 5, 10): in[i] = i on every rank,
    result i*P at every root, counts 1..2^16 doubling, with and without
    MPI_IN_PLACE; the oracle's two simulations give the same closed form"""
    from mpich_amd import ccl
    comms = host_comms(P, oracle)
    count = 1
    while count < 130000:
        src = np.arange(count, dtype=np.int32)
        for algo in ('binomial', 'reduce_scatter_gather'):
            if algo == 'reduce_scatter_gather' and count < (1 << (P.bit_length() - 1)):
                continue
            for root in (0, P - 1, P // 2):
                out = np.full(count, -1, np.int32)
                rcs = run_ranks(comms, lambda r, c: ccl.reduce(src, out if r == root else None,
                                                               count, MPI_INT, MPI_SUM, root, c,
                                                               algo))
                assert rcs == [0] * P
                assert np.array_equal(out, src * P), (count, algo, root)
                inp = src.copy()
                rcs = run_ranks(comms, lambda r, c: ccl.reduce(None if r == root else src,
                                                               inp if r == root else None, count,
                                                               MPI_INT, MPI_SUM, root, c, algo))
                assert rcs == [0] * P
                assert np.array_equal(inp, src * P), (count, algo, root, 'in place')
                sim = oracle.reduce_schedule([src.view(np.uint8)] * P, count, MPI_INT, MPI_SUM,
                                             root, algo)
                assert sim.tobytes() == (src * P).tobytes()
        count *= 8
    free_all(comms)


@pytest.mark.gpu
@pytest.mark.parametrize('algo', ['binomial', 'reduce_scatter_gather'])
@pytest.mark.parametrize('P', [3, 4, 6])
def test_reduce_device_matches_oracle(oracle, P, algo):
    """MPI_Reduce on device buffers (device transport, HIP combine), fp64 MAX
    with NaN / +-0 and fp32 SUM, two roots, bit-identical to the oracle"""
    import torch
    from mpich_amd import ccl
    count = 50021
    comms = _dev_comms(P)
    for dt, op, sends in ((MPI_DOUBLE, MPI_MAX, _special_doubles(P, count, 9)),
                          (MPI_FLOAT, MPI_SUM, float_sends(P, count, 0x5EED0700))):
        dsend = [torch.from_numpy(s).cuda() for s in sends]
        for root in (0, P - 1):
            out = torch.zeros_like(dsend[0])
            torch.cuda.synchronize()
            rcs = run_ranks(comms, lambda r, c: ccl.reduce(dsend[r], out if r == root else None,
                                                           count, dt, op, root, c, algo))
            assert rcs == [0] * P
            exp = oracle.reduce_schedule([s.view(np.uint8) for s in sends], count, dt, op, root,
                                         algo)
            assert out.cpu().numpy().view(np.uint8).tobytes() == exp.tobytes(), (dt, root)
    free_all(comms)


# ------------------------------------------------------- MPI_Scan / Exscan
@pytest.mark.parametrize('exclusive', [False, True])
@pytest.mark.parametrize('P', [1, 2, 3, 4, 5, 7, 8, 11, 16])
def test_scan_host_matches_oracle(oracle, P, exclusive):
    """recursive-doubling Scan / Exscan, fp64 MAX over NaN / +-0 (operand
    order in the bits) and fp32 SUM, plain and MPI_IN_PLACE, against the
    oracle's simulation"""
    from mpich_amd import ccl
    count = 777
    comms = host_comms(P, oracle)
    for dt, op, sends in ((MPI_DOUBLE, MPI_MAX, _special_doubles(P, count, 21)),
                          (MPI_FLOAT, MPI_SUM, float_sends(P, count, 0x5EED0800))):
        for in_place in (False, True):
            prior = [np.full_like(s, 7) for s in sends]         # Exscan: rank 0 keeps these
            outs = [s.copy() if in_place else p.copy() for s, p in zip(sends, prior)]
            rcs = run_ranks(comms, lambda r, c: ccl.scan(None if in_place else sends[r], outs[r],
                                                         count, dt, op, c, exclusive))
            assert rcs == [0] * P
            exp = [(s.copy() if in_place else p.copy()).view(np.uint8)
                   for s, p in zip(sends, prior)]
            oracle.scan_schedule([s.view(np.uint8) for s in sends], exp, count, dt, op,
                                 exclusive)
            for r in range(P):
                assert outs[r].view(np.uint8).tobytes() == exp[r].tobytes(), (dt, in_place, r)
    free_all(comms)


@pytest.mark.parametrize('P', [4, 5, 10])
def test_scan_exscan_kats(oracle, P):
    """scantst.c:60-70 (data = rank, result sum 0..rank) and exscan.c:38-85
    (counts 1..2^15, in[i] = rank + i*P, result rank*i*P + rank(rank-1)/2 on
    rank > 0; MPI_IN_PLACE leaves rank 0's buffer as it was)"""
    from mpich_amd import ccl
    comms = host_comms(P, oracle)
    outs = [np.full(1, -100, np.int32) for _ in range(P)]
    rcs = run_ranks(comms, lambda r, c: ccl.scan(np.array([r], np.int32), outs[r], 1, MPI_INT,
                                                 MPI_SUM, c))
    assert rcs == [0] * P
    assert [int(o[0]) for o in outs] == [r * (r + 1) // 2 for r in range(P)]
    count = 1
    while count < 65000:
        i = np.arange(count)
        sends = [(r + i * P).astype(np.int32) for r in range(P)]
        outs = [np.full(count, -1, np.int32) for _ in range(P)]
        rcs = run_ranks(comms, lambda r, c: ccl.scan(sends[r], outs[r], count, MPI_INT, MPI_SUM,
                                                     c, exclusive=True))
        assert rcs == [0] * P
        for r in range(1, P):
            assert np.array_equal(outs[r], r * i * P + r * (r - 1) // 2), (count, r)
        bufs = [s.copy() for s in sends]
        rcs = run_ranks(comms, lambda r, c: ccl.scan(None, bufs[r], count, MPI_INT, MPI_SUM, c,
                                                     exclusive=True))
        assert rcs == [0] * P
        assert np.array_equal(bufs[0], sends[0])
        for r in range(1, P):
            assert np.array_equal(bufs[r], r * i * P + r * (r - 1) // 2), (count, r)
        count *= 4
    free_all(comms)


@pytest.mark.gpu
@pytest.mark.parametrize('exclusive', [False, True])
def test_scan_device_matches_oracle(oracle, exclusive):
    import torch
    from mpich_amd import ccl
    P, count = 6, 30011
    sends = _special_doubles(P, count, 41)
    dsend = [torch.from_numpy(s).cuda() for s in sends]
    douts = [torch.full((count,), 7.0, dtype=torch.float64, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    rcs = run_ranks(comms, lambda r, c: ccl.scan(dsend[r], douts[r], count, MPI_DOUBLE, MPI_MAX,
                                                 c, exclusive))
    free_all(comms)
    assert rcs == [0] * P
    exp = [np.full(count, 7.0).view(np.uint8) for _ in range(P)]
    oracle.scan_schedule([s.view(np.uint8) for s in sends], exp, count, MPI_DOUBLE, MPI_MAX,
                         exclusive)
    for r in range(P):
        assert douts[r].cpu().numpy().view(np.uint8).tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
def test_collectives_ignore_support_knob(oracle):
    """MPIX_REDOP_ENABLE=0 (set_support(enable=False)) only answers
    MPIX_Redop_is_supported's callers; the collectives keep their kernels
    (the reference's MPIR_CVAR_ENABLE_YAKSA_REDUCTION only moves
    reductions back to the CPU)"""
    import torch
    from mpich_amd import ccl, redop
    P, n = 3, 10007
    sends = float_sends(P, P * n, 0x5EED0A00)
    dsend = [torch.from_numpy(s).cuda() for s in sends]
    drecv = [torch.zeros(n, dtype=torch.float32, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    before = redop.get_support()
    redop.check(redop.set_support(enable=False))
    comms = _dev_comms(P)
    try:
        assert not redop.is_supported(MPI_SUM, MPI_FLOAT)
        assert redop.has_gpu_path(MPI_SUM, MPI_FLOAT)
        rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
            dsend[r], drecv[r], n, MPI_FLOAT, MPI_SUM, c, 'recursive_halving'))
        assert rcs == [0] * P
    finally:
        free_all(comms)
        redop.check(redop.set_support(before['enable'], before['threshold_bytes'],
                                      before['host_floor_bytes'], before['pinned_floor_bytes']))
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], n, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert drecv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r


@pytest.mark.gpu
def test_state_on_device_local_communicator(oracle):
    """MPIX_Comm_get_state on the device transport: the pulls run as asked
    (no fallback) and AUTO resolves to the generic.json choice"""
    import torch
    from mpich_amd import ccl
    P, n = 4, 4099
    dsend = [torch.from_numpy(s).cuda() for s in float_sends(P, P * n, 7)]
    drecv = [torch.zeros(n, dtype=torch.float32, device='cuda') for _ in range(P)]
    torch.cuda.synchronize()
    comms = _dev_comms(P)
    try:
        for algo, ran in (('recursive_halving_pull', 'recursive_halving_pull'), ('pull', 'pull'),
                          ('auto', 'recursive_halving'), ('pairwise', 'pairwise')):
            rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
                dsend[r], drecv[r], n, MPI_FLOAT, MPI_SUM, c, algo))
            assert rcs == [0] * P
            for c in comms:
                st = c.state()
                assert st['last_rs'] == ran and st['pulls_enabled'] and st['fallbacks'] == 0, st
    finally:
        free_all(comms)


def _ndev():
    import torch
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.gpu
@pytest.mark.parametrize('algo', ['pull', 'recursive_halving_pull', 'recursive_halving'])
def test_local_communicator_on_distinct_devices(oracle, algo):
    """MPIX_Comm_create_local(P, [0..P-1]): peer access is enabled for every
    device pair at creation (yaksuri_hip_init_hooks.c:164-181), so the pulls
    read the other GPUs' buffers directly; bit-identical to the oracle.
    Skipped below 2 devices (the test box has one)."""
    import torch
    from mpich_amd import ccl, redop
    P = min(_ndev(), 8)
    if P < 2:
        pytest.skip('needs >= 2 GPUs for ranks on distinct devices (this box has %d)' % P)
    n = 40961
    sends = float_sends(P, P * n, 0x5EED0B00)
    dsend = [torch.from_numpy(s).to('cuda:%d' % r) for r, s in enumerate(sends)]
    drecv = [torch.zeros(n, dtype=torch.float32, device='cuda:%d' % r) for r in range(P)]
    for r in range(P):
        torch.cuda.synchronize(r)
    comms = ccl.comm_create_local(P, list(range(P)))
    try:
        rcs = run_ranks(comms, lambda r, c: ccl.reduce_scatter_block(
            dsend[r], drecv[r], n, MPI_FLOAT, MPI_SUM, c, algo))
        assert rcs == [0] * P
        peers = all(redop.peer_access(a, b) for a in range(P) for b in range(P))
        st = comms[0].state()
        assert st['pulls_enabled'] == peers, st
        if peers:
            assert st['last_rs'] == algo, st
    finally:
        free_all(comms)
    sim = oracle.rsb_pairwise if algo == 'pull' else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], n, MPI_FLOAT, MPI_SUM)
    for r in range(P):
        assert drecv[r].cpu().numpy().tobytes() == exp[r].tobytes(), r
