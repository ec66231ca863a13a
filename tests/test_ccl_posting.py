"""What the RCCL transport will be handed, checked on CPU.

RCCL matches the p2p operations of a pair in posting order and needs the
k-th ncclSend of a -> b and the k-th ncclRecv of b <- a to have the same size.
libmpix_coll splits a schedule's message above the communicator's maximum
(1 GiB on RCCL communicators, MPIX_Comm_set_max_message) into consecutive
same-peer messages inside the same exchange group; exchange_ccl then posts
the list as it is.  Here a custom host transport records every exchange group
of every rank -- the exact list exchange_ccl would post -- under a small
maximum, so that the 4 GiB/rank splitting and the non-power-of-two folds of
reduce_scatter_block_intra_recursive_halving.c:110-136,193-201 are exercised
at test sizes, and asserts:

- every message is at most the maximum, and a split message's pieces are
  consecutive in the group, contiguous in memory and all full but the last;
- per ordered pair, the sequence of send sizes equals the sequence of receive
  sizes (the posting-order match RCCL performs);
- the results are the oracle's bits (the split changes no association).
"""
import ctypes
import threading

import numpy as np
import pytest

MPI_FLOAT, MPI_INT, MPI_SUM = 0x4c00040a, 0x4c000405, 0x58000003


class Recorder:
    """a mailbox transport for P threads over host memory that keeps every
    group each rank posts"""

    def __init__(self, P):
        self.P = P
        self.cv = threading.Condition()
        self.box = {}
        self.seq_s = {}
        self.seq_r = {}
        self.groups = [[] for _ in range(P)]

    def exchange(self, rank, ops):
        self.groups[rank].append(list(ops))
        with self.cv:
            for peer, is_recv, addr, n in ops:
                if is_recv:
                    continue
                k = self.seq_s.get((rank, peer), 0)
                self.seq_s[(rank, peer)] = k + 1
                self.box[(rank, peer, k)] = ctypes.string_at(addr, n)
            self.cv.notify_all()
        for peer, is_recv, addr, n in ops:
            if not is_recv:
                continue
            k = self.seq_r.get((peer, rank), 0)
            self.seq_r[(peer, rank)] = k + 1
            with self.cv:
                if not self.cv.wait_for(lambda: (peer, rank, k) in self.box, timeout=60):
                    return 1
                data = self.box.pop((peer, rank, k))
            if len(data) != n:      # RCCL: the pair's k-th sizes must agree
                return 2
            ctypes.memmove(addr, data, n)
        return 0


def _run(P, fn):
    out = [None] * P
    ts = [threading.Thread(target=lambda r=r: out.__setitem__(r, fn(r))) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts), 'a rank hung'
    return out


def _check_posting(rec, maxb):
    P = rec.P
    sends = {(a, b): [] for a in range(P) for b in range(P)}
    recvs = {(a, b): [] for a in range(P) for b in range(P)}
    splits = 0
    for r in range(P):
        for g in rec.groups[r]:
            for i, (peer, is_recv, addr, n) in enumerate(g):
                assert 0 < n <= maxb, (r, g)
                (recvs[(peer, r)] if is_recv else sends[(r, peer)]).append(n)
                if i and n and g[i - 1][0] == peer and g[i - 1][1] == is_recv and \
                        g[i - 1][2] + g[i - 1][3] == addr:
                    assert g[i - 1][3] == maxb, 'a split piece before the last is short'
                    splits += 1
    for pair in sends:
        assert sends[pair] == recvs[pair], (pair, sends[pair], recvs[pair])
    return splits


@pytest.mark.parametrize('P', [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize('algo', ['recursive_halving', 'pairwise'])
def test_rsb_posting_order_with_split(oracle, P, algo):
    from mpich_amd import ccl
    rc = 3001                   # 12004-byte blocks, several halves per message
    maxb = 4096 + 12            # a maximum that divides nothing evenly
    rec = Recorder(P)
    comms = [ccl.comm_create_custom(r, P, rec.exchange, ccl.XPORT_HOST) for r in range(P)]
    sends = [np.random.default_rng(0x5EED0400 + r).uniform(-1, 1, P * rc).astype(np.float32)
             for r in range(P)]
    recvs = [np.zeros(rc, np.float32) for _ in range(P)]
    try:
        for c in comms:
            c.set_combine(oracle.combine_fn_address())
            c.set_max_message(maxb)
        rcs = _run(P, lambda r: ccl.reduce_scatter_block(sends[r], recvs[r], rc, MPI_FLOAT, MPI_SUM,
                                                         comms[r], algo))
        assert rcs == [0] * P
    finally:
        for c in comms:
            c.free()
    want = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], rc, MPI_FLOAT, MPI_SUM,
                                        algorithm=algo)
    for r in range(P):
        assert recvs[r].tobytes() == want[r].tobytes(), r
    assert _check_posting(rec, maxb) > 0, 'no message was split: the test proves nothing'


@pytest.mark.parametrize('P', [3, 5, 8])
def test_reduce_scatter_ragged_and_allreduce_posting(oracle, P):
    """per-rank recvcounts (MPI_Reduce_scatter, some 0) and the allreduce's
    reduce-scatter + allgather under the same split"""
    from mpich_amd import ccl
    maxb = 1000
    counts = [(r * 797) % 2011 for r in range(P)]
    counts[1] = 0
    total = sum(counts)
    rec = Recorder(P)
    comms = [ccl.comm_create_custom(r, P, rec.exchange, ccl.XPORT_HOST) for r in range(P)]
    sends = [np.random.default_rng(0x5EED0500 + r).integers(-9, 9, total).astype(np.int32)
             for r in range(P)]
    recvs = [np.zeros(max(1, c), np.int32) for c in counts]
    outs = [np.zeros(total, np.int32) for _ in range(P)]
    try:
        for c in comms:
            c.set_combine(oracle.combine_fn_address())
            c.set_max_message(maxb)
        rcs = _run(P, lambda r: ccl.reduce_scatter(sends[r], recvs[r], counts, MPI_INT, MPI_SUM,
                                                   comms[r], 'recursive_halving'))
        assert rcs == [0] * P
        rcs = _run(P, lambda r: ccl.allreduce(sends[r], outs[r], total, MPI_INT, MPI_SUM, comms[r],
                                              'reduce_scatter_allgather'))
        assert rcs == [0] * P
    finally:
        for c in comms:
            c.free()
    want = oracle.rs_schedule([s.view(np.uint8) for s in sends], counts, MPI_INT, MPI_SUM)
    for r in range(P):
        assert recvs[r][:counts[r]].tobytes() == want[r].tobytes(), r
        assert np.array_equal(outs[r], sum(s.astype(np.int64) for s in sends).astype(np.int32))
    assert _check_posting(rec, maxb) > 0


def test_max_message_arguments():
    from mpich_amd import ccl, redop
    rec = Recorder(1)
    c = ccl.comm_create_custom(0, 1, rec.exchange, ccl.XPORT_HOST)
    try:
        with pytest.raises(redop.RedopError):
            c.set_max_message(-1)
        c.set_max_message(0)            # never split: allowed off RCCL
        c.set_max_message(1 << 40)
    finally:
        c.free()
