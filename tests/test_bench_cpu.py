"""bench.py's own host logic on CPU: the numpy restatement of the
recursive-halving association that gates the N > 1 value (checked here
against the oracle's simulation of reduce_scatter_block_intra_recursive_halving.c),
and the watchdogs that turn a hung leg into rank 0's error line plus a
non-zero exit status."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize('world', [2, 3, 4, 5, 6, 7, 8])
def test_rh_expected_block_matches_oracle(oracle, world):
    import bench
    rc = 1031
    sends = [bench.rsb_inputs_host(r, world, rc) for r in range(world)]
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], rc, 0x4c00040a, 0x58000003)
    for r in range(world):
        assert bench.rh_expected_block(sends, r, rc).tobytes() == exp[r].tobytes(), r


def _run(code):
    return subprocess.run([sys.executable, '-c', textwrap.dedent(code)], cwd=ROOT,
                          capture_output=True, text=True, timeout=60)


def test_value_leg_watchdog_prints_error_and_exits_2():
    p = _run("""
        import time, bench
        e = bench._Emitter(0, {'metric': 'm', 'value': None, 'error': 'value leg did not finish'})
        bench._watchdog(0.3, e, note=False, code=2)
        time.sleep(10)
        """)
    assert p.returncode == 2
    assert '"error": "value leg did not finish"' in p.stdout
    assert 'extras_watchdog' not in p.stdout


def test_extras_watchdog_keeps_headline_and_exits_3():
    p = _run("""
        import time, bench
        e = bench._Emitter(0, {'metric': 'm', 'value': 1.5})
        bench._watchdog(0.3, e)
        time.sleep(10)
        """)
    assert p.returncode == 3
    assert '"value": 1.5' in p.stdout and 'extras_watchdog' in p.stdout and '"error"' in p.stdout


def test_emitter_prints_once_and_only_on_rank0():
    p = _run("""
        import bench
        e = bench._Emitter(0, {'v': 1})
        e.emit(); e.emit('late')
        bench._Emitter(1, {'v': 2}).emit()
        """)
    assert p.returncode == 0
    assert p.stdout.strip().splitlines() == ['{"v": 1}']


def _threads(comms, fn):
    import threading
    out = [None] * len(comms)
    ts = [threading.Thread(target=lambda r=r: out.__setitem__(r, fn(r, comms[r])))
          for r in range(len(comms))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts), 'a rank hung'
    return out


def test_schedule_ran_reports_fallback(oracle, monkeypatch):
    """a requested schedule that cannot run is reported as
    'fell back to ...' by the bench helper and never timed under its name.
    On host communicators the pulls cannot run (no device memory to map), so
    'pull' runs one-group pairwise and 'recursive_halving_pull' recursive
    halving -- with MPIX_COLL_WINDOW_FAULT set as in the GPU fault test."""
    import bench
    from mpich_amd import ccl
    monkeypatch.setenv('MPIX_COLL_WINDOW_FAULT', '1')
    P, n = 4, 1003
    comms = ccl.comm_create_local(P)
    for c in comms:
        c.set_combine(oracle.combine_fn_address())
    sends = [np.random.default_rng(r).uniform(-1, 1, P * n).astype(np.float32) for r in range(P)]
    recvs = [np.zeros(n, np.float32) for _ in range(P)]
    MPI_FLOAT, MPI_SUM = 0x4c00040a, 0x58000003
    try:
        for algo, ran in (('pull', 'pairwise'), ('recursive_halving_pull', 'recursive_halving'),
                          ('recursive_halving_multipath', 'recursive_halving'),  # P=4 ok on host
                          ('pairwise', 'pairwise')):
            rcs = _threads(comms, lambda r, c: ccl.reduce_scatter_block(
                sends[r], recvs[r], n, MPI_FLOAT, MPI_SUM, c, algo))
            assert rcs == [0] * P
            for c in comms:
                got = bench.schedule_ran(c, algo)
                if algo == 'recursive_halving_multipath':
                    assert got['schedule_ran'] == algo and 'error' not in got, got
                else:
                    assert got['schedule_ran'] == ran, got
                    assert ('error' in got) == (ran != algo), got
                    if ran != algo:
                        assert got['error'] == 'fell back to ' + ran
                assert got['pulls_enabled'] is False
        st = comms[0].state()
        assert st['fallbacks'] == 2 and st['window_retries'] == 0, st
        # allreduce: pull -> reduce_scatter_allgather; multipath on P=3-like
        # shapes (count % P) -> reduce_scatter_allgather
        outs = [np.zeros(P * n, np.float32) for _ in range(P)]
        for algo, count in (('pull', P * n), ('rsag_multipath', P * n - 1),
                            ('rsag_multipath', P * n)):
            rcs = _threads(comms, lambda r, c: ccl.allreduce(sends[r][:count], outs[r][:count],
                                                              count, MPI_FLOAT, MPI_SUM, c, algo))
            assert rcs == [0] * P
            got = bench.schedule_ran(comms[1], algo, 'ar')
            fell = algo == 'pull' or count % P
            assert got['schedule_ran'] == ('reduce_scatter_allgather' if fell else algo), got
            assert ('error' in got) == bool(fell)
    finally:
        for c in comms:
            c.free()


def test_state_before_first_collective():
    from mpich_amd import ccl
    comms = ccl.comm_create_local(2)
    try:
        st = comms[0].state()
        assert st == dict(pulls_enabled=False, last_rs=None, last_allreduce=None,
                          window_retries=0, fallbacks=0), st
    finally:
        for c in comms:
            c.free()


def test_leg_without_symmetric_memory_is_reported_not_fatal():
    """MPIX_Comm_alloc_shared answers MPI_ERR_OTHER on every rank when no
    verified mapping could be made (mpix_coll.h); the bench then reports that
    leg with its reason and no time, and goes on with the others (found by the
    window-fault rehearsal, profiles/r03_rehearsal_n4.json)"""
    import bench
    from mpich_amd import redop
    leg = bench._no_shared(redop.RedopError(15, 'MPIX_Comm_alloc_shared'))
    assert leg['schedule_ran'] is None and 'ms' not in leg
    assert leg['error'].startswith('no symmetric memory') and 'MPIX_Comm_alloc_shared' in leg['error']
