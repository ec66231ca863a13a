"""CPU checks of the support predicate's knobs and of the failure semantics
at the boundary (no GPU compute calls):

  * MPIX_Redop_is_supported mirrors MPIR_Typerep_reduce_is_supported
    (typerep_yaksa_pack.c:227-271): MPIX_REDOP_ENABLE=0 declines everything,
    MPIX_REDOP_THRESHOLD declines count > 0 whose packed size exceeds it;
  * MPIX_Redop_is_supported_buffers declines host-resident operands below the
    floor of their memory kind (here: pageable numpy buffers);
  * an MPIX_Op_table entry on a pair no kernel covers (MAX on MPIX_BFLOAT16,
    which the reference's MPIR_MAXF asserts on too)
    aborts like op_fns.c:51-53's MPIR_Assert(0), or only records the error
    with MPIX_REDOP_OPFN_ABORT=0;
  * libmpix_coll declines such a type on every rank before any exchange, and
    refuses MPIX_EQUAL in the schedules that split the message.
"""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def R():
    from mpich_amd import redop
    return redop


@pytest.fixture(scope='module')
def H():
    from mpich_amd import handles
    return handles


@pytest.fixture()
def knobs(R):
    before = R.get_support()
    yield R
    R.check(R.lib().MPIX_Redop_set_support(1 if before['enable'] else 0,
                                           before['threshold_bytes'],
                                           before['host_floor_bytes'],
                                           before['pinned_floor_bytes']))


def test_enable_knob(knobs, H):
    R = knobs
    assert R.is_supported(H.MPI_SUM, H.MPI_FLOAT)
    R.check(R.set_support(enable=False))
    assert not R.is_supported(H.MPI_SUM, H.MPI_FLOAT)
    assert not R.is_supported(H.MPI_MAXLOC, H.MPI_2INT, 10)
    # the legality checks do not depend on the knob
    assert R.op_dt_check(H.MPI_SUM, H.MPI_FLOAT)
    R.check(R.set_support(enable=True))
    assert R.is_supported(H.MPI_SUM, H.MPI_FLOAT)


def test_threshold_on_packed_size(knobs, H):
    """data_sz = count * size (MPIR_Pack_size), declined when > threshold;
    count 0 (reduce_local.c:68) only asks about the pair"""
    R = knobs
    R.check(R.set_support(enable=True, threshold_bytes=4096))
    assert R.is_supported(H.MPI_SUM, H.MPI_FLOAT, 1024)        # 4096 bytes: not above
    assert not R.is_supported(H.MPI_SUM, H.MPI_FLOAT, 1025)
    assert R.is_supported(H.MPI_SUM, H.MPI_FLOAT, 0)
    # DOUBLE_INT: size 12 (padding excluded), extent 16
    assert R.is_supported(H.MPI_MAXLOC, H.MPI_DOUBLE_INT, 341)   # 4092 bytes
    assert not R.is_supported(H.MPI_MAXLOC, H.MPI_DOUBLE_INT, 342)
    R.check(R.set_support(enable=True, threshold_bytes=-1))
    assert R.is_supported(H.MPI_SUM, H.MPI_FLOAT, 1 << 40)


def test_buffer_predicate_host_floor(knobs, H):
    """both operands pageable host memory: below the floor the caller's CPU
    loop keeps the chunk; at or above it the GPU path takes it"""
    R = knobs
    a = np.zeros(1 << 16, np.float32)
    b = np.zeros(1 << 16, np.float32)
    R.check(R.set_support(enable=True, threshold_bytes=-1, host_floor_bytes=65536))
    assert not R.is_supported_buffers(H.MPI_SUM, H.MPI_FLOAT, 16383, a, b)
    assert R.is_supported_buffers(H.MPI_SUM, H.MPI_FLOAT, 16384, a, b)
    R.check(R.set_support(enable=True, threshold_bytes=-1, host_floor_bytes=0))
    assert R.is_supported_buffers(H.MPI_SUM, H.MPI_FLOAT, 1, a, b)
    # unsupported pairs stay unsupported whatever the buffers
    assert not R.is_supported_buffers(H.MPI_MAX, H.MPIX_BFLOAT16, 16, a, b)
    R.check(R.set_support(enable=False))
    assert not R.is_supported_buffers(H.MPI_SUM, H.MPI_FLOAT, 1 << 20, a, b)


def test_env_knobs_read_at_first_use(H):
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from mpich_amd import redop as R, handles as H\n'
            's = R.get_support()\n'
            'assert s == dict(enable=False, threshold_bytes=123, host_floor_bytes=7, '
            'pinned_floor_bytes=9), s\n'
            'assert not R.is_supported(H.MPI_SUM, H.MPI_FLOAT)\n' % ROOT)
    env = dict(os.environ, MPIX_REDOP_ENABLE='0', MPIX_REDOP_THRESHOLD='123',
               MPIX_REDOP_HOST_FLOOR='7', MPIX_REDOP_PINNED_FLOOR='9')
    subprocess.run([sys.executable, '-c', code], check=True, env=env, timeout=120)


def _op_table_unsupported(env_extra):
    code = ('import ctypes, sys; sys.path.insert(0, %r)\n'
            'from mpich_amd import redop as R, handles as H\n'
            'L = R.lib()\n'
            'tab = (ctypes.c_void_p * 16).in_dll(L, "MPIX_Op_table")\n'
            'fn = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,\n'
            '                      ctypes.POINTER(ctypes.c_ssize_t), ctypes.POINTER(ctypes.c_int))'
            '(tab[H.MPI_MAX & 0xf])\n'
            'a = (ctypes.c_char * 64)(); b = (ctypes.c_char * 64)()\n'
            'n = ctypes.c_ssize_t(4); t = ctypes.c_int(H.as_c_int(H.MPIX_BFLOAT16))\n'
            'fn(a, b, ctypes.byref(n), ctypes.byref(t))\n'
            'print("returned", L.MPIX_Redop_last_error(), bytes(b) == bytes(64))\n' % ROOT)
    return subprocess.run([sys.executable, '-c', code], capture_output=True, text=True,
                          env=dict(os.environ, **env_extra), timeout=120)


def test_op_table_unsupported_type_aborts(H):
    """op_fns.c:51-53: MPIR_Assert(0) on a type the op function does not cover"""
    p = _op_table_unsupported({})
    assert p.returncode == -6, (p.returncode, p.stdout, p.stderr)
    assert 'MPIX_MAXF' in p.stderr and '0x%08x' % H.MPIX_BFLOAT16 in p.stderr, p.stderr
    assert 'returned' not in p.stdout


def test_op_table_unsupported_type_recorded_without_abort():
    p = _op_table_unsupported({'MPIX_REDOP_OPFN_ABORT': '0'})
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ['returned', '3', 'True'], p.stdout   # MPI_ERR_TYPE, untouched


def _run_threads(n, fn):
    out = [None] * n
    ts = [threading.Thread(target=lambda r=r: out.__setitem__(r, fn(r))) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts), 'a rank hung'
    return out


def test_collectives_decline_unsupported_type_on_every_rank(H):
    """MAX on MPIX_BFLOAT16 has no kernel: every rank returns MPI_ERR_TYPE before
    any exchange (no rank is left waiting on a peer), buffers untouched"""
    from mpich_amd import ccl
    P = 3
    comms = ccl.comm_create_local(P)        # host transport, no combine installed
    try:
        send = [np.arange(P * 8 * 2, dtype=np.uint8) for _ in range(P)]    # extent 2
        recv = [np.full(8 * 2, 0xAB, np.uint8) for _ in range(P)]
        rcs = _run_threads(P, lambda r: ccl.reduce_scatter_block(
            send[r], recv[r], 8, H.MPIX_BFLOAT16, H.MPI_MAX, comms[r], 'recursive_halving'))
        assert rcs == [H.MPI_ERR_TYPE] * P
        assert all((x == 0xAB).all() for x in recv)
        rcs = _run_threads(P, lambda r: ccl.allreduce(
            send[r], recv[r], 8, H.MPIX_BFLOAT16, H.MPI_MAX, comms[r], 'ring'))
        assert rcs == [H.MPI_ERR_TYPE] * P
    finally:
        for c in comms:
            c.free()


def test_collectives_refuse_split_equal(oracle, H):
    """MPIX_EQUAL's header covers the whole message (opequal.c; MPIR_Reduce_equal
    uses only non-splitting schedules): the reduce-scatter schedules refuse it,
    the recursive-doubling allreduce (auto picks it) computes it"""
    from mpich_amd import ccl
    P = 2
    comms = ccl.comm_create_local(P)
    for c in comms:
        c.set_combine(oracle.combine_fn_address())
    try:
        n = 64
        bufs = []
        for r in range(P):
            b = np.zeros(n, np.uint8)
            b[:8] = np.frombuffer(np.uint64(1).tobytes(), np.uint8)
            b[8:] = 7
            bufs.append(b)
        rcs = _run_threads(P, lambda r: ccl.reduce_scatter_block(
            np.tile(bufs[r], P), np.zeros(n, np.uint8), n, H.MPI_BYTE, H.MPIX_EQUAL, comms[r],
            'pairwise'))
        assert rcs == [H.MPI_ERR_OP] * P
        outs = [np.zeros(n, np.uint8) for _ in range(P)]
        rcs = _run_threads(P, lambda r: ccl.allreduce(bufs[r], outs[r], n, H.MPI_BYTE,
                                                       H.MPIX_EQUAL, comms[r], 'auto'))
        assert rcs == [0] * P
        assert all(o[:8].view(np.uint64)[0] == 1 for o in outs)
        rcs = _run_threads(P, lambda r: ccl.allreduce(bufs[r], outs[r], n, H.MPI_BYTE,
                                                       H.MPIX_EQUAL, comms[r],
                                                       'reduce_scatter_allgather'))
        assert rcs == [H.MPI_ERR_OP] * P
    finally:
        for c in comms:
            c.free()


def test_default_host_floors():
    """the floors MPIX_Redop_is_supported_buffers applies by default: the
    measured crossover (128 MiB pageable, 4 MiB page-locked
    per operand), in a fresh process with no MPIX_REDOP_* in the environment"""
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from mpich_amd import redop as R\n'
            's = R.get_support()\n'
            'assert s == dict(enable=True, threshold_bytes=-1, host_floor_bytes=128 << 20, '
            'pinned_floor_bytes=4 << 20), s\n' % ROOT)
    env = {k: v for k, v in os.environ.items() if not k.startswith('MPIX_REDOP_')}
    subprocess.run([sys.executable, '-c', code], check=True, env=env, timeout=120)
