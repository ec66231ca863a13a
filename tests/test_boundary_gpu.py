"""GPU checks of boundary semantics added in round 2:

  * MPIX_EQUAL on host operands larger than every staging chunk is ONE
    comparison behind ONE header (opequal.c:20-35; MPIR_Reduce_equal "can't
    split the message"): no payload byte of inout changes, the header reflects
    the whole buffer (a difference in the last byte, or past the first 64 MiB,
    clears it);
  * a call the GPU path declines (a type no kernel covers) returns the
    documented MPI_ERR_TYPE and leaves both buffers untouched, on device and
    host operands, so the caller can run its own op table on them.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def R():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


@pytest.fixture(scope='module')
def H():
    from mpich_amd import handles
    return handles


def _equal_bufs(n, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    a[:8] = np.frombuffer(np.uint64(1).tobytes(), np.uint8)
    return a, a.copy()


def _header(b):
    return int(np.frombuffer(b[:8].tobytes(), np.uint64)[0])


@pytest.mark.parametrize('mib', [80, 300])
@pytest.mark.parametrize('where', ['pageable', 'pinned'])
def test_equal_large_host_not_chunked(R, H, mib, where):
    n = (mib << 20) + 13
    for diff_at in (None, n - 1, (70 << 20) + 5):
        a, b = _equal_bufs(n, 0x5EED0500 + mib)
        if diff_at is not None:
            a[diff_at] ^= 0x5A
        if where == 'pinned':
            ta = torch.from_numpy(a).pin_memory()
            tb = torch.from_numpy(b).pin_memory()
            R.check(R.MPI_Reduce_local(ta, tb, n, H.MPI_BYTE, H.MPIX_EQUAL))
            got = tb.numpy()
        else:
            R.check(R.MPI_Reduce_local(a, b, n, H.MPI_BYTE, H.MPIX_EQUAL))
            got = b
        assert _header(got) == (1 if diff_at is None else 0), (where, diff_at)
        ref = a.copy()
        if diff_at is not None:
            ref[diff_at] ^= 0x5A            # inout's payload is the untouched original
        assert np.array_equal(got[8:], ref[8:]), 'EQUAL changed payload bytes'


def test_equal_header_rules_on_device(R, H):
    """either header != 1 clears inout's header; payload never written"""
    n = (3 << 20) + 7
    for hin, hio, exp in ((1, 1, 1), (0, 1, 0), (1, 0, 0), (2, 1, 0)):
        a, b = _equal_bufs(n, 0x5EED0501)
        a[:8] = np.frombuffer(np.uint64(hin).tobytes(), np.uint8)
        b[:8] = np.frombuffer(np.uint64(hio).tobytes(), np.uint8)
        da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
        torch.cuda.synchronize()
        R.check(R.MPI_Reduce_local(da, db, n, H.MPI_BYTE, H.MPIX_EQUAL))
        got = db.cpu().numpy()
        assert _header(got) == exp, (hin, hio)
        assert np.array_equal(got[8:], b[8:])


@pytest.mark.parametrize('op_name', ['MPI_MAX', 'MPI_MIN', 'MPI_PROD'])
def test_declined_call_leaves_buffers_untouched(R, H, op_name):
    # the only legal pairs without a kernel: bf16 ops other than SUM (the
    # reference's op functions assert on them too, op_fns.c:459-493)
    dt, op = H.MPIX_BFLOAT16, getattr(H, op_name)
    assert not R.is_supported(op, dt)
    ext = R.datatype_extent(dt)
    n = 4099
    rng = np.random.default_rng(0x5EED0502)
    a = rng.integers(0, 256, n * ext, dtype=np.uint8)
    b = rng.integers(0, 256, n * ext, dtype=np.uint8)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    torch.cuda.synchronize()
    assert R.MPI_Reduce_local(da, db, n, dt, op) == H.MPI_ERR_TYPE
    assert R.reduce_local_async(da, db, n, dt, op) == H.MPI_ERR_TYPE
    torch.cuda.synchronize()
    assert np.array_equal(db.cpu().numpy(), b) and np.array_equal(da.cpu().numpy(), a)
    hb = b.copy()
    assert R.MPI_Reduce_local(a, hb, n, dt, op) == H.MPI_ERR_TYPE
    assert np.array_equal(hb, b)
