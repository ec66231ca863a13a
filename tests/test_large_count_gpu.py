"""Counts past 32 bits (MPI_Reduce_local_c).

The reference binding declares MPI_Reduce_local's count as
POLYXFER_NUM_ELEM_NNI (src/binding/mpi_standard_api.txt:1762-1767), which
generates the MPI_Count form MPI_Reduce_local_c, and MPIR_Reduce_local takes
an MPI_Aint (src/include/mpir_coll.h:62-63).  The library's surface takes
MPIX_Aint throughout; these tests run it where a 32-bit index would wrap:

  * MPI_INT8_T SUM, count = 2^31 + 4099 (more elements than an int holds);
  * MPI_FLOAT SUM, count = 2^30 + 5 (more than 4 GiB per operand);

each through the synchronous, stream-ordered, batch (one segment > 2^31
elements for INT8_T beside a small one) and multi-input (k = 2) entries, with
the operands at offsets off the 16-byte grid so the head / packet / tail split
runs (and, for the async call, `in` at another 16-byte phase than inout: the
unaligned-load form).  Every byte of every result is compared with the
oracle (oracle/redop_oracle.c, 8 host threads) on the same inputs."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

MPI_INT8_T, MPI_FLOAT, MPI_SUM = 0x4c000137, 0x4c00040a, 0x58000003

CASES = [('int8', MPI_INT8_T, 1, (1 << 31) + 4099, 3, 5),
         ('float', MPI_FLOAT, 4, (1 << 30) + 5, 4, 8)]


@pytest.fixture(scope='module')
def R():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    return redop


def _random_bytes(nbytes, seed, ext):
    """seeded operand bytes made on the GPU (fast at 4 GiB); floats uniform in
    [-1, 1) so sums stay finite, int8 the full byte range"""
    g = torch.Generator(device='cuda')
    g.manual_seed(seed)
    if ext == 4:
        t = torch.empty(nbytes // 4, dtype=torch.float32, device='cuda').uniform_(-1, 1, generator=g)
    else:
        t = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device='cuda', generator=g)
    return t.view(torch.uint8)


def _bytes_equal(dev_u8, host_u8):
    got = dev_u8.cpu().numpy()
    if np.array_equal(got, host_u8):
        return None
    bad = np.flatnonzero(got != host_u8)
    return '%d bytes differ, first at %d, last at %d' % (bad.size, bad[0], bad[-1])


@pytest.mark.timeout(600)
@pytest.mark.parametrize('name,dt,ext,count,off_io,off_in2', CASES, ids=[c[0] for c in CASES])
def test_large_count_every_entry_matches_oracle(R, oracle, name, dt, ext, count, off_io, off_in2):
    nb = count * ext
    pad = 64
    # operand bytes: in, in2 (multi's second input), inout's initial value
    d_in_src = _random_bytes(nb, 0x5EED1A00 + ext, ext)
    d_io_src = _random_bytes(nb, 0x5EED1A10 + ext, ext)
    h_in = d_in_src.cpu().numpy()
    h_io = d_io_src.cpu().numpy()
    exp = h_io.copy()
    assert oracle.reduce_local(h_in, exp, count, dt, MPI_SUM, nthreads=8) == 0
    # device buffers: inout at off_io bytes past a 256-byte boundary (head
    # elements before the first packet, a ragged tail), `in` at the same phase
    # or (off_in2) at another one
    io_buf = torch.empty(nb + pad, dtype=torch.uint8, device='cuda')
    in_buf = torch.empty(nb + pad, dtype=torch.uint8, device='cuda')
    io = io_buf[off_io:off_io + nb]
    bad = {}

    def reset(in_off):
        io.copy_(d_io_src)
        v = in_buf[in_off:in_off + nb]
        v.copy_(d_in_src)
        torch.cuda.synchronize()
        return v

    # synchronous MPIX_Reduce_local (the MPIR_Reduce_local drop-in)
    src = reset(off_io)
    assert R.lib().MPIX_Reduce_local(src.data_ptr(), io.data_ptr(), count, dt, MPI_SUM) == 0
    bad['sync'] = _bytes_equal(io, exp)
    # stream-ordered, `in` at another 16-byte phase
    src = reset(off_in2)
    s = torch.cuda.current_stream()
    assert R.reduce_local_async(src.data_ptr(), io.data_ptr(), count, dt, MPI_SUM, s) == 0
    s.synchronize()
    bad['async'] = _bytes_equal(io, exp)
    # batch: a small segment, then the whole large one (> 2^31 elements for int8)
    src = reset(off_io)
    small_io = torch.zeros(4099 * ext + pad, dtype=torch.uint8, device='cuda')
    small_in = torch.ones(4099 * ext + pad, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    h_small_io = small_io.cpu().numpy()[4:4 + 4099 * ext].copy()
    h_small_in = small_in.cpu().numpy()[4:4 + 4099 * ext].copy()
    assert oracle.reduce_local(h_small_in, h_small_io, 4099, dt, MPI_SUM) == 0
    ins = (ctypes.c_void_p * 2)(small_in.data_ptr() + 4, src.data_ptr())
    ios = (ctypes.c_void_p * 2)(small_io.data_ptr() + 4, io.data_ptr())
    cnt = (ctypes.c_ssize_t * 2)(4099, count)
    assert R.lib().MPIX_Reduce_local_batch_async(ins, ios, cnt, 2, dt, MPI_SUM, s.cuda_stream) == 0
    s.synchronize()
    bad['batch'] = _bytes_equal(io, exp)
    bad['batch_small'] = _bytes_equal(small_io[4:4 + 4099 * ext], h_small_io)
    del small_io, small_in
    # multi-input k = 2: inout = (inout + in) + in2, one pass
    src = reset(off_io)
    d_in2 = _random_bytes(nb, 0x5EED1A20 + ext, ext)
    in2_buf = torch.empty(nb + pad, dtype=torch.uint8, device='cuda')
    in2 = in2_buf[off_io:off_io + nb]
    in2.copy_(d_in2)
    h_in2 = d_in2.cpu().numpy()
    del d_in2
    exp2 = exp.copy()
    assert oracle.reduce_local(h_in2, exp2, count, dt, MPI_SUM, nthreads=8) == 0
    torch.cuda.synchronize()
    arr = (ctypes.c_void_p * 2)(src.data_ptr(), in2.data_ptr())
    assert R.lib().MPIX_Reduce_local_multi_async(arr, 2, io.data_ptr(), count, dt, MPI_SUM,
                                                 s.cuda_stream) == 0
    s.synchronize()
    bad['multi'] = _bytes_equal(io, exp2)
    assert all(v is None for v in bad.values()), bad


# ---------------------------------------------------------------- 2^32 packets
# with one 16-byte packet per lane in one-wave blocks, an operand
# of 2^32 packets (64 GiB) needs 2^26 blocks of 64 lanes -- exactly where a
# dispatch passes UINT32_MAX work-items.  grid_for caps the grid at
# floor((2^32 - 1) / block) blocks (tests/test_grid_cap.py checks the rule on
# the host); here the capped kernels run on the GPU and stride over the rest.
# 64 GiB per operand: the operands are closed-form byte patterns made and
# checked chunk by chunk on the device (in[i] = 7i + 3, inout[i] = 13i + 1,
# mod 256; MPI_INT8_T SUM wraps mod 256, so the result is 20i + 4, and the
# two-input fold inout + in + in is 27i + 7) -- an oracle pass over 128 GiB of
# host memory would take minutes.
HUGE = (1 << 36) + 4099             # elements (bytes) per operand, > 2^32 packets
CHUNK = 1 << 28


def _pattern(t, a, b, start=0):
    """t[j] = (a * (start + j) + b) mod 256, made in CHUNK pieces"""
    for s in range(0, t.numel(), CHUNK):
        e = min(t.numel(), s + CHUNK)
        i = torch.arange(start + s, start + e, dtype=torch.int64, device='cuda')
        t[s:e].copy_(((i * a + b) & 0xff).to(torch.uint8))
        del i


def _pattern_mismatch(t, a, b):
    for s in range(0, t.numel(), CHUNK):
        e = min(t.numel(), s + CHUNK)
        i = torch.arange(s, e, dtype=torch.int64, device='cuda')
        want = ((i * a + b) & 0xff).to(torch.uint8)
        if not torch.equal(t[s:e], want):
            bad = torch.nonzero(t[s:e] != want)
            return 'chunk at %d: %d bytes differ, first at %d' % (s, bad.numel(), s + int(bad[0]))
    return None


@pytest.mark.timeout(900)
def test_past_2_32_packets_every_entry(R):
    free, _ = torch.cuda.mem_get_info()
    if free < 2 * HUGE + (16 << 30):
        pytest.skip('needs ~144 GiB of free device memory (have %d GiB)' % (free >> 30))
    off = 3                         # inout and in off the 16-byte grid, same phase
    io_buf = torch.empty(HUGE + 64, dtype=torch.uint8, device='cuda')
    in_buf = torch.empty(HUGE + 64, dtype=torch.uint8, device='cuda')
    io = io_buf[off:off + HUGE]
    src = in_buf[off:off + HUGE]
    io_buf[:off].fill_(0xA5)
    io_buf[off + HUGE:].fill_(0xA5)
    _pattern(src, 7, 3)
    s = torch.cuda.current_stream()
    bad = {}

    def reset():
        _pattern(io, 13, 1)
        torch.cuda.synchronize()

    reset()
    assert R.lib().MPIX_Reduce_local(src.data_ptr(), io.data_ptr(), HUGE, MPI_INT8_T, MPI_SUM) == 0
    bad['sync'] = _pattern_mismatch(io, 20, 4)
    reset()
    assert R.reduce_local_async(src.data_ptr(), io.data_ptr(), HUGE, MPI_INT8_T, MPI_SUM, s) == 0
    s.synchronize()
    bad['async'] = _pattern_mismatch(io, 20, 4)
    # batch: a small segment beside the huge one (the huge one exceeds one
    # grid's blocks, so it goes as a capped launch of its own)
    reset()
    small_io = torch.zeros(4099 + 64, dtype=torch.uint8, device='cuda')
    small_in = torch.full((4099 + 64,), 5, dtype=torch.uint8, device='cuda')
    ins = (ctypes.c_void_p * 2)(small_in.data_ptr() + 4, src.data_ptr())
    ios = (ctypes.c_void_p * 2)(small_io.data_ptr() + 4, io.data_ptr())
    cnt = (ctypes.c_ssize_t * 2)(4099, HUGE)
    assert R.lib().MPIX_Reduce_local_batch_async(ins, ios, cnt, 2, MPI_INT8_T, MPI_SUM,
                                                 s.cuda_stream) == 0
    s.synchronize()
    bad['batch'] = _pattern_mismatch(io, 20, 4)
    bad['batch_small'] = None if bool(torch.all(small_io[4:4 + 4099] == 5)) and \
        bool(torch.all(small_io[:4] == 0)) and bool(torch.all(small_io[4 + 4099:] == 0)) \
        else 'small segment wrong'
    # multi-input k = 2, the same input twice: inout + in + in
    reset()
    arr = (ctypes.c_void_p * 2)(src.data_ptr(), src.data_ptr())
    assert R.lib().MPIX_Reduce_local_multi_async(arr, 2, io.data_ptr(), HUGE, MPI_INT8_T, MPI_SUM,
                                                 s.cuda_stream) == 0
    s.synchronize()
    bad['multi'] = _pattern_mismatch(io, 27, 7)
    # the bytes around inout never written
    bad['guard'] = None if bool(torch.all(io_buf[:off] == 0xA5)) and \
        bool(torch.all(io_buf[off + HUGE:] == 0xA5)) else 'bytes outside inout written'
    del io_buf, in_buf, io, src
    torch.cuda.empty_cache()
    assert all(v is None for v in bad.values()), bad
