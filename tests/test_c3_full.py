"""BASELINE config 3 at its stated size: every (op, type) pair of the GPU
path (the 170 cases of test_gpu_parity's sweep) on 256 MiB per operand, the
HIP result bit for bit against the oracle (MPI_SUM/PROD on fp: a NaN need only
be a NaN, arithmetic NaN payloads are unpinned -- test_gpu_parity's rule).

At that size the operands are drawn on the GPU (torch's seeded Philox
generator, the same value distributions as test_gpu_parity's numpy
generators: logical zeros, fp specials and subnormals, bf16 ties-away cases,
pair ties and NaNs, random pair padding), the oracle runs on 8 host threads
and the comparison runs on the device, so the 170 cases fit the GPU suite.
MPIX_C3_BYTES overrides the per-operand size."""
import os

import numpy as np
import pytest
import torch

from tests.test_gpu_parity import SWEEP

pytestmark = pytest.mark.gpu

C3_BYTES = int(os.environ.get('MPIX_C3_BYTES', 256 << 20))
ORACLE_THREADS = 8


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


FDT = {2: torch.float16, 4: torch.float32, 8: torch.float64}
IDT = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def _bytes(g, nbytes):
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device='cuda', generator=g)


def _u(g, n, dt=torch.float32):
    return torch.rand(n, dtype=dt, device='cuda', generator=g)


def _fp(g, n, size):
    x = (_u(g, n, torch.float64 if size == 8 else torch.float32) * 2 - 1).to(FDT[size])
    sp = torch.tensor([0.0, -0.0, float('inf'), float('-inf'), float('nan')], dtype=FDT[size],
                      device='cuda')
    k = _u(g, n) < 0.01
    x[k] = sp[torch.randint(0, 5, (int(k.sum()),), device='cuda', generator=g)]
    if size == 4:       # subnormals must not be flushed
        d = _u(g, n) < 0.003
        x[d] = ((_u(g, int(d.sum())) * 2 - 1) * 1e-39).to(torch.float32)
    return x.view(torch.uint8)


def operand(g, kind, size, n):
    """one operand of n elements as a device uint8 tensor"""
    if kind == 'int':
        a = _bytes(g, n * size).view(n, size)
        a[_u(g, n) < 0.3] = 0                   # logical-false elements
        return a.reshape(-1)
    if kind == 'flog':
        vals = torch.tensor([0, 1, -1, 5, 0], dtype=torch.int64, device='cuda')
        v = vals[torch.randint(0, 5, (n,), device='cuda', generator=g)]
        if size <= 8:
            return v.to(IDT[size]).view(torch.uint8)
        return torch.stack([v, torch.where(v < 0, -1, 0)], 1).view(torch.uint8).reshape(-1)
    if kind == 'fp':
        return _fp(g, n, size)
    if kind == 'cplx':
        return _fp(g, 2 * n, size)
    if kind == 'bf16':
        f = _u(g, n) * 8 - 4
        k = _u(g, n) < 0.01
        sp = torch.tensor([float('inf'), float('-inf'), 0.0, -0.0], device='cuda')
        f[k] = sp[torch.randint(0, 4, (int(k.sum()),), device='cuda', generator=g)]
        b = (f.view(torch.int32) >> 16).to(torch.int32) & 0xffff
        b ^= torch.randint(0, 2, (n,), dtype=torch.int32, device='cuda', generator=g)
        nan = ((b & 0x7f80) == 0x7f80) & ((b & 0x7f) != 0)
        b[nan] = 0x3f80
        return b.to(torch.int16).view(torch.uint8)
    vdt, ldt, ext, loff = kind[1:]
    buf = _bytes(g, n * ext).view(n, ext)       # random padding
    vs, ls = np.dtype(vdt).itemsize, np.dtype(ldt).itemsize
    v = torch.randint(0, 16, (n,), device='cuda', generator=g)
    if vdt.startswith('<f'):
        v = v.to(FDT[vs])
        v[_u(g, n) < 0.02] = float('nan')
    else:
        v = v.to(IDT[vs])
    lv = torch.randint(-1000, 1000, (n,), device='cuda', generator=g).to(IDT[ls])
    buf[:, :vs] = v.view(torch.uint8).view(n, vs)
    buf[:, loff:loff + ls] = lv.view(torch.uint8).view(n, ls)
    return buf.reshape(-1)


def _nan(t, kind, size):
    if kind in ('fp', 'cplx'):
        return torch.isnan(t.view(FDT[size]))
    b = t.view(torch.int16).to(torch.int32) & 0xffff
    return ((b & 0x7f80) == 0x7f80) & ((b & 0x7f) != 0)


def mismatches(got, exp, kind, size, opname, ext):
    """test_gpu_parity.compare on the device"""
    if opname in ('MPI_SUM', 'MPI_PROD') and kind in ('fp', 'cplx', 'bf16'):
        comp = size if kind != 'bf16' else 2
        gb, eb = got.view(-1, comp), exp.view(-1, comp)
        bits = (gb != eb).any(1)                # per scalar component
        gn, en = _nan(got, kind, size), _nan(exp, kind, size)
        bad = torch.where(gn | en, gn != en, bits)
        per = 2 if kind == 'cplx' else 1
        return int(bad.view(-1, per).any(1).sum())
    return int((got.view(-1, ext) != exp.view(-1, ext)).any(1).sum())


@pytest.mark.parametrize('dtname,opname,kind,size', SWEEP,
                         ids=['%s-%s' % (s[0], s[1]) for s in SWEEP])
def test_c3_full_size(R, H, oracle, dtname, opname, kind, size):
    dt, op = getattr(H, dtname), getattr(H, opname)
    assert R.is_supported(op, dt), (dtname, opname)
    ext = R.datatype_extent(dt)
    n = C3_BYTES // ext + 7                     # ragged: not a multiple of any packet
    g = torch.Generator(device='cuda')
    g.manual_seed((0x5EED0003 * 31 + dt * 7 + op) & 0xffffffff)
    da = operand(g, kind, size, n)
    db = operand(g, kind, size, n)
    torch.cuda.synchronize()
    a, b = da.cpu().numpy(), db.cpu().numpy()
    assert R.MPI_Reduce_local(db, da, n, dt, op) == 0
    assert oracle.reduce_local(b, a, n, dt, op, nthreads=ORACLE_THREADS) == 0
    exp = torch.from_numpy(a).cuda()
    assert torch.equal(db, torch.from_numpy(b).cuda())      # inbuf untouched
    assert mismatches(da, exp, kind, size, opname, ext) == 0
