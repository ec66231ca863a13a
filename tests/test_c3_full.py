"""BASELINE config 3 at its stated size: every (op, type) pair of the GPU
path (the 170 cases of test_gpu_parity's sweep) on 256 MiB per operand, the
HIP result bit for bit against the oracle (MPI_SUM/PROD on fp: a NaN need only
be a NaN, arithmetic NaN payloads are unpinned -- test_gpu_parity's rule).

At that size the operands are drawn on the GPU (bench.c3_operand: torch's
seeded Philox generator, the same value distributions as test_gpu_parity's
numpy generators: logical zeros, fp specials and subnormals, bf16 ties-away
cases, pair ties and NaNs, random pair padding; the bench's config-3 rows time
on the same generator), the oracle runs on 8 host threads
and the comparison runs on the device, so the 170 cases fit the GPU suite.
MPIX_C3_BYTES overrides the per-operand size."""
import os

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


from bench import C3_FDT as FDT  # noqa: E402
from bench import c3_operand as operand  # noqa: E402


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
