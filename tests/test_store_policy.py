"""The contiguous, multi-input and tree kernels' store policy
(MPIX_Redop_set_store_policy: write-through on some XCDs / blocks, the rest
non-temporal) is a performance knob: every policy must give the same bits,
equal to the oracle's.  The CPU part checks the knob's arguments."""
import numpy as np
import pytest
import torch

POLICIES = [(0, 0, 0, 0), (0x88, 0, 0, 0), (0xff, 0, 0, 0), (0, 4, 3, 0), (0, 0, 0, 7),
            (0x22, 3, 1, 5)]


def test_store_policy_arguments():
    from mpich_amd import redop
    old = redop.get_store_policy()
    try:
        for bad in ((-2, 0, 0, 0), (0x100, 0, 0, 0), (0, -1, 0, 0), (0, 4, 4, 0), (0, 0, 1, 0),
                    (0, 0, 0, -1)):
            assert redop.set_store_policy(*bad) != 0, bad
        assert redop.set_store_policy(0x81, 8, 5, 16) == 0
        assert redop.get_store_policy() == dict(xcd_mask=0x81, every=8, phase=5, tail_blocks=16)
        # -1: back to the default (settled at the first launch; -1 until then)
        assert redop.set_store_policy(-1, 0, 0, 0) == 0
        assert redop.get_store_policy()['xcd_mask'] in (-1, 0, 0x88)
    finally:
        assert redop.set_store_policy(old['xcd_mask'], old['every'], old['phase'],
                                      old['tail_blocks']) == 0


def test_sync_store_policy_resolution():
    """the synchronous entry has its own mask.  Unset
    (-1) it follows an explicit MPIX_Redop_set_store_policy mask, else its
    own default (0x22 on 8-XCD devices, settled at the first launch; -1 until
    then); set, it wins for the synchronous entry only"""
    from mpich_amd import redop
    old = redop.get_store_policy()
    old_sync = redop.get_sync_store_policy()
    try:
        for bad in (-2, 0x100):
            assert redop.set_sync_store_policy(bad) != 0, bad
        assert redop.set_sync_store_policy(-1) == 0
        assert redop.set_store_policy(0x81, 0, 0, 0) == 0
        assert redop.get_sync_store_policy() == 0x81           # the explicit mask
        assert redop.set_sync_store_policy(0x22) == 0
        assert redop.get_sync_store_policy() == 0x22
        assert redop.get_store_policy()['xcd_mask'] == 0x81    # the others keep theirs
        assert redop.set_sync_store_policy(-1) == 0
        assert redop.set_store_policy(-1, 0, 0, 0) == 0
        assert redop.get_sync_store_policy() in (-1, 0, 0x22)
    finally:
        assert redop.set_store_policy(old['xcd_mask'], old['every'], old['phase'],
                                      old['tail_blocks']) == 0
        assert redop.set_sync_store_policy(-1 if old_sync in (-1, 0x22) else old_sync) == 0


@pytest.mark.gpu
@pytest.mark.parametrize('dtname,opname', [('MPI_FLOAT', 'MPI_SUM'), ('MPI_INT64_T', 'MPI_BXOR'),
                                           ('MPI_2INT', 'MPI_MAXLOC'), ('MPIX_C_FLOAT16', 'MPI_MAX')])
def test_every_store_policy_same_bits(oracle, dtname, opname):
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mpich_amd import handles as H
    from mpich_amd import redop
    assert redop.lib().MPIX_Redop_init() == 0
    dt, op = getattr(H, dtname), getattr(H, opname)
    ext = redop.datatype_extent(dt)
    rng = np.random.default_rng(0x5EED0300)
    n = (3 << 20) // ext + 5           # > 2 blocks per XCD, ragged tail
    a = rng.integers(0, 16, n * ext, dtype=np.uint8)
    bs = [rng.integers(0, 16, n * ext, dtype=np.uint8) for _ in range(4)]
    cdt, cop = H.as_c_int(dt), H.as_c_int(op)

    def orc(inb, inout):        # the oracle works in place: inout OP= inb
        assert oracle.reduce_local(inb, inout, n, cdt, cop) == 0
        return inout
    want1 = orc(bs[0], a.copy())
    want4 = a.copy()
    for b in bs:
        orc(b, want4)
    # tree of 4: ((b0 OP b1) OP (b2 OP b3)) with slot s = OP(slot s, slot s + m)
    want_tree = orc(orc(bs[3], bs[2].copy()), orc(bs[1], bs[0].copy()))
    old = redop.get_store_policy()
    dbs = [torch.from_numpy(b).cuda() for b in bs]
    try:
        for pol in POLICIES:
            assert redop.set_store_policy(*pol) == 0
            # the synchronous entry's own mask: the same masks in turn, and
            # the default (-1) for the first policy
            assert redop.set_sync_store_policy(pol[0] if pol != POLICIES[0] else -1) == 0
            d = torch.from_numpy(a.copy()).cuda()
            redop.check(redop.MPI_Reduce_local(dbs[0], d, n, dt, op))
            assert np.array_equal(d.cpu().numpy(), want1), ('contig', pol)
            d = torch.from_numpy(a.copy()).cuda()
            redop.check(redop.reduce_local_multi_async(dbs, d, n, dt, op))
            torch.cuda.synchronize()
            assert np.array_equal(d.cpu().numpy(), want4), ('multi', pol)
            out = torch.empty_like(dbs[0])
            redop.check(redop.reduce_local_tree_async(dbs, out, n, dt, op))
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), want_tree), ('tree', pol)
    finally:
        redop.set_store_policy(old['xcd_mask'], old['every'], old['phase'], old['tail_blocks'])
        redop.set_sync_store_policy(-1)
