"""Fused pull + combine reduce-scatter over hipIpc-mapped peer buffers
(MPIX_RSB_PULL of libmpix_coll, the C entry point), rehearsed with several
processes sharing the one GPU of the test box: the library publishes IPC
handles and runs its barriers over the communicator's transport (gloo through
pinned staging here); the kernel reads the peers' device memory directly.
Result must equal the reference pairwise schedule (oracle simulation) bit for
bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, recvcount, dtype_name):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from mpich_amd import coll
    from mpich_amd import handles as H
    rng = np.random.default_rng(0x5EED0300 + rank)
    in_place = dtype_name.endswith('_inplace')
    if dtype_name.startswith('float'):
        send = rng.uniform(-1, 1, world * recvcount).astype(np.float32)
        dt, op = H.MPI_FLOAT, H.MPI_SUM
    else:
        send = rng.integers(-100, 100, world * recvcount).astype(np.int32)
        dt, op = H.MPI_INT, H.MPI_MAX
    ds = torch.from_numpy(send).cuda()
    if in_place:                # MPI_IN_PLACE: peers pull from recvbuf itself
        dr = ds.clone()
        coll.reduce_scatter_block_pull(None, dr, recvcount, dt, op)
    else:
        dr = torch.empty(recvcount, dtype=ds.dtype, device='cuda')
        for _ in range(2):      # second call reuses the cached peer mappings
            coll.reduce_scatter_block_pull(ds, dr, recvcount, dt, op)
    torch.cuda.synchronize()
    np.save(os.path.join(outdir, 'send%d.npy' % rank), send)
    np.save(os.path.join(outdir, 'recv%d.npy' % rank), dr[:recvcount].cpu().numpy())
    dist.barrier()
    coll.free_comms()           # closes the cached peer mappings
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,dtype_name', [(2, 'float'), (3, 'int'), (4, 'float'),
                                              (3, 'float_inplace')])
def test_pull_combine_matches_pairwise(oracle, tmp_path, world, dtype_name):
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    recvcount = 100003
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), recvcount, dtype_name),
             nprocs=world, join=True)
    sends = [np.load(tmp_path / ('send%d.npy' % r)) for r in range(world)]
    dt, op = (0x4c00040a, 0x58000003) if dtype_name.startswith('float') else \
        (0x4c000405, 0x58000001)
    exp = oracle.rsb_pairwise([s.view(np.uint8) for s in sends], recvcount, dt, op)
    for r in range(world):
        assert np.load(tmp_path / ('recv%d.npy' % r)).tobytes() == exp[r].tobytes(), r
