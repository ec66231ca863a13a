"""Multi-process CPU coverage of the N>1 path: the C++ schedules of
libmpix_coll.so (the library MPICH would link, include/mpix_coll.h) run as
one process per rank, over a custom host-memory communicator whose exchange
steps are gloo batch_isend_irecv groups (mpich_amd/coll.py), the oracle
installed as the combine (a C function: the product has no CPU compute path).
World sizes 2..8, power-of-two and not.  Checks (a) bit-identity with the
oracle's single-process simulation of the reference schedule
(reduce_scatter_block_intra_recursive_halving.c:38-260, …_pairwise.c:42-104)
and (b) the reference's own closed form (test/mpi/coll/redscatblk3.c:48-78)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, recvcount, mode, algo='recursive_halving'):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from oracle import oracle as orc
    from mpich_amd import coll
    if algo.endswith('+small'):     # every message split into 256-byte pieces
        coll.MAX_MSG_BYTES = 256
        algo = algo[:-len('+small')]
    in_place = algo.endswith('+inplace')    # MPI_IN_PLACE: inputs in recvbuf, sendbuf None
    if in_place:
        algo = algo[:-len('+inplace')]
    MPI_FLOAT, MPI_INT, MPI_SUM = 0x4c00040a, 0x4c000405, 0x58000003
    if mode == 'float':
        rng = np.random.default_rng(0x5EED0100 + rank)
        send = rng.uniform(-1, 1, world * recvcount).astype(np.float32)
        dt = MPI_FLOAT
    else:   # redscatblk3.c:43-48: block i of rank r holds r + i
        send = np.concatenate([np.full(recvcount, rank + i, np.int32) for i in range(world)])
        dt = MPI_INT
    sendt = torch.from_numpy(send.copy())
    recv = torch.zeros(recvcount, dtype=sendt.dtype)
    if in_place:
        recv, sendt = sendt, None

    combine = orc.combine_fn_address()
    if algo == 'recursive_halving':
        tl = []     # the per-step timer is inert on host buffers
        coll.reduce_scatter_block(sendt, recv, recvcount, dt, MPI_SUM, combine=combine, timer=tl)
        assert tl == []
    elif algo == 'pull':        # host communicator: the pairwise schedule, same bits
        coll.reduce_scatter_block_pull(sendt, recv, recvcount, dt, MPI_SUM, combine=combine)
    else:
        coll.reduce_scatter_block_pairwise(sendt, recv, recvcount, dt, MPI_SUM, combine=combine,
                                           concurrent=(algo == 'pairwise'))
    np.save(os.path.join(outdir, 'send%d.npy' % rank), send)
    np.save(os.path.join(outdir, 'recv%d.npy' % rank), recv.numpy()[:recvcount])
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


def _run(world, recvcount, mode, tmp_path, algo='recursive_halving'):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), recvcount, mode, algo),
             nprocs=world, join=True)
    sends = [np.load(tmp_path / ('send%d.npy' % r)) for r in range(world)]
    recvs = [np.load(tmp_path / ('recv%d.npy' % r)) for r in range(world)]
    return sends, recvs


@pytest.mark.parametrize('world,algo', [(2, 'recursive_halving'), (3, 'recursive_halving'),
                                        (5, 'recursive_halving'), (4, 'pairwise'),
                                        (3, 'pairwise_sequential')])
def test_rsb_gloo_in_place(oracle, tmp_path, world, algo):
    """MPI_IN_PLACE (sendbuf None): the inputs sit in recvbuf, the result
    lands in its first block; same bits as the oracle's schedule"""
    recvcount = 1001
    sends, recvs = _run(world, recvcount, 'float', tmp_path, algo + '+inplace')
    sim = oracle.rsb_pairwise if algo != 'recursive_halving' else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], recvcount, 0x4c00040a, 0x58000003)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('world', [2, 3, 4, 5, 8])
def test_rsb_gloo_matches_oracle_schedule(oracle, tmp_path, world):
    recvcount = 1001
    sends, recvs = _run(world, recvcount, 'float', tmp_path)
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], recvcount, 0x4c00040a,
                                       0x58000003)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('world,algo', [(3, 'recursive_halving'), (4, 'recursive_halving'),
                                        (4, 'pairwise'), (3, 'pairwise_sequential')])
def test_rsb_gloo_split_messages(oracle, tmp_path, world, algo):
    """messages above MAX_MSG_BYTES travel as several same-peer messages
    (here every block in 256-byte pieces): same bits as the oracle"""
    recvcount = 1001
    sends, recvs = _run(world, recvcount, 'float', tmp_path, algo + '+small')
    sim = oracle.rsb_pairwise if algo != 'recursive_halving' else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], recvcount, 0x4c00040a, 0x58000003)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('world', [2, 3, 4])
def test_rsb_gloo_redscatblk3(tmp_path, world):
    recvcount = (1024 * 1024) // world // 64
    _, recvs = _run(world, recvcount, 'int', tmp_path)
    for r in range(world):
        assert np.all(recvs[r] == world * r + world * (world - 1) // 2)


@pytest.mark.parametrize('algo', ['pairwise', 'pairwise_sequential', 'pull'])
@pytest.mark.parametrize('world', [2, 3, 4, 7])
def test_pairwise_gloo_matches_oracle(oracle, tmp_path, world, algo):
    """concurrent (one group, all links) and the reference's sequential
    exchange give the reference pairwise association bit-for-bit."""
    recvcount = 777
    sends, recvs = _run(world, recvcount, 'float', tmp_path, algo)
    exp = oracle.rsb_pairwise([s.view(np.uint8) for s in sends], recvcount, 0x4c00040a,
                              0x58000003)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r
    sends, recvs = _run(world, 1000, 'int', tmp_path, algo)
    for r in range(world):
        assert np.all(recvs[r] == world * r + world * (world - 1) // 2)


def _ar_worker(rank, world, port, outdir, count, algo='reduce_scatter_allgather'):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from oracle import oracle as orc
    from mpich_amd import coll
    from tests import golden_util as gu
    MPI_FLOAT, MPI_SUM = 0x4c00040a, 0x58000003
    rng = np.random.default_rng(0x5EED0200 + rank)
    send = rng.uniform(-1, 1, count).astype(np.float32)
    recv = torch.zeros(count, dtype=torch.float32)

    combine = orc.combine_fn_address()
    if algo == 'recursive_doubling':
        fn = coll.allreduce_recursive_doubling
    elif algo == 'rsag_multipath':
        def fn(*a, **k):
            return coll.allreduce(*a, algorithm='rsag_multipath', **k)
    else:   # second phase: one group of direct sends, or the reference's exchanges
        ag = 'recursive_doubling' if algo == 'rsag_rd_allgather' else 'direct'

        def fn(*a, **k):
            return coll.allreduce(*a, allgather=ag, **k)
    fn(torch.from_numpy(send.copy()), recv, count, MPI_FLOAT, MPI_SUM, combine=combine)
    np.save(os.path.join(outdir, 'send%d.npy' % rank), send)
    np.save(os.path.join(outdir, 'recv%d.npy' % rank), recv.numpy())
    # the allred.c KATs that were generated for this world size, end to end
    bad = []
    for c in gu.load_cases():
        if c['nranks'] != world or not c['name'].startswith('allred ') or \
                (algo != 'recursive_doubling' and
                 c['count'] < (1 << (world.bit_length() - 1))):
            continue
        ext = len(c['expected']) // c['count']
        out = torch.zeros(c['count'] * ext, dtype=torch.uint8)
        fn(torch.from_numpy(c['inputs'][rank].copy()), out, c['count'], c['datatype'], c['op'],
           combine=combine)
        if gu.mismatches(c, out.numpy()):
            bad.append(c['id'])
    with open(os.path.join(outdir, 'bad%d.txt' % rank), 'w') as f:
        f.write(' '.join(bad))
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize('algo', ['reduce_scatter_allgather', 'rsag_rd_allgather',
                                  'recursive_doubling', 'rsag_multipath'])
@pytest.mark.parametrize('world', [2, 3, 4, 7, 8])
def test_allreduce_gloo(oracle, tmp_path, world, algo):
    """Rabenseifner allreduce over gloo (direct or the reference's
    recursive-doubling allgather): bit-identical on every rank to the
    oracle's simulation of the reference schedule, and all allred.c KATs
    generated for this world size pass end to end."""
    if algo == 'rsag_multipath' and world not in (4, 8):
        pytest.skip('other P run the plain steps (the fallback is covered in test_coll_c)')
    count = 4096 if algo == 'rsag_multipath' else 1037    # multipath: P | count
    mp.spawn(_ar_worker, args=(world, _free_port(), str(tmp_path), count, algo), nprocs=world,
             join=True)
    sends = [np.load(tmp_path / ('send%d.npy' % r)) for r in range(world)]
    exp = oracle.allreduce_rabenseifner([s.view(np.uint8) for s in sends], count, 0x4c00040a,
                                        0x58000003,
                                        algorithm='recursive_doubling' if algo == 'recursive_doubling'
                                        else 'reduce_scatter_allgather')
    for r in range(world):
        assert np.load(tmp_path / ('recv%d.npy' % r)).tobytes() == exp[r].tobytes(), r
        assert open(tmp_path / ('bad%d.txt' % r)).read() == '', r
