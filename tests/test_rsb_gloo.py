"""Multi-process CPU coverage of the N>1 path: the C++ schedules of
libmpix_coll.so (the library MPICH would link, include/mpix_coll.h) run as
one process per rank, over a custom host-memory communicator whose exchange
steps are gloo batch_isend_irecv groups (mpich_amd/coll.py), the oracle
installed as the combine (a C function: the product has no CPU compute path).
World sizes 2..8, power-of-two and not.  Checks (a) bit-identity with the
oracle's single-process simulation of the reference schedule
(reduce_scatter_block_intra_recursive_halving.c:38-260, …_pairwise.c:42-104,
allreduce_intra_reduce_scatter_allgather.c:41-277) and (b) the reference's
own closed forms (test/mpi/coll/redscatblk3.c:48-78, allred.c KATs).

Every case of one world size runs in ONE spawn of `world` processes (one
gloo process group, the cases one after another), so the suite pays the
process start-up once per world size; each test then checks its own case."""
import os
import socket
from datetime import timedelta

import numpy as np
import pytest
import torch.multiprocessing as mp

MPI_FLOAT, MPI_INT, MPI_SUM = 0x4c00040a, 0x4c000405, 0x58000003


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


# (kind, mode, count, algo) per case; algo suffixes: '+small' = every message
# split into 256-byte pieces, '+inplace' = MPI_IN_PLACE (inputs in recvbuf)
RSB_IN_PLACE = [(2, 'recursive_halving'), (3, 'recursive_halving'), (5, 'recursive_halving'),
                (4, 'pairwise'), (3, 'pairwise_sequential')]
RSB_WORLDS = [2, 3, 4, 5, 8]
RSB_SPLIT = [(3, 'recursive_halving'), (4, 'recursive_halving'), (4, 'pairwise'),
             (3, 'pairwise_sequential')]
RSB_KAT_WORLDS = [2, 3, 4]
PAIRWISE_ALGOS = ['pairwise', 'pairwise_sequential', 'pull']
PAIRWISE_WORLDS = [2, 3, 4, 7]
AR_ALGOS = ['reduce_scatter_allgather', 'rsag_rd_allgather', 'recursive_doubling',
            'rsag_multipath']
AR_WORLDS = [2, 3, 4, 7, 8]


def _ar_count(algo):
    return 4096 if algo == 'rsag_multipath' else 1037    # multipath: P | count


def _cases(world):
    cs = []
    for w, a in RSB_IN_PLACE:
        if w == world:
            cs.append(('rsb', 'float', 1001, a + '+inplace'))
    if world in RSB_WORLDS:
        cs.append(('rsb', 'float', 1001, 'recursive_halving'))
    for w, a in RSB_SPLIT:
        if w == world:
            cs.append(('rsb', 'float', 1001, a + '+small'))
    if world in RSB_KAT_WORLDS:
        cs.append(('rsb', 'int', (1024 * 1024) // world // 64, 'recursive_halving'))
    if world in PAIRWISE_WORLDS:
        for a in PAIRWISE_ALGOS:
            cs.append(('rsb', 'float', 777, a))
            cs.append(('rsb', 'int', 1000, a))
    if world in AR_WORLDS:
        for a in AR_ALGOS:
            if a != 'rsag_multipath' or world in (4, 8):
                cs.append(('ar', 'float', _ar_count(a), a))
    return cs


def _case_dir(outdir, case):
    return os.path.join(outdir, '_'.join(str(x) for x in case).replace('+', '-'))


def _rsb_case(rank, world, outdir, mode, recvcount, algo, coll, orc):
    import torch
    small = algo.endswith('+small')
    if small:
        algo = algo[:-len('+small')]
    in_place = algo.endswith('+inplace')    # MPI_IN_PLACE: inputs in recvbuf, sendbuf None
    if in_place:
        algo = algo[:-len('+inplace')]
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
    saved = coll.MAX_MSG_BYTES
    if small:
        coll.MAX_MSG_BYTES = 256
    try:
        if algo == 'recursive_halving':
            tl = []     # the per-step timer is inert on host buffers
            coll.reduce_scatter_block(sendt, recv, recvcount, dt, MPI_SUM, combine=combine,
                                      timer=tl)
            assert tl == []
        elif algo == 'pull':        # host communicator: the pairwise schedule, same bits
            coll.reduce_scatter_block_pull(sendt, recv, recvcount, dt, MPI_SUM, combine=combine)
        else:
            coll.reduce_scatter_block_pairwise(sendt, recv, recvcount, dt, MPI_SUM,
                                               combine=combine, concurrent=(algo == 'pairwise'))
    finally:
        coll.MAX_MSG_BYTES = saved
    np.save(os.path.join(outdir, 'send%d.npy' % rank), send)
    np.save(os.path.join(outdir, 'recv%d.npy' % rank), recv.numpy()[:recvcount])


def _ar_case(rank, world, outdir, count, algo, coll, orc):
    import torch
    from tests import golden_util as gu
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
                (algo != 'recursive_doubling' and c['count'] < (1 << (world.bit_length() - 1))):
            continue
        ext = len(c['expected']) // c['count']
        out = torch.zeros(c['count'] * ext, dtype=torch.uint8)
        fn(torch.from_numpy(c['inputs'][rank].copy()), out, c['count'], c['datatype'], c['op'],
           combine=combine)
        if gu.mismatches(c, out.numpy()):
            bad.append(c['id'])
    with open(os.path.join(outdir, 'bad%d.txt' % rank), 'w') as f:
        f.write(' '.join(bad))


def _worker(rank, world, port, outdir, cases):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    # a schedule that hangs fails its world's tests instead of the suite
    dist.init_process_group('gloo', rank=rank, world_size=world, timeout=timedelta(seconds=180))
    from oracle import oracle as orc
    from mpich_amd import coll
    for case in cases:
        kind, mode, count, algo = case
        d = _case_dir(outdir, case)
        os.makedirs(d, exist_ok=True)
        if kind == 'rsb':
            _rsb_case(rank, world, d, mode, count, algo, coll, orc)
        else:
            _ar_case(rank, world, d, count, algo, coll, orc)
        dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


_RUNS = {}


@pytest.fixture(scope='module')
def world_run(tmp_path_factory):
    """world -> directory holding every case's outputs (one spawn per world)"""
    def get(world):
        if world not in _RUNS:
            outdir = str(tmp_path_factory.mktemp('gloo%d' % world))
            try:
                mp.spawn(_worker, args=(world, _free_port(), outdir, _cases(world)),
                         nprocs=world, join=True)
                _RUNS[world] = (outdir, None)
            except Exception as e:      # every test of this world reports it
                _RUNS[world] = (outdir, e)
        outdir, err = _RUNS[world]
        if err is not None:
            raise err
        return outdir
    return get


def _load(world_run, world, case):
    d = _case_dir(world_run(world), case)
    sends = [np.load(os.path.join(d, 'send%d.npy' % r)) for r in range(world)]
    recvs = [np.load(os.path.join(d, 'recv%d.npy' % r)) for r in range(world)]
    return d, sends, recvs


@pytest.mark.parametrize('world,algo', RSB_IN_PLACE)
def test_rsb_gloo_in_place(oracle, world_run, world, algo):
    """MPI_IN_PLACE (sendbuf None): the inputs sit in recvbuf, the result
    lands in its first block; same bits as the oracle's schedule"""
    _, sends, recvs = _load(world_run, world, ('rsb', 'float', 1001, algo + '+inplace'))
    sim = oracle.rsb_pairwise if algo != 'recursive_halving' else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], 1001, MPI_FLOAT, MPI_SUM)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('world', RSB_WORLDS)
def test_rsb_gloo_matches_oracle_schedule(oracle, world_run, world):
    _, sends, recvs = _load(world_run, world, ('rsb', 'float', 1001, 'recursive_halving'))
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], 1001, MPI_FLOAT, MPI_SUM)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('world,algo', RSB_SPLIT)
def test_rsb_gloo_split_messages(oracle, world_run, world, algo):
    """messages above MAX_MSG_BYTES travel as several same-peer messages
    (here every block in 256-byte pieces): same bits as the oracle"""
    _, sends, recvs = _load(world_run, world, ('rsb', 'float', 1001, algo + '+small'))
    sim = oracle.rsb_pairwise if algo != 'recursive_halving' else oracle.rsb_recursive_halving
    exp = sim([s.view(np.uint8) for s in sends], 1001, MPI_FLOAT, MPI_SUM)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r


@pytest.mark.parametrize('world', RSB_KAT_WORLDS)
def test_rsb_gloo_redscatblk3(world_run, world):
    _, _, recvs = _load(world_run, world,
                        ('rsb', 'int', (1024 * 1024) // world // 64, 'recursive_halving'))
    for r in range(world):
        assert np.all(recvs[r] == world * r + world * (world - 1) // 2)


@pytest.mark.parametrize('algo', PAIRWISE_ALGOS)
@pytest.mark.parametrize('world', PAIRWISE_WORLDS)
def test_pairwise_gloo_matches_oracle(oracle, world_run, world, algo):
    """concurrent (one group, all links) and the reference's sequential
    exchange give the reference pairwise association bit-for-bit."""
    _, sends, recvs = _load(world_run, world, ('rsb', 'float', 777, algo))
    exp = oracle.rsb_pairwise([s.view(np.uint8) for s in sends], 777, MPI_FLOAT, MPI_SUM)
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r
    _, _, recvs = _load(world_run, world, ('rsb', 'int', 1000, algo))
    for r in range(world):
        assert np.all(recvs[r] == world * r + world * (world - 1) // 2)


@pytest.mark.parametrize('algo', AR_ALGOS)
@pytest.mark.parametrize('world', AR_WORLDS)
def test_allreduce_gloo(oracle, world_run, world, algo):
    """Rabenseifner allreduce over gloo (direct or the reference's
    recursive-doubling allgather): bit-identical on every rank to the
    oracle's simulation of the reference schedule, and all allred.c KATs
    generated for this world size pass end to end."""
    if algo == 'rsag_multipath' and world not in (4, 8):
        pytest.skip('other P run the plain steps (the fallback is covered in test_coll_c)')
    count = _ar_count(algo)
    d, sends, recvs = _load(world_run, world, ('ar', 'float', count, algo))
    exp = oracle.allreduce_rabenseifner([s.view(np.uint8) for s in sends], count, MPI_FLOAT,
                                        MPI_SUM,
                                        algorithm='recursive_doubling' if algo == 'recursive_doubling'
                                        else 'reduce_scatter_allgather')
    for r in range(world):
        assert recvs[r].tobytes() == exp[r].tobytes(), r
        assert open(os.path.join(d, 'bad%d.txt' % r)).read() == '', r
