"""The C++ schedules of libmpix_coll.so with the HIP combine, one PROCESS per
rank -- the way MPICH runs every collective test (test/mpi/coll/testlist.in,
`mpiexec -n N`; redscatblk3.c:48-78):

  * test_staged_*: any number of ranks on the test box's one GPU, over a
    custom communicator whose transport is gloo on host memory
    (MPIX_XPORT_STAGED: the library stages the device buffers through pinned
    memory around each exchange step, the MPIR_Coll_host_buffer_alloc pattern);
  * test_rccl_*: one rank per GPU over RCCL (MPIX_Comm_create_ccl, the
    transport of the 8-GPU bench), skipped below 2 devices.

Every rank's block is compared bit for bit with the oracle's single-process
simulation of the reference schedule (recursive halving:
reduce_scatter_block_intra_recursive_halving.c:38-260; pairwise, pipelined
pairwise and the fused pull: …_intra_pairwise.c:42-104; allreduce:
allreduce_intra_reduce_scatter_allgather.c:41-277)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

MPI_FLOAT, MPI_2INT = 0x4c00040a, 0x4c000816
MPI_SUM, MPI_MAXLOC = 0x58000003, 0x5800000c


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(rank, world, recvcount, kind):
    rng = np.random.default_rng(0x5EED0400 + rank)
    if kind == 'float':
        return rng.uniform(-1, 1, world * recvcount).astype(np.float32), MPI_FLOAT, MPI_SUM
    # MPI_2INT {value, loc}: values from 0..3 force ties (loc = min wins, opmaxloc.c)
    v = rng.integers(0, 4, world * recvcount).astype(np.int32)
    loc = rng.integers(0, 1 << 20, world * recvcount).astype(np.int32)
    return np.stack([v, loc], 1).reshape(-1), MPI_2INT, MPI_MAXLOC


def _worker(rank, world, port, outdir, backend, cases):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dev = rank if backend == 'nccl' else 0
    torch.cuda.set_device(dev)
    if backend == 'nccl':
        dist.init_process_group('nccl', rank=rank, world_size=world,
                                device_id=torch.device('cuda', dev))
    else:
        dist.init_process_group('gloo', rank=rank, world_size=world)
    from mpich_amd import coll
    for name, algo, kind, recvcount in cases:
        send, dt, op = _inputs(rank, world, recvcount, kind)
        ext = 8 if kind == 'pair' else 4
        ds = torch.from_numpy(send.view(np.uint8).copy()).cuda()
        if algo.startswith('allreduce'):
            dr = torch.empty_like(ds)
            coll.allreduce(ds, dr, world * recvcount, dt, op,
                           algorithm={'allreduce': 'reduce_scatter_allgather',
                                      'allreduce_rd': 'rsag_rd_allgather',
                                      'allreduce_mp': 'rsag_multipath',
                                      'allreduce_pull': 'pull'}[algo])
        else:
            dr = torch.empty(recvcount * ext, dtype=torch.uint8, device='cuda')
            timer = [] if algo == 'recursive_halving' else None
            for _ in range(2):      # the second call reuses scratch, mappings, staging
                coll.reduce_scatter_block(ds, dr, recvcount, dt, op, algorithm=algo, timer=timer)
            if timer is not None:           # per-step breakdown of both calls
                phases = [t['phase'] for t in timer]
                assert phases and phases[-1] == 'epilogue', phases
                if world & (world - 1) == 0:
                    assert phases.count('combine') + phases.count('combine (sent half)') == \
                        2 * (world.bit_length() - 1), phases
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, '%s_send%d.npy' % (name, rank)), send)
        np.save(os.path.join(outdir, '%s_recv%d.npy' % (name, rank)), dr.cpu().numpy())
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


def _check(oracle, tmp_path, world, cases):
    for name, algo, kind, recvcount in cases:
        sends = [np.load(tmp_path / ('%s_send%d.npy' % (name, r))) for r in range(world)]
        dt, op = (MPI_FLOAT, MPI_SUM) if kind == 'float' else (MPI_2INT, MPI_MAXLOC)
        raw = [s.view(np.uint8) for s in sends]
        if algo.startswith('recursive_halving'):
            exp = oracle.rsb_recursive_halving(raw, recvcount, dt, op)
        elif algo.startswith('allreduce'):
            exp = oracle.allreduce_rabenseifner(raw, world * recvcount, dt, op)
        else:
            exp = oracle.rsb_pairwise(raw, recvcount, dt, op)
        for r in range(world):
            got = np.load(tmp_path / ('%s_recv%d.npy' % (name, r)))
            assert got.tobytes() == exp[r].tobytes(), (name, r)


def _run(oracle, tmp_path, world, backend, cases):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), backend, cases), nprocs=world,
             join=True)
    _check(oracle, tmp_path, world, cases)


ALGOS = ('recursive_halving', 'pairwise', 'pairwise_pipelined', 'pull', 'recursive_halving_multipath',
         'recursive_halving_pull')


@pytest.mark.parametrize('world', [2, 3, 4, 8])
def test_staged_rsb_matches_oracle(oracle, tmp_path, world):
    """every reduce-scatter schedule, fp32 SUM and MPI_2INT MAXLOC, ranks as
    processes sharing the GPU, gloo transport through pinned staging"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    cases = [('%s_%s' % (a, k), a, k, 40009 if k == 'float' else 20011)
             for a in ALGOS for k in ('float', 'pair')]
    _run(oracle, tmp_path, world, 'gloo', cases)


def test_staged_pipelined_large_blocks(oracle, tmp_path):
    """blocks above 8 MiB: the pipelined pairwise schedule really cuts them
    into chunks (combine of chunk k on the second stream), same bits"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    cases = [('pipe', 'pairwise_pipelined', 'float', (10 << 20) // 4 + 3)]
    _run(oracle, tmp_path, 2, 'gloo', cases)


def _churn_worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mpich_amd import coll
    MPI_INT = 0x4c000405
    n = 65536 + 7
    bad = []
    for it in range(4):
        for algo in ('pull', 'recursive_halving_pull', 'allreduce_pull'):
            # block i of rank r holds r + i + 100 * it (redscatblk3.c:43-48), in a
            # fresh allocation each time: the previous one went back to the
            # driver, so a peer's cached mapping of it would read stale data
            blk = torch.cat([torch.full((n,), rank + i + 100 * it, dtype=torch.int32, device='cuda')
                             for i in range(world)])
            torch.cuda.synchronize()
            if algo == 'allreduce_pull':
                out = torch.empty_like(blk)
                coll.allreduce(blk, out, world * n, MPI_INT, MPI_SUM, algorithm='pull')
                exp = torch.cat([torch.full((n,), sum(q + i + 100 * it for q in range(world)),
                                            dtype=torch.int32, device='cuda')
                                 for i in range(world)])
            else:
                out = torch.empty(n, dtype=torch.int32, device='cuda')
                coll.reduce_scatter_block(blk, out, n, MPI_INT, MPI_SUM, algorithm=algo)
                exp = torch.full((n,), world * rank + world * (world - 1) // 2 + world * 100 * it,
                                 dtype=torch.int32, device='cuda')
            torch.cuda.synchronize()
            if not torch.equal(out, exp):
                bad.append('%s@%d' % (algo, it))
            dist.barrier()          # every peer done with this round's buffers
            del blk, out, exp
            torch.cuda.empty_cache()
    with open(os.path.join(outdir, 'churn%d.txt' % rank), 'w') as f:
        f.write(' '.join(bad))
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_staged_pulls_with_buffer_churn(tmp_path, world):
    """the pulls map peers' allocations once and cache the mappings: a buffer
    freed back to the driver and re-made (likely at the same address, maybe
    with the same IPC handle bytes) must not be read through the old mapping
    -- the published allocation identity invalidates it"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_churn_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert open(tmp_path / ('churn%d.txt' % r)).read() == '', r


def _shared_worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['MPIX_COLL_TRACE'] = '1'
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    trace = open(os.path.join(outdir, 'trace%d.txt' % rank), 'w')
    os.dup2(trace.fileno(), 2)          # the library's trace lines land in the file
    from mpich_amd import coll
    c = coll.comm_for(None, True)
    n = 40009
    send, dt, op = _inputs(rank, world, n, 'float')
    sh = c.shared_tensor(world * n, torch.float32)      # symmetric memory
    out_sh = c.shared_tensor(world * n, torch.float32)
    sh.copy_(torch.from_numpy(send))
    torch.cuda.synchronize()
    res = {}
    for algo in ('pull', 'recursive_halving_pull'):
        r = torch.empty(n, dtype=torch.float32, device='cuda')
        coll.reduce_scatter_block(sh, r, n, dt, op, algorithm=algo)
        res[algo] = r.cpu().numpy()
    coll.allreduce(sh, out_sh, world * n, dt, op, algorithm='pull')      # both shared
    res['allreduce_pull'] = out_sh.cpu().numpy()
    torch.cuda.synchronize()
    for name, v in res.items():
        np.save(os.path.join(outdir, 'sh_%s_recv%d.npy' % (name, rank)), v)
    np.save(os.path.join(outdir, 'sh_send%d.npy' % rank), send)
    c.free_shared(sh.data_ptr())
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_staged_pulls_on_shared_memory(oracle, tmp_path, world):
    """MPIX_Comm_alloc_shared: with every rank's buffers in symmetric shared
    memory the pulls read the peers' copies in place (the trace says
    'direct'), bit-identical to the oracle's schedules"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_shared_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    n = 40009
    raw = [np.load(tmp_path / ('sh_send%d.npy' % r)).view(np.uint8) for r in range(world)]
    exp = {'pull': oracle.rsb_pairwise(raw, n, MPI_FLOAT, MPI_SUM),
           'recursive_halving_pull': oracle.rsb_recursive_halving(raw, n, MPI_FLOAT, MPI_SUM),
           'allreduce_pull': oracle.allreduce_rabenseifner(raw, world * n, MPI_FLOAT, MPI_SUM)}
    for name, e in exp.items():
        for r in range(world):
            got = np.load(tmp_path / ('sh_%s_recv%d.npy' % (name, r)))
            assert got.tobytes() == e[r].tobytes(), (name, r)
    for r in range(world):
        t = open(tmp_path / ('trace%d.txt' % r)).read()
        assert t.count('shared-window pull: direct') == 3, t[-2000:]


def _fault_worker(rank, world, port, outdir, env):
    os.environ.update(env)
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from mpich_amd import coll
    seen = {}
    orig = coll.free_comms

    def record():       # what the bench helper reports for each leg, before the comm goes
        c = coll.comm_for(None, True)
        seen['state'] = c.state()
        seen['helper_allreduce_pull'] = bench.schedule_ran(c, 'pull', 'ar')
        orig()
    coll.free_comms = record
    cases = [('rhp_f', 'recursive_halving_pull', 'float', 40009),
             ('pull_f', 'pull', 'float', 40009), ('arp_f', 'allreduce_pull', 'float', 40009)]
    _worker(rank, world, port, outdir, 'gloo', cases)
    with open(os.path.join(outdir, 'state%d.json' % rank), 'w') as f:
        json.dump(seen, f)


FAULT_CASES = [('pull_f', 'pull', 'float', 40009),
               ('rhp_f', 'recursive_halving_pull', 'float', 40009),
               ('arp_f', 'allreduce_pull', 'float', 40009)]


@pytest.mark.parametrize('fault', ['window', 'node'])
def test_staged_pull_window_verification_failure(oracle, tmp_path, fault):
    """window: a window whose nonce does not read back on every peer -- all
    ranks retry (3 times), then agree to give the pulls up and run the
    RCCL-transport schedules; node: one rank reports another node, so no
    window is even allocated.  Same bits as the oracle, nobody hangs, and
    MPIX_Comm_get_state / bench.schedule_ran report the fallback (VERDICT r02
    item 2: never one schedule's time under another's name)"""
    import json
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    world = 4
    env = {'MPIX_COLL_WINDOW_FAULT': '1'} if fault == 'window' else {}
    envs = [dict(env, MPIX_COLL_NODE_ID='elsewhere') if fault == 'node' and r == 1 else env
            for r in range(world)]
    ctx = mp.get_context('spawn')
    port = _free_port()
    ps = [ctx.Process(target=_fault_worker, args=(r, world, port, str(tmp_path), envs[r]))
          for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
        assert p.exitcode == 0, p.exitcode
    _check(oracle, tmp_path, world, FAULT_CASES)
    for r in range(world):
        st = json.load(open(tmp_path / ('state%d.json' % r)))
        assert st['state']['pulls_enabled'] is False, st
        assert st['state']['last_allreduce'] == 'reduce_scatter_allgather', st
        # every pull call fell back: 2 calls each reduce-scatter case, 1 allreduce
        assert st['state']['fallbacks'] == 5, st
        assert st['state']['window_retries'] == (3 if fault == 'window' else 0), st
        h = st['helper_allreduce_pull']
        assert h['error'] == 'fell back to reduce_scatter_allgather', h


@pytest.mark.parametrize('world', [3, 4])
def test_staged_allreduce_matches_oracle(oracle, tmp_path, world):
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    cases = [('ar', 'allreduce', 'float', 25013), ('ar_rd', 'allreduce_rd', 'float', 25013),
             ('ar_mp', 'allreduce_mp', 'float', 2 << 20),    # P=4: 8 MiB parts, 2 relay chunks
             ('ar_pull', 'allreduce_pull', 'float', 25013)]
    _run(oracle, tmp_path, world, 'gloo', cases)


def _ragged_worker(rank, world, port, outdir):
    """MPI_Reduce_scatter with ragged / empty per-rank counts and MPI_IN_PLACE
    (reduce_scatter_intra_recursive_halving.c:38-262 / _pairwise.c:42-115)
    over the staged transport, every algorithm"""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mpich_amd import coll
    counts = [0 if q == 1 else (q * 37 + 11) % 5 * 1000 + q for q in range(world)]
    total = sum(counts)
    send = np.random.default_rng(0x5EED0D00 + rank).uniform(-1, 1, total).astype(np.float32)
    np.save(os.path.join(outdir, 'rg_send%d.npy' % rank), send)
    for algo in ('recursive_halving', 'pairwise', 'pairwise_pipelined', 'pull'):
        for in_place in (False, True):
            ds = torch.from_numpy(send.copy()).cuda()
            if in_place:
                coll.reduce_scatter(None, ds, counts, MPI_FLOAT, MPI_SUM, algorithm=algo)
                out = ds[:counts[rank]]
            else:
                out = torch.empty(max(counts[rank], 1), dtype=torch.float32, device='cuda')
                coll.reduce_scatter(ds, out, counts, MPI_FLOAT, MPI_SUM, algorithm=algo)
                out = out[:counts[rank]]
            np.save(os.path.join(outdir, 'rg_%s_%d_%d.npy' % (algo, in_place, rank)),
                    out.cpu().numpy())
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [3, 5])
def test_staged_reduce_scatter_ragged_in_place(oracle, tmp_path, world):
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_ragged_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    counts = [0 if q == 1 else (q * 37 + 11) % 5 * 1000 + q for q in range(world)]
    raw = [np.load(tmp_path / ('rg_send%d.npy' % r)).view(np.uint8) for r in range(world)]
    exp_rh = oracle.rs_schedule(raw, counts, MPI_FLOAT, MPI_SUM, 'recursive_halving')
    exp_pw = oracle.rs_schedule(raw, counts, MPI_FLOAT, MPI_SUM, 'pairwise')
    for algo in ('recursive_halving', 'pairwise', 'pairwise_pipelined', 'pull'):
        exp = exp_rh if algo == 'recursive_halving' else exp_pw
        for in_place in (0, 1):
            for r in range(world):
                got = np.load(tmp_path / ('rg_%s_%d_%d.npy' % (algo, in_place, r)))
                assert got.tobytes() == exp[r].tobytes(), (algo, in_place, r)


def _config4_worker(rank, world, port, outdir, total_bytes):
    """BASELINE config 4's vector size on the staged transport: 2 ranks, a
    4 GiB fp32 vector each, recursive halving + HIP combine; each rank checks
    its 2 GiB block on the device, bit for bit, against the schedule's one
    IEEE add per element (P = 2: inout = own + partner's) computed by torch
    from the partner's regenerated input, and an MPI_INT run against the
    redscatblk3.c closed form at the same size"""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mpich_amd import coll
    n = total_bytes // 4
    rc = n // world

    def vec(r):
        g = torch.Generator(device='cuda')
        g.manual_seed(0x5EED0C40 + r)
        return torch.empty(n, dtype=torch.float32, device='cuda').uniform_(-1, 1, generator=g)
    x = vec(rank)
    out = torch.empty(rc, dtype=torch.float32, device='cuda')
    coll.reduce_scatter_block(x, out, rc, MPI_FLOAT, MPI_SUM, algorithm='recursive_halving')
    del x
    torch.cuda.empty_cache()
    mine = vec(rank)[rank * rc:(rank + 1) * rc].clone()
    other = vec(1 - rank)[rank * rc:(rank + 1) * rc].clone()
    torch.cuda.empty_cache()
    ok_f = bool(torch.equal((mine + other).view(torch.int32), out.view(torch.int32)))
    del mine, other, out
    torch.cuda.empty_cache()
    xi = torch.cat([torch.full((rc,), rank + b, dtype=torch.int32, device='cuda')
                    for b in range(world)])
    oi = torch.empty(rc, dtype=torch.int32, device='cuda')
    coll.reduce_scatter_block(xi, oi, rc, 0x4c000405, MPI_SUM, algorithm='recursive_halving')
    want = world * rank + world * (world - 1) // 2
    bad = (oi != want).nonzero()
    ok_i = bad.numel() == 0
    with open(os.path.join(outdir, 'ok%d.txt' % rank), 'w') as f:
        f.write('%d %d' % (ok_f, ok_i))
    if not ok_i:
        with open(os.path.join(outdir, 'bad%d.txt' % rank), 'w') as f:
            f.write('%d bad of %d, first %s, last %s, values %s' % (
                bad.numel(), rc, bad[:3].flatten().tolist(), bad[-3:].flatten().tolist(),
                torch.unique(oi[bad.flatten()[:1000000]]).tolist()[:10]))
    del xi, oi
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


def test_staged_rsb_config4_full_size(tmp_path):
    """recursive halving at the 4 GiB-per-rank vector of BASELINE configs[3]
    (two ranks on the test GPU), fp32 bit-exact and MPI_INT closed form"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_config4_worker, args=(2, _free_port(), str(tmp_path), 4 << 30), nprocs=2,
             join=True)
    for r in range(2):
        got = open(tmp_path / ('ok%d.txt' % r)).read()
        detail = open(tmp_path / ('bad%d.txt' % r)).read() if got != '1 1' else ''
        assert got == '1 1', (r, detail)


def _c4_shape_worker(rank, world, port, outdir, total_bytes):
    """The exact shape of the N > 1 value leg (bench.multi_gpu at the default
    --rsb-bytes), ranks as processes on the test GPU: a 4 GiB fp32 vector per
    rank, recursive halving with the combine overlap at the RCCL default
    (half-steps >= 1 MiB split, kept half on the second stream) and off, and
    every message above 1 GiB split into consecutive 1 GiB messages (the
    RCCL communicators' maximum) -- the step-1 send of 2 GiB goes as two.
    Each rank checks its 512 MiB (P = 8) block bit for bit on the device
    against the schedule's association (bench.rh_expected_block: per step with
    mask = P/2 .. 1 every rank adds its partner's partial, one IEEE add each)
    over inputs regenerated from the seeds."""
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['MPIX_COLL_TRACE'] = '1'
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    trace = open(os.path.join(outdir, 'c4trace%d.txt' % rank), 'w')
    os.dup2(trace.fileno(), 2)          # the library's trace lines land in the file
    from mpich_amd import coll
    n = total_bytes // 4
    rc = n // world

    def vec(r):
        g = torch.Generator(device='cuda')
        g.manual_seed(0x5EED0C80 + r)
        return torch.empty(n, dtype=torch.float32, device='cuda').uniform_(-1, 1, generator=g)
    # the expected block: block `rank` of every rank's vector, folded as the
    # schedule folds it (parts[q] = parts[q] + parts[q ^ m]; an IEEE add is
    # commutative, so both members of a pair share one sum tensor)
    parts = []
    for q in range(world):
        v = vec(q)
        parts.append(v[rank * rc:(rank + 1) * rc].clone())
        del v
    m = world // 2
    while m:
        for q in range(world):
            if q < q ^ m:
                t = parts[q] + parts[q ^ m]
                parts[q] = parts[q ^ m] = t
        m //= 2
    expected = parts[rank]
    del parts, t
    torch.cuda.empty_cache()
    c = coll.comm_for(None, True)
    x = vec(rank)
    out = torch.empty(rc, dtype=torch.float32, device='cuda')
    res = {}
    for mode in (1 << 20, 0):
        c.set_rh_overlap(mode)
        out.fill_(float('nan'))
        timer = []
        coll.reduce_scatter_block(x, out, rc, MPI_FLOAT, MPI_SUM, algorithm='recursive_halving',
                                  timer=timer)
        torch.cuda.synchronize()
        phases = [t['phase'] for t in timer]
        res[str(mode)] = dict(bits=bool(torch.equal(out.view(torch.int32),
                                                     expected.view(torch.int32))),
                              split=phases.count('combine (sent half)'),
                              whole=phases.count('combine'),
                              state=c.state()['last_rs'])
    trace.flush()
    with open(os.path.join(outdir, 'c4res%d.json' % rank), 'w') as f:
        import json
        json.dump(res, f)
    del x, out, expected
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('world', [4, 8])
def test_staged_rsb_config4_value_leg_shape(tmp_path, world):
    """P = 4 and 8 at 4 GiB fp32 per rank, overlap at the
    RCCL default and off, 1 GiB message split -- bit-exact on every rank"""
    import json
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_c4_shape_worker, args=(world, _free_port(), str(tmp_path), 4 << 30), nprocs=world,
             join=True)
    steps = world.bit_length() - 1
    for r in range(world):
        res = json.load(open(tmp_path / ('c4res%d.json' % r)))
        on, off = res[str(1 << 20)], res['0']
        assert on['bits'] and off['bits'], (r, res)
        assert on['state'] == off['state'] == 'recursive_halving', res
        # overlap on: every step but the last (no next split) cuts its combine
        assert on['split'] == steps - 1 and on['whole'] == 1, (r, on)
        assert off['split'] == 0 and off['whole'] == steps, (r, off)
        import re
        lines = [ln for ln in open(tmp_path / ('c4trace%d.txt' % r)).read().splitlines()
                 if ln.startswith('[mpix_coll rank') and len(ln.split()) > 3 and
                 all(re.fullmatch(r'[<>]\d+:\d+', f) for f in ln.split()[3:])]
        # step 1 of each call: 2 GiB each way, posted as two 1 GiB messages each
        first = lines[0].split()[3:]
        assert len(first) == 4 and all(f.endswith(':%d' % (1 << 30)) for f in first), lines[0]
        assert max(int(f.split(':')[1]) for ln in lines for f in ln.split()[3:]) == 1 << 30


def test_rccl_rsb_matches_oracle(oracle, tmp_path):
    """one process per GPU over RCCL (the bench's transport at N > 1)"""
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if ndev < 2:
        pytest.skip('RCCL across processes needs >= 2 GPUs (this box has %d); RCCL refuses two '
                    'ranks on one device (profiles/r01_rccl_probe.txt)' % ndev)
    world = min(ndev, 8)
    cases = [('%s_%s' % (a, k), a, k, 100003 if k == 'float' else 50021)
             for a in ALGOS for k in ('float', 'pair')]
    cases.append(('ar', 'allreduce', 'float', 25013))
    cases.append(('ar_mp', 'allreduce_mp', 'float', 25013))
    cases.append(('ar_pull', 'allreduce_pull', 'float', 25013))
    _run(oracle, tmp_path, world, 'nccl', cases)


def _streams_worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mpich_amd import ccl, coll
    MPI_INT = 0x4c000405
    c = coll.comm_for(None, True)
    n = 30011
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ins, outs = [], []
    for it in range(6):
        # block i of rank r holds r + i + 10 * it (redscatblk3.c:43-48)
        ins.append(torch.cat([torch.full((n,), rank + i + 10 * it, dtype=torch.int32, device='cuda')
                              for i in range(world)]))
        outs.append(torch.empty(n, dtype=torch.int32, device='cuda'))
    torch.cuda.synchronize()
    for it in range(6):         # async pulls alternating between two streams, no host sync
        algo = ('pull', 'recursive_halving_pull')[it % 2]
        st = streams[it % 2]
        rc = ccl.reduce_scatter_block(ins[it], outs[it], n, MPI_INT, MPI_SUM, c, algo, stream=st,
                                      blocking=False)
        assert rc == 0, rc
    torch.cuda.synchronize()
    bad = [it for it in range(6)
           if not bool(torch.all(outs[it] == world * rank + world * (world - 1) // 2 + world * 10 * it))]
    with open(os.path.join(outdir, 'streams%d.txt' % rank), 'w') as f:
        f.write(' '.join(map(str, bad)))
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_staged_async_pulls_on_two_streams(tmp_path, world):
    """the pull window is shared by every call on the communicator: async
    pulls issued back to back on alternating streams (each call ordered
    behind the previous user of the window) all give the closed form"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_streams_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert open(tmp_path / ('streams%d.txt' % r)).read() == '', r


def _growth_worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['MPIX_COLL_TRACE'] = '1'
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    trace = open(os.path.join(outdir, 'gtrace%d.txt' % rank), 'w')
    os.dup2(trace.fileno(), 2)          # the library's trace lines land in the file
    from mpich_amd import coll
    MPI_INT = 0x4c000405
    bad = []
    # the bench's order: a small window first, then growth to a large one
    for it, (algo, n) in enumerate((('recursive_halving_pull', 4099), ('recursive_halving_pull', 1 << 22),
                                    ('pull', 1 << 22), ('pull', 1 << 23))):
        blk = torch.cat([torch.full((n,), rank + i + it, dtype=torch.int32, device='cuda')
                         for i in range(world)])
        o = torch.empty(n, dtype=torch.int32, device='cuda')
        torch.cuda.synchronize()
        coll.reduce_scatter_block(blk, o, n, MPI_INT, MPI_SUM, algorithm=algo)
        torch.cuda.synchronize()
        if not bool(torch.all(o == world * rank + world * (world - 1) // 2 + world * it)):
            bad.append('%s@%d' % (algo, n))
        del blk, o
        torch.cuda.empty_cache()
    with open(os.path.join(outdir, 'growth%d.txt' % rank), 'w') as f:
        f.write(' '.join(bad))
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_staged_pull_windows_grow_and_verify(tmp_path, world):
    """the pull window starts small and grows twice with the message (to
    world x 16 MiB, then world x 32 MiB per rank) and every window verifies
    -- exported one rank at a time, a retry allowed -- so the pulls really
    run instead of falling back (which would give the same bits, hiding a
    broken window path)"""
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    mp.spawn(_growth_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert open(tmp_path / ('growth%d.txt' % r)).read() == '', r
        lines = open(tmp_path / ('gtrace%d.txt' % r)).read().splitlines()
        assert not any('given up' in ln for ln in lines), lines
        sizes = [ln for ln in lines if 'pull window' in ln and 'all 1' in ln]
        assert len(sizes) == 3, lines       # the first window, then two growths
