"""bench.py's own host logic on CPU: the numpy restatement of the
recursive-halving association that gates the N > 1 value (checked here
against the oracle's simulation of reduce_scatter_block_intra_recursive_halving.c),
and the watchdogs: a hung value leg becomes rank 0's error line plus a
non-zero exit status, a hung secondary leg an `extras_error` beside the kept
value (exit 0)."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize('world', [2, 3, 4, 5, 6, 7, 8])
def test_rh_expected_block_matches_oracle(oracle, world):
    import bench
    rc = 1031
    sends = [bench.rsb_inputs_host(r, world, rc) for r in range(world)]
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], rc, 0x4c00040a, 0x58000003)
    for r in range(world):
        assert bench.rh_expected_block(sends, r, rc).tobytes() == exp[r].tobytes(), r


def _run(code):
    return subprocess.run([sys.executable, '-c', textwrap.dedent(code)], cwd=ROOT,
                          capture_output=True, text=True, timeout=60)


def test_value_leg_watchdog_prints_error_and_exits_2():
    p = _run("""
        import time, bench
        e = bench._Emitter(0, {'metric': 'm', 'value': None, 'error': 'value leg did not finish'})
        bench._watchdog(0.3, e, note=False, code=2)
        time.sleep(10)
        """)
    assert p.returncode == 2
    assert '"error": "value leg did not finish"' in p.stdout
    assert 'extras_watchdog' not in p.stdout


def test_extras_watchdog_keeps_headline_and_exits_0():
    """a hung secondary collective: the value leg was checked and timed, so
    the line keeps it, records the hang as extras_error (no top-level
    `error`), and the run still succeeds"""
    p = _run("""
        import time, bench
        e = bench._Emitter(0, {'metric': 'm', 'value': 1.5})
        bench._watchdog(0.3, e)
        time.sleep(10)
        """)
    assert p.returncode == 0
    assert '"value": 1.5' in p.stdout and 'extras_watchdog' in p.stdout
    assert '"extras_error"' in p.stdout and '"error"' not in p.stdout


def test_emitter_prints_once_and_only_on_rank0():
    p = _run("""
        import bench
        e = bench._Emitter(0, {'v': 1})
        e.emit(); e.emit('late')
        bench._Emitter(1, {'v': 2}).emit()
        """)
    assert p.returncode == 0
    assert p.stdout.strip().splitlines() == ['{"v": 1}']


def _threads(comms, fn):
    import threading
    out = [None] * len(comms)
    ts = [threading.Thread(target=lambda r=r: out.__setitem__(r, fn(r, comms[r])))
          for r in range(len(comms))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts), 'a rank hung'
    return out


def test_schedule_ran_reports_fallback(oracle, monkeypatch):
    """a requested schedule that cannot run is reported as
    'fell back to ...' by the bench helper and never timed under its name.
    On host communicators the pulls cannot run (no device memory to map), so
    'pull' runs one-group pairwise and 'recursive_halving_pull' recursive
    halving -- with MPIX_COLL_WINDOW_FAULT set as in the GPU fault test."""
    import bench
    from mpich_amd import ccl
    monkeypatch.setenv('MPIX_COLL_WINDOW_FAULT', '1')
    P, n = 4, 1003
    comms = ccl.comm_create_local(P)
    for c in comms:
        c.set_combine(oracle.combine_fn_address())
    sends = [np.random.default_rng(r).uniform(-1, 1, P * n).astype(np.float32) for r in range(P)]
    recvs = [np.zeros(n, np.float32) for _ in range(P)]
    MPI_FLOAT, MPI_SUM = 0x4c00040a, 0x58000003
    try:
        for algo, ran in (('pull', 'pairwise'), ('recursive_halving_pull', 'recursive_halving'),
                          ('recursive_halving_multipath', 'recursive_halving'),  # P=4 ok on host
                          ('pairwise', 'pairwise')):
            rcs = _threads(comms, lambda r, c: ccl.reduce_scatter_block(
                sends[r], recvs[r], n, MPI_FLOAT, MPI_SUM, c, algo))
            assert rcs == [0] * P
            for c in comms:
                got = bench.schedule_ran(c, algo)
                if algo == 'recursive_halving_multipath':
                    assert got['schedule_ran'] == algo and 'error' not in got, got
                else:
                    assert got['schedule_ran'] == ran, got
                    assert ('error' in got) == (ran != algo), got
                    if ran != algo:
                        assert got['error'] == 'fell back to ' + ran
                assert got['pulls_enabled'] is False
        st = comms[0].state()
        assert st['fallbacks'] == 2 and st['window_retries'] == 0, st
        # allreduce: pull -> reduce_scatter_allgather; multipath on P=3-like
        # shapes (count % P) -> reduce_scatter_allgather
        outs = [np.zeros(P * n, np.float32) for _ in range(P)]
        for algo, count in (('pull', P * n), ('rsag_multipath', P * n - 1),
                            ('rsag_multipath', P * n)):
            rcs = _threads(comms, lambda r, c: ccl.allreduce(sends[r][:count], outs[r][:count],
                                                              count, MPI_FLOAT, MPI_SUM, c, algo))
            assert rcs == [0] * P
            got = bench.schedule_ran(comms[1], algo, 'ar')
            fell = algo == 'pull' or count % P
            assert got['schedule_ran'] == ('reduce_scatter_allgather' if fell else algo), got
            assert ('error' in got) == bool(fell)
    finally:
        for c in comms:
            c.free()


def test_state_before_first_collective():
    from mpich_amd import ccl
    comms = ccl.comm_create_local(2)
    try:
        st = comms[0].state()
        assert st == dict(pulls_enabled=False, last_rs=None, last_allreduce=None,
                          window_retries=0, fallbacks=0), st
    finally:
        for c in comms:
            c.free()


def test_leg_without_symmetric_memory_is_reported_not_fatal():
    """MPIX_Comm_alloc_shared answers MPI_ERR_OTHER on every rank when no
    verified mapping could be made (mpix_coll.h); the bench then reports that
    leg with its reason and no time, and goes on with the others (found by the
    window-fault rehearsal, profiles/r03_rehearsal_n4.json)"""
    import bench
    from mpich_amd import redop
    leg = bench._no_shared(redop.RedopError(15, 'MPIX_Comm_alloc_shared'))
    assert leg['schedule_ran'] is None and 'ms' not in leg
    assert leg['error'].startswith('no symmetric memory') and 'MPIX_Comm_alloc_shared' in leg['error']


# ------------------------------------------------------- the rank launcher
# `python3 bench.py --gpus N` must yield the
# N-rank line by itself (no torchrun), and never a 1-GPU line for N > 1.

def _bench(args, env_extra=None, drop=('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, cwd=ROOT,
                          capture_output=True, text=True, timeout=120, env=env)


@pytest.mark.parametrize('n', [2, 3])
def test_gpus_n_launches_n_ranks_itself(n):
    import json
    p = _bench(['--gpus', str(n), '--dry-run', '--no-extras', '--no-cpu-baseline'])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == n and d['ranks_seen'] == n and d['launcher'] == 'bench.py', d


def _torchrun(nproc, args, env_extra=None):
    """the driver's N-rank form: python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py ..."""
    import bench
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT', 'MASTER_ADDR')}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                           '--nproc-per-node', str(nproc), '--master-addr', '127.0.0.1',
                           '--master-port', str(bench.free_port()), os.path.join(ROOT, 'bench.py')]
                          + args, cwd=ROOT, capture_output=True, text=True, timeout=180, env=env)


@pytest.mark.parametrize('n', [1, 2])
def test_dry_run_under_torchrun_is_one_n_rank_line(n):
    """under the driver's launcher (WORLD_SIZE set by torchrun) every rank runs
    as given, and only rank 0 prints: one line with n_gpus = N"""
    import json
    p = _torchrun(n, ['--gpus', str(n), '--dry-run', '--no-extras', '--no-cpu-baseline'])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == n, d
    if n > 1:
        assert d['ranks_seen'] == n and d['launcher'] == 'external', d


def test_gpus_1_dry_run_is_single():
    import json
    p = _bench(['--dry-run'])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d['n_gpus'] == 1 and d['launcher'] is None


def test_world_size_and_gpus_disagree_exits_nonzero():
    p = _bench(['--gpus', '4', '--dry-run'], env_extra={'WORLD_SIZE': '2', 'RANK': '0'}, drop=())
    assert p.returncode != 0
    assert 'disagree' in p.stderr and '{' not in p.stdout


def test_too_few_gpus_exits_nonzero_before_any_rank():
    """this container shows no GPU: --gpus 2 without the rehearsal knob must
    refuse, not fall back to one rank"""
    p = _bench(['--gpus', '2', '--no-extras', '--no-cpu-baseline'],
               env_extra={'HIP_VISIBLE_DEVICES': '', 'CUDA_VISIBLE_DEVICES': ''})
    assert p.returncode != 0
    assert 'need 2 GPUs' in p.stderr and '{' not in p.stdout


def test_failing_rank_fails_the_launch():
    """a rank that dies (here every rank does: an unknown process-group
    backend, or no GPU to select in this container) ends the whole launch
    non-zero, with the failed rank named, and the survivors are stopped"""
    p = _bench(['--gpus', '2', '--steps', '1'],
               env_extra={'MPIX_BENCH_SAME_DEVICE': '1', 'MPIX_BENCH_BACKEND': 'nosuchbackend'})
    assert p.returncode != 0
    assert 'exited with status' in p.stderr


def test_world_plan_rules():
    import bench
    a = bench.parse(['--gpus', '8'])
    assert bench.world_plan(a, {}) == ('launch', 8)
    assert bench.world_plan(a, {'WORLD_SIZE': '8'}) == ('rank', 8)
    assert bench.world_plan(bench.parse([]), {}) == ('single', 1)
    assert bench.world_plan(bench.parse([]), {'WORLD_SIZE': '4'}) == ('rank', 4)
    assert bench.world_plan(bench.parse(['--gpus', '1']), {'WORLD_SIZE': '1'}) == ('single', 1)
    with pytest.raises(SystemExit):
        bench.world_plan(a, {'WORLD_SIZE': '2'})
    with pytest.raises(SystemExit):
        bench.world_plan(bench.parse(['--gpus', '0']), {})


def test_multipath_allreduce_small_step_reported_as_plain(oracle):
    """rsag_multipath needs send_cnt >= parts * (parts - 1)
    at a reduce-scatter step; a step below that runs the plain exchange.  A
    call none of whose steps could use the relays is reported as
    reduce_scatter_allgather (count 6: not a multiple of P = 4); a call whose
    first step went over the relays and whose last did not (count 4: 2 then 1
    element per step) ran multipath and is reported so; count 8 keeps 2 per
    step"""
    import bench
    from mpich_amd import ccl
    P = 4
    comms = ccl.comm_create_local(P)
    for c in comms:
        c.set_combine(oracle.combine_fn_address())
    MPI_FLOAT, MPI_SUM = 0x4c00040a, 0x58000003
    try:
        for count, fell in ((6, True), (4, False), (8, False), (4096, False)):
            sends = [np.arange(count, dtype=np.float32) + r for r in range(P)]
            outs = [np.zeros(count, np.float32) for _ in range(P)]
            before = comms[0].state()['fallbacks']
            rcs = _threads(comms, lambda r, c: ccl.allreduce(sends[r], outs[r], count, MPI_FLOAT,
                                                              MPI_SUM, c, 'rsag_multipath'))
            assert rcs == [0] * P
            want = sum(sends)
            for r in range(P):
                assert np.array_equal(outs[r], want), (count, r)
                got = bench.schedule_ran(comms[r], 'rsag_multipath', 'ar')
                assert ('error' in got) == fell, (count, got)
                assert got['schedule_ran'] == ('reduce_scatter_allgather' if fell
                                               else 'rsag_multipath'), (count, got)
            assert comms[0].state()['fallbacks'] - before == (1 if fell else 0)
    finally:
        for c in comms:
            c.free()


def test_overlap_note_names_what_ran():
    """the N > 1 line says whether the recursive-halving combine overlap ran
    in its timed calls (the communicator's MPIX_Comm_get_rh_overlap)"""
    import bench
    assert bench.overlap_note(1 << 20).startswith('each step')
    assert '1048576 B' in bench.overlap_note(1 << 20)
    assert bench.overlap_note(0).startswith('off')


def test_rh_overlap_setting_per_communicator(monkeypatch):
    """the overlap threshold is read once, when a communicator is
    created (env MPIX_COLL_RH_OVERLAP), and set per communicator afterwards --
    never re-read from the environment mid-call"""
    from mpich_amd import ccl, redop
    monkeypatch.delenv('MPIX_COLL_RH_OVERLAP', raising=False)
    comms = ccl.comm_create_local(2)
    try:
        assert comms[0].rh_overlap() == 0           # local communicators: off by default
        monkeypatch.setenv('MPIX_COLL_RH_OVERLAP', '4096')
        assert comms[0].rh_overlap() == 0           # not re-read after creation
        comms[0].set_rh_overlap(1 << 20)
        assert comms[0].rh_overlap() == 1 << 20 and comms[1].rh_overlap() == 0
        comms[0].set_rh_overlap(-1)                 # the creation-time value
        assert comms[0].rh_overlap() == 0
        with pytest.raises(redop.RedopError):
            comms[0].set_rh_overlap(-2)
    finally:
        for c in comms:
            c.free()
    comms = ccl.comm_create_local(2)                # created with the env set
    try:
        assert [c.rh_overlap() for c in comms] == [4096, 4096]
        # -1 restores what the communicator was created with (the
        # env's 4096 here), not the kind's compiled default
        comms[0].set_rh_overlap(0)
        comms[0].set_rh_overlap(-1)
        assert comms[0].rh_overlap() == 4096
    finally:
        for c in comms:
            c.free()


def test_dry_run_line_names_the_defaults_ab():
    """the N > 1 line carries `defaults_ab`, the four
    overlap x store-policy variants of the value leg"""
    import json
    import bench
    p = _bench(['--gpus', '2', '--dry-run', '--no-extras', '--no-cpu-baseline'])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{')][0])
    assert sorted(d['defaults_ab']) == sorted(bench.AB_VARIANTS), d


def test_launcher_counts_devices_in_a_child(monkeypatch):
    """the launcher's device count runs in a child process (count_devices):
    here (no GPU) it is 0, and the parent never imports the HIP runtime's
    device state for it"""
    import bench
    import torch
    assert bench.count_devices() == 0
    assert not torch.cuda.is_initialized()
    with pytest.raises(SystemExit):
        bench.check_devices(2, {})
    bench.check_devices(4, {'MPIX_BENCH_SAME_DEVICE': '1'})


# ------------------------------------------------- round 6
@pytest.mark.parametrize('world', [2, 3, 4, 8])
def test_rh_expected_block_device_matches_numpy_restatement(world):
    """the full-size check's expected block (built with torch, on the device
    in the bench; here on the CPU, same generator calls) equals the numpy
    restatement the parity gate uses, itself pinned to the oracle above"""
    import torch
    import bench
    rc = 1031
    sends = []
    for r in range(world):
        v = torch.empty(world * rc, dtype=torch.float32)
        bench.fill_uniform(v, 0x5EED0100 + r)
        sends.append(v.numpy().copy())
    own = torch.from_numpy(sends[1].copy())
    for r in range(world):
        got = bench.rh_expected_block_device(world, r, rc, 0x5EED0100, 'cpu',
                                             own=own if r == 1 else None)
        assert got.numpy().tobytes() == bench.rh_expected_block(sends, r, rc).tobytes(), r


def test_secondary_parity_failure_fails_the_run():
    """a secondary leg whose closed form / bit check fails sets
    the top-level error and exits EXIT_PARITY; an ordinary exception in an
    extra keeps the value (exit 0); later legs do not run after a failure"""
    import bench
    ran = []

    def ok(part):
        ran.append('ok')
        part['ms'] = 1.0

    def bad_bits(part):
        raise bench.ParityError('pairwise RSB differs from the oracle')

    def boom(part):
        raise RuntimeError('timed out')

    r = {'value': 1.0}
    failed, code = bench.run_secondary(r, [('a', ok), ('b', bad_bits), ('c', ok)])
    assert code == bench.EXIT_PARITY != 0 and 'parity' in r['error'] and 'b' in failed
    assert ran == ['ok'] and 'c' not in r and r['value'] == 1.0
    r = {'value': 1.0}
    failed, code = bench.run_secondary(r, [('a', boom), ('b', ok)])
    assert code == 0 and 'error' not in r and r['extras_error'].startswith('a:')
    r = {'value': 1.0}
    assert bench.run_secondary(r, [('a', ok), ('b', ok)]) == (None, 0)
    assert 'extras_error' not in r


@pytest.mark.parametrize('launch', ['bench', 'torchrun'])
def test_dry_run_line_carries_the_rsb_cpu_baseline(launch):
    """the N > 1 line carries a cpu_baseline -- MPICH's
    recursive-halving host work (copy in, log2(P) combines through the oracle
    loop, copy out) on one pinned core per rank, max over ranks"""
    import json
    args = ['--gpus', '2', '--dry-run', '--no-extras', '--rsb-bytes', str(16 << 20)]
    p = _bench(args) if launch == 'bench' else _torchrun(2, args)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{')][0])
    c = d['cpu_baseline']
    assert c['kind'] == 'port' and c['unit'] == 'GB/s' and c['cores'] == 2, c
    assert c['value'] > 0 and c['ms_per_call'] > 0 and c['combine_ms'] > 0, c
    assert c['combined_elements_per_rank'] == (16 << 20) // 4 // 2, c     # P = 2: half the vector
    assert 'full_size_bit_exact_all_ranks' in d['parity'], d


@pytest.mark.parametrize('P', [2, 3, 4, 5, 8])
def test_rsb_host_work_combines_what_the_schedule_combines(oracle, P):
    """oracle_bench_rsb_rank runs the reference's index arithmetic: a rank of a
    power-of-two world combines (P-1)/P of the vector; with rem = P - pof2
    the odd ranks below 2 rem also fold the whole vector first and the even
    ones combine nothing"""
    from oracle import oracle as orc
    rc = 4096
    pof2 = 1
    while pof2 * 2 <= P:
        pof2 *= 2
    rem = P - pof2
    for r in range(P):
        got = orc.bench_rsb_rank(rc, P, r, -1, 1, 0x4c00040a, 0x58000003)['combined_elements']
        if r < 2 * rem and r % 2 == 0:
            want = 0
        else:
            nr = r // 2 if r < 2 * rem else r - rem
            cnts = [2 * rc if (i * 2 + 1 if i < rem else i + rem) < 2 * rem else rc
                    for i in range(pof2)]
            want = P * rc if r < 2 * rem else 0
            lo, hi, m = 0, pof2, pof2 // 2
            while m:            # the half of [lo, hi) that stays with nr
                if nr < (nr ^ m):
                    hi = lo + m
                else:
                    lo = lo + m
                want += sum(cnts[lo:hi])
                m //= 2
        assert got == want, (P, r, got, want)


def test_cpu_baseline_reads_reduce_and_triad_from_the_same_passes(oracle):
    """the host-triad denominator is timed in the same
    passes as the reduce (same threads, slices and quota windows); the line
    carries both the ratio of medians and the median per-pass ratio"""
    import bench
    c = bench.cpu_baseline(1.0, 1 << 22, None)
    for k in ('frac_of_host_triad_1core', 'frac_of_host_triad_1core_per_pass',
              'host_triad_1core_gibs', 'host_triad_timing'):
        assert k in c, k
    assert 0 < c['frac_of_host_triad_1core'] < 3
    # every core where no quota throttles them, else the quota leg instead
    quota, ncores = c['cgroup_cpu_quota'], c['physical_cores']
    if quota is not None and quota < ncores:
        assert 'skipped' in c['allcores'] and c['quota_threads']['threads'] == max(1, int(quota))
    else:
        assert 'frac_of_host_triad_per_pass' in c['allcores']
        assert 0 < c['allcores']['frac_of_host_triad'] < 3
