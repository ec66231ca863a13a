"""bench.py's N > 1 path end to end on one GPU: `bench.py --gpus 2` starts
its two ranks itself (no torchrun), both on device 0 over the gloo staged
transport (the rehearsal knobs; RCCL refuses two ranks on one device), runs
the recursive-halving reduce-scatter value leg with its bit-exact parity gate,
and rank 0's one line carries n_gpus = 2, the schedule that ran and the
defaults A/B; then the same under torch.distributed.run, the driver's own N > 1
form."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_gpus_2_self_launched_line():
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(MPIX_BENCH_SAME_DEVICE='1', MPIX_BENCH_BACKEND='gloo')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--steps', '2', '--warmup', '1', '--count', str(1 << 22),
                        '--rsb-bytes', str(16 << 20), '--no-extras'],
                       cwd=ROOT, capture_output=True, text=True, timeout=100, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['schedule_ran'] == 'recursive_halving', d
    assert d['parity']['bit_exact_all_ranks'] and d['value'] > 0, d
    # the timed result itself, at the timed size, on every rank
    assert d['parity']['full_size_bit_exact_all_ranks'], d['parity']
    assert d['parity']['full_size_recvcount'] == (16 << 20) // 4 // 2, d['parity']
    # the overlap x store-policy defaults
    # timed beside the shipped one, every variant first bit-exact on every
    # rank against the association (not against the default's own output)
    ab = d['defaults_ab']
    for k in ('overlap_on_policy_on', 'overlap_off_policy_on', 'overlap_on_policy_off',
              'overlap_off_policy_off'):
        assert ab[k]['bit_exact_vs_association_all_ranks'] and ab[k]['ms_per_step'] > 0, ab
    # the reference schedule's host work as the baseline
    c = d['cpu_baseline']
    assert c['kind'] == 'port' and c['cores'] == 2 and c['value'] > 0, c


@pytest.mark.gpu
def test_bench_full_size_check_catches_a_flipped_bit():
    """the full-size check is live: one bit flipped in rank 1's timed result
    (MPIX_BENCH_FAULT_RANK, a test hook) fails the run with EXIT_PARITY and a
    top-level error naming the timed size"""
    sys.path.insert(0, ROOT)
    import bench
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(MPIX_BENCH_SAME_DEVICE='1', MPIX_BENCH_BACKEND='gloo', MPIX_BENCH_FAULT_RANK='1')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2',
                        '--steps', '2', '--warmup', '1', '--count', str(1 << 22),
                        '--rsb-bytes', str(16 << 20), '--no-extras', '--no-cpu-baseline',
                        '--no-ab'], cwd=ROOT, capture_output=True, text=True, timeout=100, env=env)
    assert p.returncode == bench.EXIT_PARITY, (p.returncode, p.stderr[-3000:])
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{')][0])
    assert d['value'] is None and 'timed size' in d['error'], d


@pytest.mark.gpu
def test_bench_gpus_2_under_torchrun_line():
    """the same line in the driver's own N > 1 form, `python -m
    torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
    --master-port P bench.py --gpus 2 ...`: the ranks run as the launcher gives
    them (WORLD_SIZE set, no self-launch) and rank 0's one line is the N-rank
    line"""
    sys.path.insert(0, ROOT)
    import bench
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT', 'MASTER_ADDR')}
    env.update(MPIX_BENCH_SAME_DEVICE='1', MPIX_BENCH_BACKEND='gloo')
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
                        '--nproc-per-node', '2', '--master-addr', '127.0.0.1',
                        '--master-port', str(bench.free_port()), os.path.join(ROOT, 'bench.py'),
                        '--gpus', '2', '--steps', '2', '--warmup', '1', '--count', str(1 << 22),
                        '--rsb-bytes', str(16 << 20), '--no-extras', '--no-cpu-baseline'],
                       cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['launcher'] == 'external', d
    assert d['schedule_ran'] == 'recursive_halving' and d['parity']['bit_exact_all_ranks'], d
    for k in ('overlap_on_policy_on', 'overlap_off_policy_on', 'overlap_on_policy_off',
              'overlap_off_policy_off'):
        assert d['defaults_ab'][k]['bit_exact_vs_association_all_ranks'], d['defaults_ab']
    assert d['parity']['full_size_bit_exact_all_ranks'], d['parity']
