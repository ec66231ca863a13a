"""bench.py's rank launcher stays off the GPU.

`python bench.py --gpus N` with no WORLD_SIZE starts its N ranks itself with
subprocess; the parent must never initialise HIP (a process that did must not
outlive or exec around the ranks on this pool).  It counts the GPUs in a
child process (bench.count_devices), so the parent's own state shows no HIP
runtime and no /dev/kfd file descriptor -- checked here in a fresh process on
the GPU box, on the real launch branch (no MPIX_BENCH_SAME_DEVICE), with a
positive control that the same check does see an initialised runtime."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, %r)
    import torch
    import bench

    def kfd_fds():
        out = []
        for fd in os.listdir('/proc/self/fd'):
            try:
                if os.readlink('/proc/self/fd/' + fd).startswith('/dev/kfd'):
                    out.append(fd)
            except OSError:
                pass
        return out

    res = {}
    have = bench.count_devices()
    res['count'] = have
    # the launch branch of main(): world_plan, then check_devices in the
    # launcher; one rank more than the node has must stop before any rank
    try:
        bench.main(['--gpus', str(have + 1), '--no-extras', '--no-cpu-baseline'])
        res['refused'] = False
    except SystemExit as e:
        res['refused'] = 'need %%d GPUs' %% (have + 1) in str(e)
    bench.check_devices(have)                   # enough GPUs: passes
    res['plan'] = list(bench.world_plan(bench.parse(['--gpus', str(have)]), {}))
    res['initialized_before'] = torch.cuda.is_initialized()
    res['kfd_before'] = kfd_fds()
    torch.cuda.init()                           # positive control
    torch.zeros(1, device='cuda')
    res['initialized_after'] = torch.cuda.is_initialized()
    res['kfd_after'] = len(kfd_fds())
    print(json.dumps(res))
""") % ROOT


def test_launcher_parent_never_initialises_hip():
    env = {k: v for k, v in os.environ.items()
           if k not in ('MPIX_BENCH_SAME_DEVICE', 'WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    p = subprocess.run([sys.executable, '-c', PROBE], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res['count'] >= 1, res
    assert res['refused'] is True, res
    assert res['plan'] == (['launch', res['count']] if res['count'] > 1 else ['single', 1]), res
    assert res['initialized_before'] is False, res
    assert res['kfd_before'] == [], res
    # the check sees a runtime when there is one
    assert res['initialized_after'] is True and res['kfd_after'] >= 1, res
