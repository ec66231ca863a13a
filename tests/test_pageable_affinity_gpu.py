"""Pageable host operands with fewer CPUs than wave workers.

The wave form of the synchronous call (redop_capi.cpp `waved`) splits each
chunk's host copies over W = 8 workers that meet at a barrier every step.  A
rank bound to one or two cores (mpirun --bind-to core) must neither starve the
worker everyone waits for (the barrier spins only briefly, then sleeps on a
futex) nor run eight workers on two cores (W is capped at the CPUs the process
may use).  Run in a child process pinned to 1 and to 2 CPUs: the bits equal
the oracle's and the call takes about what it takes unpinned, not scheduler
slices per step (the times are kept in the assertion message)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, %r)
    ncpu = int(sys.argv[1])
    import numpy as np
    import torch
    from mpich_amd import redop
    from oracle import oracle
    oracle.build()
    MPI_FLOAT, MPI_SUM = 0x4c00040a, 0x58000003
    n = 1 << 27                     # 512 MiB per operand: eight 64 MiB wave chunks
    rng = np.random.default_rng(0x5EED1B00)
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    exp = b.copy()
    assert oracle.reduce_local(a, exp, n, MPI_FLOAT, MPI_SUM, nthreads=1) == 0
    torch.cuda.init()
    assert redop.lib().MPIX_Redop_init() == 0
    # after the runtime's start-up, which resets the calling thread's mask
    if ncpu:
        os.sched_setaffinity(0, sorted(os.sched_getaffinity(0))[:ncpu])
    times = []
    ok = True
    for _ in range(3):
        io = b.copy()
        t0 = time.perf_counter()
        assert redop.MPI_Reduce_local(a, io, n, MPI_FLOAT, MPI_SUM) == 0
        times.append(time.perf_counter() - t0)
        ok = ok and io.tobytes() == exp.tobytes()
    print(json.dumps(dict(ok=ok, ms=[round(1e3 * t, 2) for t in times],
                          cpus=len(os.sched_getaffinity(0)))))
""") % ROOT


def _run(ncpu):
    p = subprocess.run([sys.executable, '-c', CHILD, str(ncpu)], cwd=ROOT, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(600)
def test_wave_workers_on_few_cpus():
    free = _run(0)
    assert free['ok'], free
    seen = {'unpinned': free}
    for ncpu in (1, 2):
        got = seen['cpus%d' % ncpu] = _run(ncpu)
        if os.path.isdir(os.path.join(ROOT, 'gpurun_out')):       # on the GPU box: keep the times
            with open(os.path.join(ROOT, 'gpurun_out', 'pageable_affinity.json'), 'w') as f:
                json.dump(seen, f)
        assert got['ok'] and got['cpus'] == ncpu, got
        # no pathological stall: a 512 MiB call is ~25 ms unpinned and its
        # host copies alone on one core ~150 ms; spinning waiters keeping
        # the last worker off its core would cost scheduler slices per step
        assert min(got['ms']) < 2000, (free, got)
