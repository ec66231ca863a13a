"""Where the time of a host-resident (pageable) MPIX_Reduce_local goes, per
size, and how much it varies from call to call and from box to box
(the 256 MiB pageable call took 17.05 ms in the driver's
bench against 11.8-12.5 ms in every builder profile).

Per size (4 MiB .. 1 GiB per operand, fp32 SUM, fresh numpy operands touched
before timing): `reps` synchronous calls timed one by one, the oracle's one-
core loop on the same operands timed the same way, a one-thread host copy of
the operand (the host-memory rate at that moment), the cgroup's cpu.stat
throttling counters across the calls, and for the wave form the per-step
trace (MPIX_REDOP_PIPE_TRACE: copy-in / kernel wait / copy-out / barrier per
worker, and the CPU each worker ran on).  The NUMA node of the operands'
pages and of the GPU are recorded once.  One JSON line per size to stdout.

usage (GPU box): python3 tools/pageable_swing.py [--reps 12] [--chunk MiB]
    [--threads N] [--label text]
env MPIX_REDOP_PAGEABLE_AFFINITY=gpu pins the workers to the GPU's node.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ['MPIX_REDOP_PIPE_TRACE'] = '1'

import torch  # noqa: E402

from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def cpu_stat():
    out = {}
    try:
        for line in open('/sys/fs/cgroup/cpu.stat'):
            k, v = line.split()
            out[k] = int(v)
    except OSError:
        pass
    return out


def pages_node(arr, samples=64):
    """NUMA nodes of `samples` pages spread over arr (move_pages, query only)"""
    libc = ctypes.CDLL(None, use_errno=True)
    page = 4096
    base = arr.ctypes.data & ~(page - 1)
    span = arr.nbytes
    addrs = [(base + (span * i // samples)) & ~(page - 1) for i in range(samples)]
    pv = (ctypes.c_void_p * samples)(*addrs)
    st = (ctypes.c_int * samples)()
    SYS_move_pages = 279
    rc = libc.syscall(SYS_move_pages, 0, samples, pv, None, st, 0)
    if rc != 0:
        return None
    nodes = {}
    for s in st:
        nodes[s] = nodes.get(s, 0) + 1
    return nodes


def gpu_node():
    """the GPU's NUMA node from sysfs (its PCI function's numa_node)"""
    try:
        pr = torch.cuda.get_device_properties(0)
        bdf = '%04x:%02x:%02x.0' % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
    except Exception:
        return None, None
    try:
        return int(open('/sys/bus/pci/devices/%s/numa_node' % bdf).read()), bdf
    except OSError:
        return None, bdf


def traced(fn):
    """run fn() with fd 2 going to a temp file; return (fn's value, the
    wave_trace dicts it printed)"""
    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile(mode='w+') as f:
        os.dup2(f.fileno(), 2)
        try:
            v = fn()
        finally:
            os.dup2(saved, 2)
            os.close(saved)
        f.seek(0)
        traces = []
        for line in f:
            if line.startswith('{"wave_trace"'):
                traces.append(json.loads(line)['wave_trace'])
    return v, traces


def summarize_trace(t):
    W = t['W']
    ns = np.array(t['ns'], dtype=np.int64).reshape(-1, W, 5)
    steps = ns.shape[0]
    rows = []
    prev = 0
    for s in range(steps):
        bar = ns[s, :, 4].max()
        cin = ns[s, :, 1]
        wt = ns[s, :, 2]
        cout = ns[s, :, 3]
        rows.append(dict(step=s, ms=round((bar - prev) / 1e6, 3),
                         copyin_max_ms=round((cin.max() - prev) / 1e6, 3) if (cin >= 0).all() else None,
                         wait_max_ms=round((wt.max() - prev) / 1e6, 3) if (wt >= 0).all() else None,
                         copyout_max_ms=round((cout.max() - prev) / 1e6, 3) if (cout >= 0).all() else None))
        prev = bar
    return dict(chunks_MiB=[round(c * t['ext'] / 2 ** 20, 2) for c in t['chunks']], cpus=t['cpus'],
                total_ms=round(prev / 1e6, 3), steps=rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=12)
    ap.add_argument('--sizes', default='4,16,64,256,1024', help='MiB per operand')
    ap.add_argument('--chunk', type=int, default=0, help='pageable chunk MiB (0: library default)')
    ap.add_argument('--threads', type=int, default=-1)
    ap.add_argument('--label', default='')
    a = ap.parse_args()
    assert redop.lib().MPIX_Redop_init() == 0
    orc.build()
    pg = redop.get_pageable()
    if a.chunk or a.threads >= 0:
        redop.check(redop.set_pageable(pg['threads'] if a.threads < 0 else a.threads,
                                       (a.chunk << 20) if a.chunk else pg['chunk_bytes']))
    pg = redop.get_pageable()
    fn_gpu = redop.lib().MPIX_Reduce_local
    fn_cpu = orc.lib().oracle_reduce_local
    node, bus = gpu_node()
    head = dict(label=a.label, gpu_numa_node=node, gpu_bus=bus, pageable=pg,
                affinity_env=os.environ.get('MPIX_REDOP_PAGEABLE_AFFINITY', 'none'),
                sched_affinity_cpus=len(os.sched_getaffinity(0)), cpu_stat=cpu_stat())
    print(json.dumps(dict(header=head)), flush=True)
    for mib in [int(x) for x in a.sizes.split(',')]:
        n = (mib << 20) // 4
        rng = np.random.default_rng(0x5EED0009)
        x = rng.uniform(-1, 1, n).astype(np.float32)
        y = rng.uniform(-1, 1, n).astype(np.float32)
        t0 = time.perf_counter()
        z = x.copy()
        host_copy_gbs = x.nbytes * 2 / (time.perf_counter() - t0) / 1e9    # read + write
        del z
        nodes = dict(in_pages=pages_node(x), inout_pages=pages_node(y))
        st0 = cpu_stat()
        # warm-up (the pinned ring is allocated at the first wave call)
        redop.check(fn_gpu(ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(y.ctypes.data), n,
                           H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM)))

        def run_gpu():
            ts = []
            for _ in range(a.reps):
                t = time.perf_counter()
                rc = fn_gpu(ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(y.ctypes.data), n,
                            H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM))
                ts.append(time.perf_counter() - t)
                redop.check(rc)
            return ts
        ts, traces = traced(run_gpu)
        st1 = cpu_stat()
        tc = []
        for _ in range(max(3, a.reps // 2)):
            t = time.perf_counter()
            fn_cpu(ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(y.ctypes.data), n,
                   H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM))
            tc.append(time.perf_counter() - t)
        ms = sorted(1e3 * t for t in ts)
        cms = sorted(1e3 * t for t in tc)
        row = dict(mib=mib, gpu_ms=[round(v, 3) for v in (1e3 * t for t in ts)],
                   gpu_min_ms=round(ms[0], 3), gpu_median_ms=round(ms[len(ms) // 2], 3),
                   gpu_max_ms=round(ms[-1], 3), cpu_1core_min_ms=round(cms[0], 3),
                   cpu_1core_median_ms=round(cms[len(cms) // 2], 3),
                   ratio_median=round(ms[len(ms) // 2] / cms[len(cms) // 2], 3),
                   host_copy_GBs=round(host_copy_gbs, 1), numa=nodes,
                   throttled_usec=st1.get('throttled_usec', 0) - st0.get('throttled_usec', 0),
                   nr_throttled=st1.get('nr_throttled', 0) - st0.get('nr_throttled', 0),
                   path='wave' if traces else 'staged/bounce')
        if traces:
            tot = [tr for tr in (summarize_trace(t) for t in traces)]
            slow = max(tot, key=lambda r: r['total_ms'])
            fast = min(tot, key=lambda r: r['total_ms'])
            row['trace_fastest'] = fast
            row['trace_slowest'] = slow
        print(json.dumps(row), flush=True)
        del x, y


if __name__ == '__main__':
    main()
