#!/usr/bin/env python3
"""Benchmark of the MI355X-native local reduction and the reduce-scatter it feeds.

N = 1 (BASELINE.json metric "GiB/s device-resident MPI_Reduce_local (fp32
SUM, 1 GiB) vs HBM roofline", configs[1] at 1 GiB): one step = one
synchronous MPIX_Reduce_local call (the MPIR_Reduce_local drop-in) over
count = 2^28 MPI_FLOAT per operand, both operands resident in HBM before the
timed region; GiB/s = algorithmic bytes 3 * count * 4 (read in, read inout,
write inout) / wall time.  `roofline` is the kernel alone (HIP events on its
stream), `cpu_baseline` the oracle (clean-room C restatement of MPICH's
op_fns.c loop) on a bounded sample of the same workload on this host's cores,
`host_crossover` where the GPU path starts to beat one core on host-resident
operands (the floor of MPIX_Redop_is_supported_buffers).

N > 1 (one rank per GPU, started either by torchrun or -- `bench.py --gpus N`
with no WORLD_SIZE in the environment -- by this script itself as N child
processes, see launch_ranks; BASELINE configs[3] and north_star's
"1/2/4/8-GPU reduce-scatter throughput ... absolute GB/s and fraction of
roofline"): one step = one MPI_Reduce_scatter_block (fp32 SUM, a 4 GiB vector
per rank, recvcount = 2^30 / N) by the reference's recursive-halving schedule
(reduce_scatter_block_intra_recursive_halving.c:38-260) in libmpix_coll's C++
host code over its own RCCL communicator, every received half combined by the
HIP kernel; `value` = bus bandwidth (N-1)/N * 4 GiB / max-over-ranks time
(nccl-tests' reduce-scatter convention, GB/s), checked bit for bit against a
numpy restatement of the schedule's association before timing.  The N
independent 1 GiB local reductions of round 1 are reported as an extra
(`reduce_local_replicas`); the pairwise, pipelined, fused-pull schedules and
the allreduce are secondary figures under a watchdog.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402

METRIC = "GiB/s device-resident MPI_Reduce_local (fp32 SUM, 1 GiB) vs HBM roofline"
METRIC_RSB = ("GB/s MPI_Reduce_scatter_block bus bandwidth (fp32 SUM, 4 GiB vector per rank, "
              "recursive halving over RCCL/xGMI, HIP combine)")
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
XGMI_LINK_GBS = 153.0       # one xGMI link, one direction (task brief: 7 x ~153 GB/s per GPU)
GIB = float(1 << 30)
EXIT_PARITY = 3             # a rank's result failed a bit / closed-form check


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=None,
                   help='ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1); '
                        'N > 1 without a launcher starts the N rank processes itself')
    p.add_argument('--dry-run', action='store_true',
                   help='bootstrap the ranks (gloo) and print the line skeleton without '
                        'touching a GPU: checks the launch path on any host')
    p.add_argument('--steps', type=int, default=50)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--count', type=int, default=1 << 28, help='fp32 elements per operand')
    p.add_argument('--cpu-seconds', type=float, default=20.0,
                   help='bounded CPU-baseline sample duration per leg')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-extras', action='store_true',
                   help='skip triad / end-to-end / crossover / secondary collective figures')
    p.add_argument('--sweep', action='store_true', help='config 2 chunk/size sweep')
    p.add_argument('--rsb-bytes', type=int, default=4 << 30, help='RSB vector bytes per rank')
    p.add_argument('--extras-timeout', type=float, default=300.0,
                   help='watchdog (s) over the N>1 secondary collective figures and teardown')
    p.add_argument('--value-timeout', type=float, default=600.0,
                   help='watchdog (s) over the N>1 value leg (bootstrap, parity check, timed steps)')
    p.add_argument('--no-ab', action='store_true',
                   help='N>1: skip the interleaved A/B of the overlap and store-policy defaults')
    p.add_argument('--ab-reps', type=int, default=3, help='N>1 defaults A/B: calls per variant')
    p.add_argument('--ab-rounds', type=int, default=2, help='N>1 defaults A/B: interleaved passes')
    p.add_argument('--pmc', default=os.path.join(ROOT, 'profiles', 'r06g_pmc_summary.json'),
                   help='PMC traffic summary (from tools/pmc_summary.py) to quote as traffic')
    return p.parse_args(argv)


def bench_lib():
    path = os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so')
    L = ctypes.CDLL(path)
    L.mpix_bench_triad.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p]
    L.mpix_bench_triad_xcd.argtypes = L.mpix_bench_triad.argtypes + [ctypes.c_uint]
    L.mpix_bench_call_latency.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_call_loop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_chunked_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_chunked_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_issue_burst.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_issue_noargs.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.mpix_bench_issue_noargs.restype = ctypes.c_double
    L.mpix_bench_query_us.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_issue_hidden.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_double)]
    return L


def call_floor_parts(B, inb, inout, stream, count=16384, burst=64, rounds=100):
    """where the host time of one stream-ordered MPIX_Reduce_local_async goes
    (64 KiB fp32 SUM), measured in bursts of `burst` calls so issue separates
    from the GPU: the launch with no kernel arguments (HIP's floor), the
    argument upload (an empty one-argument kernel minus that), the library's
    own host work (the reduce call minus the empty kernel)"""
    fa = ctypes.cast(redop.lib().MPIX_Reduce_local_async, ctypes.c_void_p).value
    o = (ctypes.c_double * 10)()
    rc = B.mpix_bench_issue_burst(fa, inb.data_ptr(), inout.data_ptr(), count,
                                  H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM),
                                  stream.cuda_stream, burst, rounds, o)
    if rc:
        raise RuntimeError('issue burst loop failed: MPI error class %d' % rc)
    none = B.mpix_bench_issue_noargs(stream.cuda_stream, burst, rounds)
    if none < 0:
        raise RuntimeError('no-argument issue loop failed')
    q = (ctypes.c_double * 3)()
    rc = B.mpix_bench_query_us(inout.data_ptr(), stream.cuda_stream, 20000, q)
    if rc:
        raise RuntimeError('HIP query loop failed (%d)' % rc)
    hid = (ctypes.c_double * 3)()
    rc = B.mpix_bench_issue_hidden(stream.cuda_stream, burst, rounds, inb.data_ptr(),
                                   inout.data_ptr(), hid)
    if rc:
        raise RuntimeError('hidden-argument issue loop failed (%d)' % rc)
    lib = o[0] - o[2]
    queries = 2 * q[0] + q[1] + q[2]
    return dict(count=count, burst=burst, rounds=rounds,
                launch_noargs_us=round(none, 3),
                argument_upload_us=round(o[2] - none, 3),
                library_host_us=round(lib, 3),
                library_hip_queries_us=dict(pointer_attributes_x2=round(2 * q[0], 3),
                                            stream_device=round(q[1], 3),
                                            last_error=round(q[2], 3)),
                library_own_code_us=round(lib - queries, 3),
                empty_issue_args104_us=round(hid[0], 3),
                empty_issue_args104_hidden_us=round(hid[1], 3),
                empty_issue_two_device_pointers_us=round(hid[2], 3),
                call_issue_us=round(o[0], 3), call_burst_us=round(o[1], 3),
                note='host us per call; launch_noargs + argument_upload + library_host = '
                     'call_issue; library_host = the HIP queries it makes (timed alone, '
                     'warm) + its own code; call_burst includes the drain of each burst')


def c_call_median_us(B, fn_addr, inp, io, n, reps):
    """median host time (us) of a synchronous C reduce function with the
    MPIR_Reduce_local signature, timed in C by libmpix_bench"""
    med, p90 = ctypes.c_double(), ctypes.c_double()
    rc = B.mpix_bench_call_latency(fn_addr, inp, io, n, H.as_c_int(H.MPI_FLOAT),
                                   H.as_c_int(H.MPI_SUM), reps, ctypes.byref(med), ctypes.byref(p90))
    if rc:
        raise RuntimeError('call latency loop failed: MPI error class %d' % rc)
    return med.value


def chunked_async_c(B, inb, inout, n, stream, chunk_bytes):
    """1 GiB (n fp32) combined as back-to-back MPIX_Reduce_local_async calls of
    chunk_bytes each, issued and timed in C by libmpix_bench (the loop a
    pipelined collective runs per arriving chunk, without binding overhead)"""
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local_async, ctypes.c_void_p).value
    out = []
    for ck in chunk_bytes:
        m = ck // 4
        if m > n:
            break
        nch = n // m
        issue, total = ctypes.c_double(), ctypes.c_double()
        rc = B.mpix_bench_chunked_async(fn, inb.data_ptr(), inout.data_ptr(), nch * m, m, 4,
                                        H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM),
                                        stream.cuda_stream, ctypes.byref(issue), ctypes.byref(total))
        if rc:
            raise RuntimeError('chunked async loop failed: MPI error class %d' % rc)
        out.append(dict(chunk_bytes=ck, calls=nch, GiBs=round(3 * nch * ck / total.value / GIB, 1),
                        us_per_call=round(1e6 * total.value / nch, 2),
                        issue_us_per_call=round(1e6 * issue.value / nch, 2)))
    return out


def chunked_batch_c(B, inb, inout, n, stream, chunk_bytes, batch=64):
    """the same chunked loop with the chunks handed over `batch` at a time
    through MPIX_Reduce_local_batch_async (one launch per batch): the per-chunk
    cost of an engine with several chunks ready"""
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local_batch_async, ctypes.c_void_p).value
    out = []
    for ck in chunk_bytes:
        m = ck // 4
        nch = n // m
        issue, total = ctypes.c_double(), ctypes.c_double()
        rc = B.mpix_bench_chunked_batch(fn, inb.data_ptr(), inout.data_ptr(), nch * m, m, 4,
                                        H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM),
                                        stream.cuda_stream, batch, ctypes.byref(issue),
                                        ctypes.byref(total))
        if rc:
            raise RuntimeError('chunked batch loop failed: MPI error class %d' % rc)
        out.append(dict(chunk_bytes=ck, batch=batch, calls=(nch + batch - 1) // batch,
                        GiBs=round(3 * nch * ck / total.value / GIB, 1),
                        us_per_chunk=round(1e6 * total.value / nch, 3),
                        issue_us_per_chunk=round(1e6 * issue.value / nch, 3)))
    return out


def sync_call_latency(B, dev, counts=(1, 4096, 1 << 20), reps=2000):
    """per-call host time of the synchronous MPIX_Reduce_local (fp32 SUM,
    device-resident), timed in C by libmpix_bench (no binding overhead);
    checked: after the warm-up + reps calls on zeros with in = 1, inout = reps+1"""
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local, ctypes.c_void_p).value
    out = []
    for n in counts:
        xin = torch.ones(n, dtype=torch.float32, device=dev)
        xio = torch.zeros(n, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        med, p90 = ctypes.c_double(), ctypes.c_double()
        rc = B.mpix_bench_call_latency(fn, xin.data_ptr(), xio.data_ptr(), n,
                                       H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM), reps,
                                       ctypes.byref(med), ctypes.byref(p90))
        ok = rc == 0 and bool(torch.all(xio == reps + 1))
        if not ok:
            raise RuntimeError('sync call latency check failed at count %d (rc %d)' % (n, rc))
        out.append(dict(count=n, median_us=round(med.value, 2), p90_us=round(p90.value, 2),
                        checked=ok))
    return out


CROSSOVER_BYTES = (4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 8 << 20, 16 << 20,
                   64 << 20, 128 << 20, 256 << 20, 512 << 20, 1 << 30)


def _reps_for(nbytes):
    """calls per crossover point (median): at least 7, so one call that a
    busy host stalls cannot set the median (profiles/r04_pageable_swing.json)"""
    return max(7, min(2000, (256 << 20) // max(nbytes, 1)))


def host_crossover_gpu(B):
    """GPU side of the host-resident crossover: MPIX_Reduce_local on pageable
    (numpy) and page-locked (torch pin_memory) operands of each size, timed
    in C (median us per call)"""
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local, ctypes.c_void_p).value
    out = []
    for nb in CROSSOVER_BYTES:
        n = nb // 4
        rng = np.random.default_rng(0x5EED0009)
        a = rng.uniform(-1, 1, n).astype(np.float32)
        b = rng.uniform(-1, 1, n).astype(np.float32)
        reps = _reps_for(nb)
        pg = c_call_median_us(B, fn, a.ctypes.data, b.ctypes.data, n, reps)
        ta, tb = torch.from_numpy(a).pin_memory(), torch.from_numpy(b).pin_memory()
        pn = c_call_median_us(B, fn, ta.data_ptr(), tb.data_ptr(), n, reps)
        out.append(dict(bytes=nb, gpu_pageable_us=round(pg, 2), gpu_pinned_us=round(pn, 2)))
        del a, b, ta, tb
    return out


def crossover_from(rows, key, tol=1.05):
    """smallest size from which the GPU path is faster than one core, or
    within 5 % of it, at every larger size too (None: the CPU wins at every
    measured size)"""
    best = None
    for r in reversed(rows):
        if r[key] <= tol * r['cpu_1core_us']:
            best = r['bytes']
        else:
            break
    return best


def event_time_per_launch(launch, reps, stream, rounds=3):
    """average duration of one `launch()` measured with HIP events on
    `stream`: one event pair brackets `reps` back-to-back launches (so the
    event-record overhead is amortised and the figure is comparable with the
    per-dispatch durations rocprofv3 reports); `rounds` such batches."""
    per = []
    for _ in range(rounds):
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        for _ in range(reps):
            launch()
        s1.record(stream)
        stream.synchronize()
        per.append(s0.elapsed_time(s1) / reps)
    per.sort()
    return sum(per) / len(per), per[len(per) // 2], per[0]


def fill_uniform(t, seed):
    g = torch.Generator(device=t.device)
    g.manual_seed(seed)
    t.uniform_(-1.0, 1.0, generator=g)


def allreduce_scalar(x, op, dev):
    """max/min of a host scalar over ranks (device tensor for nccl, host for gloo)"""
    on = dev if dist.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor([x], dtype=torch.float64, device=on)
    dist.all_reduce(t, op=op)
    return t.item()


def host_topology():
    """this process's CPUs grouped into physical cores (first SMT sibling of
    each core kept), the sockets they sit on, and the cgroup CPU quota"""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else \
        list(range(os.cpu_count()))
    cores, sockets = {}, set()
    for c in aff:
        base = '/sys/devices/system/cpu/cpu%d/topology/' % c
        try:
            pkg = int(open(base + 'physical_package_id').read())
            core = int(open(base + 'core_id').read())
        except (OSError, ValueError):
            pkg, core = 0, c
        sockets.add(pkg)
        cores.setdefault((pkg, core), c)
    # one thread per physical core, sockets interleaved so a prefix of the
    # list spreads over both sockets' memory controllers
    by_sock = {}
    for (pkg, _), c in sorted(cores.items()):
        by_sock.setdefault(pkg, []).append(c)
    phys = []
    for i in range(max(len(v) for v in by_sock.values())):
        for pkg in sorted(by_sock):
            if i < len(by_sock[pkg]):
                phys.append(by_sock[pkg][i])
    quota = None
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()
        quota = None if q == 'max' else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    model = ''
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return dict(affinity=aff, physical=phys, sockets=len(sockets), cgroup_cpu_quota=quota,
                model=model)


def cpu_baseline(seconds, count, crossover_rows):
    """The oracle (clean-room C restatement of MPICH's op_fns.c loop) on a
    bounded sample of the SAME workload: MPI_Reduce_local(MPI_SUM, MPI_FLOAT)
    on `count`-element (1 GiB) host operands.  `value` is one core (MPICH's
    path is one thread per rank); `allcores` runs one pinned thread per
    physical core of this process's CPUs, every thread first-touching its own
    slice (NUMA-local), and is read against a host triad (a += 0.5 b, the
    combine's own traffic) on the same threads and layout.  BASELINE config 1
    (16 MiB) is reported beside it, and one core's time per call at each
    host-crossover size (timed in C, like the GPU side) fills crossover_rows."""
    from oracle import oracle as orc
    orc.build()
    topo = host_topology()
    phys = topo['physical']
    alg = 3 * count * 4

    def leg(cpus, budget, n=count):
        """the reduce and the host triad in the same passes (oracle_bench_pair):
        same pinned threads, same first-touched slices, same quota windows"""
        best, med, passes, span, tbest, tmed, ratio = orc.bench_pair(n, H.MPI_FLOAT, H.MPI_SUM,
                                                                     cpus, budget)
        nb = 3 * n * 4
        return dict(gibs=round(nb / GIB / med, 3), best=round(nb / GIB / best, 3),
                    sustained=round(passes * nb / GIB / span, 3) if span > 0 else None,
                    reps=passes, threads=len(cpus), triad_gibs=round(nb / GIB / tmed, 3),
                    frac=round(tmed / med, 4), frac_per_pass=round(1.0 / ratio, 4) if ratio else None)

    quota = topo['cgroup_cpu_quota']
    nq = max(1, min(len(phys), int(quota))) if quota else len(phys)
    one = leg(phys[:1], seconds * 0.35)
    # every physical core only where no cgroup quota throttles them: with a
    # quota below the thread count the threads run out of it within a pass
    # and the reduce / triad pair is split across throttle windows (the
    # paired ratio read 0.94 and 2.77 on one box, r06f) -- the quota leg is
    # then the multi-core figure
    allc = leg(phys, seconds * 0.25) if nq >= len(phys) else None
    c1 = leg(phys[:1], seconds * 0.1, n=4194304)
    quota_leg = None
    if nq < len(phys):
        q = leg(phys[:nq], seconds * 0.2)
        quota_leg = dict(threads=nq, value=q['gibs'], sustained=q['sustained'],
                         host_triad_gibs=q['triad_gibs'], frac_of_host_triad=q['frac'],
                         frac_of_host_triad_per_pass=q['frac_per_pass'],
                         note='as many pinned threads as the cgroup quota grants CPUs, spread '
                              'over both sockets: what this process can sustain')
    if crossover_rows:
        B = bench_lib()
        fn = ctypes.cast(orc.lib().oracle_reduce_local, ctypes.c_void_p).value
        for r in crossover_rows:
            n = r['bytes'] // 4
            rng = np.random.default_rng(0x5EED0009)
            a = rng.uniform(-1, 1, n).astype(np.float32)
            b = rng.uniform(-1, 1, n).astype(np.float32)
            r['cpu_1core_us'] = round(c_call_median_us(B, fn, a.ctypes.data, b.ctypes.data, n,
                                                       _reps_for(r['bytes'])), 2)
    return dict(
        value=one['gibs'], unit='GiB/s', cores=1, kind='port',
        sample='same workload (MPI_Reduce_local MPI_SUM MPI_FLOAT, %d elements = %d MiB per '
               'operand, host-resident) through oracle/redop_oracle.c, 1 pinned thread, %d calls, '
               'median' % (count, count * 4 >> 20, one['reps']),
        best=one['best'],
        host_triad_1core_gibs=one['triad_gibs'],
        frac_of_host_triad_1core=one['frac'],
        frac_of_host_triad_1core_per_pass=one['frac_per_pass'],
        host_triad_timing='each pass runs the reduce, a barrier, then the triad (a += 0.5 b) on '
                          'the same pinned threads and first-touched slices, so both are read in '
                          'the same quota windows; frac = triad median / reduce median time, '
                          'frac_per_pass = median over passes of triad / reduce time',
        allcores=dict(value=allc['gibs'], threads=allc['threads'], reps=allc['reps'],
                      sustained=allc['sustained'], host_triad_gibs=allc['triad_gibs'],
                      frac_of_host_triad=allc['frac'],
                      frac_of_host_triad_per_pass=allc['frac_per_pass'],
                      note='one pinned thread per physical core of this process (%d sockets), '
                           'each first-touching its own slice of both operands (NUMA-local); '
                           'value = median pass; host triad = a += 0.5 b on the same threads '
                           'and layout (12 B per element, the combine\'s own traffic)'
                           % topo['sockets']) if allc else
        dict(skipped='the cgroup CPU quota (%s CPUs) is below the %d physical cores: %d threads '
                     'would exhaust it within a pass and split each reduce / triad pair across '
                     'throttle windows; quota_threads is the multi-core figure'
                     % (quota, len(phys), len(phys))),
        quota_threads=quota_leg,
        config1_16MiB_1core=dict(value=c1['gibs'], reps=c1['reps'],
                                 note='BASELINE config 1; 48 MiB per call is cache-resident on '
                                      'this host'),
        host_cpu=topo['model'], nproc=os.cpu_count(), affinity_cpus=len(topo['affinity']),
        physical_cores=len(phys), sockets=topo['sockets'],
        cgroup_cpu_quota=quota)


def load_pmc(path, count):
    """The PMC summary of a separate rocprofv3 pass over the same command
    (tools/gpu_evidence.sh, tools/pmc_summary.py) -- quoted, not measured in
    this process, so the line names its source: (HBM bytes per launch, the
    file, the summary's kernel record with the traced average duration and
    the traced run's own ms_per_step)"""
    for p in (path, os.path.join(ROOT, 'profiles', 'r01_pmc_summary.json')):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        k = d.get('kernels', {}).get('reduce_local_fp32_sum')
        if k and k.get('count') == count:
            return k.get('hbm_bytes_per_launch'), os.path.relpath(p, ROOT), k
    return None, None, None


def overlap_note(min_bytes):
    """what the recursive-halving combine overlap does in this run's timed
    calls (libmpix_coll: MPIX_Comm_get_rh_overlap of the communicator; on by
    default -- 1 MiB -- for RCCL communicators only)"""
    if not min_bytes:
        return 'off (every combine whole on the collective\'s stream)'
    return ('each step\'s kept half combined on a second stream under the next exchange '
            '(half-steps >= %d B); the step breakdown is of one call with it off' % min_bytes)


# ------------------------------------------------------------------ N = 1
def reduce_local_leg(args, world, rank, dev):
    """the headline loop: synchronous MPIX_Reduce_local over 1 GiB operands,
    barrier + synchronize around exactly `steps` calls, max over ranks"""
    n = args.count
    inout = torch.empty(n, dtype=torch.float32, device=dev)
    inb = torch.empty(n, dtype=torch.float32, device=dev)
    fill_uniform(inout, 0x5EED0001 + 2 * rank)
    fill_uniform(inb, 0x5EED0002 + 2 * rank)
    torch.cuda.synchronize()

    # one step = one synchronous MPIX_Reduce_local, called back to back from C
    # (libmpix_bench's loop: the C-ABI as MPICH calls it, no Python between
    # the calls); the first call goes through the Python mirror, which checks
    # the buffer spans and the MPI error class
    B = bench_lib()
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local, ctypes.c_void_p).value
    redop.check(redop.MPI_Reduce_local(inb, inout, n, H.MPI_FLOAT, H.MPI_SUM))

    def steps(k):
        tl = ctypes.c_double()
        redop.check(B.mpix_bench_call_loop(fn, inb.data_ptr(), inout.data_ptr(), n,
                                           H.as_c_int(H.MPI_FLOAT), H.as_c_int(H.MPI_SUM), k,
                                           ctypes.byref(tl)), 'MPIX_Reduce_local')

    steps(args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    if world > 1:
        t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
    stream = torch.cuda.current_stream()
    kreps = max(10, min(args.steps, 50))
    call = lambda: redop.check(redop.reduce_local_async(inb, inout, n, H.MPI_FLOAT, H.MPI_SUM,  # noqa
                                                         stream))
    # the kernel as the timed loop runs it: the same synchronous calls from C,
    # back to back, the library recording a HIP event pair around each launch
    # on its own stream (MPIX_Redop_sync_timing) -- the entry's store policy,
    # idle gap and completion wait all as in the timed loop
    dev_index = dev.index if getattr(dev, 'index', None) is not None else torch.cuda.current_device()
    redop.sync_timing(dev_index, 3 * kreps)
    try:
        steps(3 * kreps)
    finally:
        per = sorted(redop.sync_timing_read(dev_index))
    if len(per) != 3 * kreps:
        raise RuntimeError('sync timing recorded %d of %d calls' % (len(per), 3 * kreps))
    k_avg, k_med, k_min = sum(per) / len(per), per[len(per) // 2], per[0]
    sync_mask = redop.get_sync_store_policy()
    # and back to back with the stream-ordered entries' policy (a
    # stream-ordered caller's steady state)
    b_avg, b_med, b_min = event_time_per_launch(call, kreps, stream)
    return dict(t=t, k_avg=k_avg, k_med=k_med, k_min=k_min, kreps=kreps, inb=inb, inout=inout,
                stream=stream, b_avg=b_avg, b_med=b_med, b_min=b_min, sync_mask=sync_mask,
                async_mask=redop.get_store_policy()['xcd_mask'])


def single_gpu(args, dev):
    n = args.count
    nbytes_alg = 3 * n * 4
    leg = reduce_local_leg(args, 1, 0, dev)
    inb, inout, stream, kreps = leg['inb'], leg['inout'], leg['stream'], leg['kreps']
    achieved = nbytes_alg / (leg['k_avg'] * 1e-3) / 1e9
    traffic, traffic_src, traced = load_pmc(args.pmc, n)
    result = {
        'metric': METRIC,
        'value': round(nbytes_alg * args.steps / leg['t'] / GIB, 2),
        'unit': 'GiB/s',
        'n_gpus': 1,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(1e3 * leg['t'] / args.steps, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic (uniform [-1,1), seeded)',
        'config': {
            'workload': 'MPI_Reduce_local(MPI_SUM, MPI_FLOAT) device-resident, BASELINE configs[1] '
                        'at its 1 GiB point',
            'count': n, 'bytes_per_operand': 4 * n, 'algorithmic_bytes_per_step': nbytes_alg,
            'parallelism': 'single GPU',
            'launch': redop.get_launch(),
            'store_policy_xcd_mask': {'synchronous_entry': leg['sync_mask'],
                                      'stream_ordered_entries': leg['async_mask']},
        },
        'roofline': {
            'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBS, 4),
            'traffic': traffic,
            'traffic_source': ('quoted from %s (a separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE '
                               'pass of the same command, gfx950-corrected)' % traffic_src)
                              if traffic_src else None,
            'kernel_ms_avg': round(leg['k_avg'], 4), 'kernel_ms_median': round(leg['k_med'], 4),
            'kernel_ms_min': round(leg['k_min'], 4), 'kernel_launches_timed': 3 * kreps,
            'kernel_timing': 'HIP events recorded by the library around the launch of each of '
                             '%d synchronous MPIX_Reduce_local calls on its own stream '
                             '(MPIX_Redop_sync_timing), the calls issued from C back to back '
                             'right after the timed loop exactly as in it' % (3 * kreps),
            'algorithmic_bytes_per_launch': nbytes_alg,
            'back_to_back': {'kernel_ms_avg': round(leg['b_avg'], 4),
                             'achieved': round(nbytes_alg / (leg['b_avg'] * 1e-3) / 1e9, 1),
                             'frac': round(nbytes_alg / (leg['b_avg'] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             'launches': 3 * kreps,
                             'note': 'one event pair around batches of launches issued back to '
                                     'back (a stream-ordered caller, with the stream-ordered '
                                     'entries\' store policy, DESIGN.md §8)'},
        },
    }
    if traced and traced.get('avg_duration_ns'):
        # the same kernel's rocprofv3 kernel-trace average from the quoted
        # evidence pass, and that run's own step time: frac_traced follows
        # from the file alone (algorithmic bytes / traced average / peak) --
        # over the launches that started from an idle GPU when the file
        # separates them (the regime `frac` is timed in), else over all
        t_ns = float(traced.get('idle_start_avg_ns') or traced['avg_duration_ns'])
        result['roofline'].update(
            frac_traced=round(nbytes_alg / t_ns / HBM_PEAK_GBS, 4),
            traced_kernel_ms_avg=round(t_ns * 1e-6, 4),
            traced_launches=traced.get('idle_start_launches') or traced.get('launches_traced'),
            traced_which=('launches after an idle gap (the synchronous calls)'
                          if traced.get('idle_start_avg_ns') else 'all launches'),
            traced_all_launches_ms_avg=round(float(traced['avg_duration_ns']) * 1e-6, 4),
            traced_run_ms_per_step=traced.get('traced_run_ms_per_step'),
            traced_source=traffic_src)
    crossover = None
    if not args.no_extras:
        B = bench_lib()
        # STREAM triad on the same GPU (three separate 1 GiB fp32 arrays)
        a3 = torch.empty(n, dtype=torch.float32, device=dev)
        tri_avg, _, _ = event_time_per_launch(
            lambda: B.mpix_bench_triad(a3.data_ptr(), inb.data_ptr(), inout.data_ptr(),
                                       ctypes.c_float(0.5), n, stream.cuda_stream), kreps, stream)
        triad = nbytes_alg / (tri_avg * 1e-3) / 1e9
        b2b = nbytes_alg / (leg['b_avg'] * 1e-3) / 1e9      # both timed back to back
        result['roofline']['triad_measured_GBs'] = round(triad, 1)
        result['roofline']['frac_of_triad'] = round(b2b / triad, 4)
        # the same triad with the library's store policy (the blocks of two
        # XCDs store write-through): how much of the combine's lead over the
        # plain triad is the policy, which any streaming kernel can use
        pol = redop.get_store_policy()
        if pol['xcd_mask']:
            trx_avg, _, _ = event_time_per_launch(
                lambda: B.mpix_bench_triad_xcd(a3.data_ptr(), inb.data_ptr(), inout.data_ptr(),
                                               ctypes.c_float(0.5), n, stream.cuda_stream,
                                               pol['xcd_mask']), kreps, stream)
            trx = nbytes_alg / (trx_avg * 1e-3) / 1e9
            result['roofline']['triad_store_policy_GBs'] = round(trx, 1)
            result['roofline']['frac_of_triad_store_policy'] = round(b2b / trx, 4)
        del a3
        result['sync_call_latency'] = sync_call_latency(B, dev)
        # the chunk loops run on a created stream, as a collective engine's
        # combine stream is; the same 64 KiB loop on torch's current (legacy
        # null) stream is reported beside it, since every launch there pays
        # the implicit synchronisation with the other blocking streams
        cs = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        chunked_async_c(B, inb, inout, n, cs, (64 << 10,))     # untimed warm-up of the loop
        result['chunked_async_c'] = chunked_async_c(
            B, inb, inout, n, cs,
            (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20) if args.sweep
            else (64 << 10, 1 << 20, 16 << 20))
        result['chunked_batch_c'] = chunked_batch_c(B, inb, inout, n, cs,
                                                    (64 << 10, 1 << 20))
        result['chunked_async_c_null_stream'] = chunked_async_c(
            B, inb, inout, n, stream, (64 << 10,))
        torch.cuda.synchronize()
        result['call_floor_parts'] = call_floor_parts(B, inb, inout, cs)
        torch.cuda.synchronize()
        end_to_end(result, n, dev)
        crossover = host_crossover_gpu(B)
        result['configs_3_and_5'] = other_configs(inb, inout, n, stream)
    if args.sweep:
        result['sweep'] = size_sweep(inb, inout, n, stream, nbytes_alg)
    del inout, inb
    torch.cuda.empty_cache()
    if not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(args.cpu_seconds, args.count, crossover)
        if crossover:
            sup = redop.get_support()
            result['host_crossover'] = dict(
                rows=crossover,
                pageable_crossover_bytes=crossover_from(crossover, 'gpu_pageable_us'),
                pinned_crossover_bytes=crossover_from(crossover, 'gpu_pinned_us'),
                library_floors=dict(pageable=sup['host_floor_bytes'],
                                    pinned=sup['pinned_floor_bytes']),
                note='bytes per operand; GPU = synchronous MPIX_Reduce_local on host operands, '
                     'CPU = the oracle loop on one core, both median per call timed in C; the '
                     'crossover is the smallest size from which the GPU path is faster or within 5 % '
                     'at every larger size (the MPIX_Redop_is_supported_buffers floor)')
    print(json.dumps(result, default=str), flush=True)


# ---------------------------------------------------------------- config 3 inputs
# SURVEY §8(d) C3 on the device (torch's seeded Philox generator): ints
# uniform over the full range (30 % zero elements, the logical ops' false),
# floats uniform [-1, 1) plus 1 % specials (+-0, +-Inf, NaN) and fp32
# subnormals, bf16 with ties-away cases, Fortran logicals .TRUE./.FALSE. and
# other values, pairs with values in 0..15 (ties) and NaNs, random pair
# padding.  tests/test_c3_full.py draws its parity operands from the same
# generator; the config-3 throughput rows below time on them.
C3_FDT = {2: torch.float16, 4: torch.float32, 8: torch.float64}
C3_IDT = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
C3_TYPES = (('MPI_INT8_T', 'int', 1), ('MPI_INT16_T', 'int', 2), ('MPI_INT32_T', 'int', 4),
            ('MPI_INT64_T', 'int', 8), ('MPI_INTEGER16', 'int', 16), ('MPIX_C_FLOAT16', 'fp', 2),
            ('MPIX_BFLOAT16', 'bf16', 2), ('MPI_FLOAT', 'fp', 4), ('MPI_DOUBLE', 'fp', 8),
            ('MPI_COMPLEX4', 'cplx', 2), ('MPI_C_FLOAT_COMPLEX', 'cplx', 4),
            ('MPI_C_DOUBLE_COMPLEX', 'cplx', 8), ('MPI_C_BOOL', 'int', 1), ('MPI_LOGICAL', 'flog', 4),
            ('MPI_BYTE', 'int', 1), ('MPI_2INT', ('pair', '<i4', '<i4', 8, 4), None),
            ('MPI_FLOAT_INT', ('pair', '<f4', '<i4', 8, 4), None),
            ('MPI_DOUBLE_INT', ('pair', '<f8', '<i4', 16, 8), None),
            ('MPI_SHORT_INT', ('pair', '<i2', '<i4', 8, 4), None))


def _c3_bytes(g, nbytes):
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device='cuda', generator=g)


def _c3_u(g, n, dt=torch.float32):
    return torch.rand(n, dtype=dt, device='cuda', generator=g)


def _c3_fp(g, n, size):
    x = (_c3_u(g, n, torch.float64 if size == 8 else torch.float32) * 2 - 1).to(C3_FDT[size])
    sp = torch.tensor([0.0, -0.0, float('inf'), float('-inf'), float('nan')], dtype=C3_FDT[size],
                      device='cuda')
    k = _c3_u(g, n) < 0.01
    x[k] = sp[torch.randint(0, 5, (int(k.sum()),), device='cuda', generator=g)]
    if size == 4:       # subnormals must not be flushed
        d = _c3_u(g, n) < 0.003
        x[d] = ((_c3_u(g, int(d.sum())) * 2 - 1) * 1e-39).to(torch.float32)
    return x.view(torch.uint8)


def c3_operand(g, kind, size, n):
    """one config-3 operand of n elements of `kind` as a device uint8 tensor"""
    if kind == 'int':
        a = _c3_bytes(g, n * size).view(n, size)
        a[_c3_u(g, n) < 0.3] = 0                # logical-false elements
        return a.reshape(-1)
    if kind == 'flog':
        vals = torch.tensor([0, 1, -1, 5, 0], dtype=torch.int64, device='cuda')
        v = vals[torch.randint(0, 5, (n,), device='cuda', generator=g)]
        if size <= 8:
            return v.to(C3_IDT[size]).view(torch.uint8)
        return torch.stack([v, torch.where(v < 0, -1, 0)], 1).view(torch.uint8).reshape(-1)
    if kind == 'fp':
        return _c3_fp(g, n, size)
    if kind == 'cplx':
        return _c3_fp(g, 2 * n, size)
    if kind == 'bf16':
        f = _c3_u(g, n) * 8 - 4
        k = _c3_u(g, n) < 0.01
        sp = torch.tensor([float('inf'), float('-inf'), 0.0, -0.0], device='cuda')
        f[k] = sp[torch.randint(0, 4, (int(k.sum()),), device='cuda', generator=g)]
        b = (f.view(torch.int32) >> 16).to(torch.int32) & 0xffff
        b ^= torch.randint(0, 2, (n,), dtype=torch.int32, device='cuda', generator=g)
        nan = ((b & 0x7f80) == 0x7f80) & ((b & 0x7f) != 0)
        b[nan] = 0x3f80
        return b.to(torch.int16).view(torch.uint8)
    vdt, ldt, ext, loff = kind[1:]
    buf = _c3_bytes(g, n * ext).view(n, ext)    # random padding
    vs, ls = np.dtype(vdt).itemsize, np.dtype(ldt).itemsize
    v = torch.randint(0, 16, (n,), device='cuda', generator=g)
    if vdt.startswith('<f'):
        v = v.to(C3_FDT[vs])
        v[_c3_u(g, n) < 0.02] = float('nan')
    else:
        v = v.to(C3_IDT[vs])
    lv = torch.randint(-1000, 1000, (n,), device='cuda', generator=g).to(C3_IDT[ls])
    buf[:, :vs] = v.view(torch.uint8).view(n, vs)
    buf[:, loff:loff + ls] = lv.view(torch.uint8).view(n, ls)
    return buf.reshape(-1)


def fill_soft_slots(buf8, enc, seed):
    """buf8 (a multiple of 16 bytes) as 16-byte slots, each a uniform [-1, 1)
    double widened exactly to `enc`: 'x87' (64-bit significand with its
    explicit integer bit, 15-bit exponent, sign; bytes 10-15 zero) or
    'binary128' (IEEE quad, 112-bit fraction)"""
    slots = buf8.view(torch.int64).view(-1, 2)
    d = torch.empty(slots.shape[0], dtype=torch.float64, device=buf8.device)
    fill_uniform(d, seed)
    bits = d.view(torch.int64)
    sign = (bits >> 63) & 1
    e = (bits >> 52) & 0x7ff
    f = bits & ((1 << 52) - 1)
    ex = torch.where(e == 0, torch.zeros_like(e), e - 1023 + 16383)   # +-0 stays zero
    if enc == 'x87':
        lo = torch.where(e == 0, torch.zeros_like(f), (f << 11) | torch.tensor(-(1 << 63), device=d.device))
        hi = (sign << 15) | ex
    else:
        lo = (f & 0xf) << 60
        hi = (sign << 63) | (ex << 48) | (f >> 4)
    slots[:, 0] = lo
    slots[:, 1] = hi
    del d


def fresh_event_time(launch, prep, reps, stream):
    """median duration of `launch()` with every launch on fresh operands:
    `prep()` (enqueued on `stream`, outside the event pair) restores them
    first, so a data-dependent combiner is timed on the distribution it
    claims rather than on values its own repeated folds moved"""
    per = []
    with torch.cuda.stream(stream):
        for _ in range(reps):
            prep()
            s0 = torch.cuda.Event(enable_timing=True)
            s1 = torch.cuda.Event(enable_timing=True)
            s0.record(stream)
            launch()
            s1.record(stream)
            s1.synchronize()
            per.append(s0.elapsed_time(s1))
    per.sort()
    return per[len(per) // 2]


def other_configs(inb, inout, n, stream):
    """BASELINE configs 3 and 5 on the same buffers (kernel-only, HIP events):
    every supported (op, type) pair at 1 GiB per operand (past the 256 MB
    MALL; min / median / max over the pairs, and the slowest three), and
    vector(2^26, 1, 2, MPI_DOUBLE) SUM on a 1 GiB target span (algorithmic
    bytes 3 x 512 MiB; physical floor 2.5 GiB)"""
    nbytes = 4 * n
    a8 = inout.view(torch.uint8)
    b8 = inb.view(torch.uint8)
    rows = []
    g = torch.Generator(device='cuda')
    for tn, kind, size in C3_TYPES:
        dt = getattr(H, tn)
        ext = redop.datatype_extent(dt)
        m = nbytes // ext
        # the C3 distributions (c3_operand), drawn per type; inout is restored
        # from a0 before each op's calls (the repeated in-place
        # folds move the values -- PROD drives them to 0 / subnormal / Inf /
        # NaN).  The complex products have a data-dependent path (the C99
        # Annex G recovery, per lane when both parts come out NaN), so their
        # rows restore inout before every timed launch; the other combiners
        # have no data-dependent path and are timed back to back.
        g.manual_seed((0x5EED0003 * 31 + dt) & 0xffffffff)
        a0 = c3_operand(g, kind, size, m)
        b8[:m * ext].copy_(c3_operand(g, kind, size, m))
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        for on, op in H.OPS.items():
            if op in (H.MPI_REPLACE, H.MPI_NO_OP) or not redop.is_supported(op, dt):
                continue
            a8[:m * ext].copy_(a0)
            call = lambda: redop.check(redop.reduce_local_async(b8, a8, m, dt, op, stream))  # noqa
            if kind == 'cplx' and op == H.MPI_PROD:
                torch.cuda.synchronize()
                med = fresh_event_time(call, lambda: a8[:m * ext].copy_(a0), 7, stream)
            else:
                call()
                # median of three batches of five: one disturbed batch (seen
                # once at 0.62 of the row's rate, profiles/r04_bench_n1.json)
                # does not set the row
                _, med, _ = event_time_per_launch(call, 5, stream, rounds=3)
            rows.append((round(3 * m * ext / (med * 1e-3) / 1e9, 1), tn, on))
        del a0
    rows.sort()
    gbs = [r[0] for r in rows]
    # beyond config 3's types: the x87 / binary128 families (software
    # arithmetic for SUM / PROD, integer compare-and-select for the rest), on
    # normal values: every 16-byte slot holds a uniform [-1, 1) double widened
    # to the type's encoding (small random bytes would make every x87 slot an
    # unnormal -- integer bit clear -- and time the invalid-operand path)
    soft = []
    for tn in ('MPI_LONG_DOUBLE', 'MPI_REAL16', 'MPI_C_LONG_DOUBLE_COMPLEX', 'MPI_COMPLEX32',
               'MPI_LONG_DOUBLE_INT'):
        enc = 'x87' if 'LONG_DOUBLE' in tn else 'binary128'
        fill_soft_slots(b8, enc, 0x5EED0004)
        torch.cuda.synchronize()
        dt = getattr(H, tn)
        ext = redop.datatype_extent(dt)
        m = nbytes // ext
        for on, op in H.OPS.items():
            if op in (H.MPI_REPLACE, H.MPI_NO_OP) or not redop.is_supported(op, dt):
                continue
            fill_soft_slots(a8, enc, 0x5EED0003)        # every op on the same normal values
            redop.check(redop.reduce_local_async(b8, a8, m, dt, op, stream))
            _, med, _ = event_time_per_launch(
                lambda: redop.check(redop.reduce_local_async(b8, a8, m, dt, op, stream)), 3, stream,
                rounds=3)
            soft.append(dict(type=tn, op=on, GBs=round(3 * m * ext / (med * 1e-3) / 1e9, 1)))
    cnt = 1 << 26
    src = inb.view(torch.float64)[:cnt]
    dst = inout.view(torch.float64)[:2 * cnt]
    src.zero_()
    dst.zero_()
    torch.cuda.synchronize()
    redop.check(redop.reduce_local_vector(src, dst, cnt, 1, 2, H.MPI_DOUBLE, H.MPI_SUM, stream))
    vavg, _, _ = event_time_per_launch(
        lambda: redop.check(redop.reduce_local_vector(src, dst, cnt, 1, 2, H.MPI_DOUBLE, H.MPI_SUM,
                                                      stream)), 10, stream)
    return dict(
        config3_per_pair_1GiB=dict(pairs=len(rows), min_GBs=gbs[0], median_GBs=gbs[len(gbs) // 2],
                                   values='SURVEY 8(d) C3 distributions per type (bench.c3_operand); '
                                          'inout restored before each op, and before every '
                                          'launch for the complex PROD rows (data-dependent '
                                          'Annex G path)',
                                   max_GBs=gbs[-1], min_frac=round(gbs[0] / HBM_PEAK_GBS, 4),
                                   slowest=[dict(GBs=g, type=t, op=o) for g, t, o in rows[:3]],
                                   every_row=[[t, o, g] for g, t, o in rows]),
        x87_binary128_1GiB=soft,
        x87_binary128_values='every 16-byte slot a uniform [-1, 1) double widened exactly to the '
                             'x87 / binary128 encoding (bench.fill_soft_slots)',
        config5_vector=dict(kernel_ms=round(vavg, 4),
                            GBs_algorithmic=round(3 * cnt * 8 / (vavg * 1e-3) / 1e9, 1),
                            GBs_physical=round(2.5 * GIB / (vavg * 1e-3) / 1e9, 1),
                            frac_algorithmic=round(3 * cnt * 8 / (vavg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                   4)))


def pcie_rates(hin, hio, dev, reps=3):
    """measured PCIe rates between this GPU and page-locked host memory
    (hipMemcpyAsync through torch copies, 1 GiB each): H2D alone, D2H alone,
    and the zero-copy call's own pattern -- `in` and `inout` in (2 x H2D)
    while the result goes out (1 x D2H) at the same time, on two streams.
    That pattern's time is the PCIe floor of a host-resident call."""
    n = hin.numel()
    d0 = torch.empty(n, dtype=torch.float32, device=dev)
    d1 = torch.empty(n, dtype=torch.float32, device=dev)
    s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        return best

    def h2d():
        with torch.cuda.stream(s_in):
            d0.copy_(hin, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s_out):
            hio.copy_(d1, non_blocking=True)

    def pattern():
        with torch.cuda.stream(s_in):
            d0.copy_(hin, non_blocking=True)
            d0.copy_(hin, non_blocking=True)
        with torch.cuda.stream(s_out):
            hio.copy_(d1, non_blocking=True)
    nb = 4 * n
    t_h2d, t_d2h = timed(h2d), timed(d2h)
    # the call's floor: its 2 GiB in at the H2D rate and its 1 GiB out at the
    # D2H rate, the two directions concurrent (full duplex)
    t_floor = max(2 * t_h2d, t_d2h)
    d1.copy_(hio)           # the operands keep their values for the timed calls
    torch.cuda.synchronize()
    t_pat = timed(pattern)
    with torch.no_grad():
        hio.copy_(d1)
    del d0, d1
    return dict(h2d_GBs=round(nb / t_h2d / 1e9, 2), d2h_GBs=round(nb / t_d2h / 1e9, 2),
                floor_ms=round(t_floor * 1e3, 2),
                sdma_pattern_2h2d_1d2h_ms=round(t_pat * 1e3, 2),
                note='page-locked host <-> HBM copies (SDMA), 1 GiB each, best of %d; floor = '
                     'max(2 GiB at the H2D rate, 1 GiB at the D2H rate), the call\'s own '
                     'traffic with both directions at once; the SDMA engines themselves reach '
                     'only sdma_pattern when both directions run together' % reps), t_floor


def end_to_end(result, n, dev=None):
    """host-resident end to end (never `value`): pinned operands read and
    written by the kernel over PCIe; pageable operands through the host
    workers and through hipMemcpyAsync staging; each against the measured
    PCIe floor of the same traffic"""
    hin = torch.empty(n, dtype=torch.float32).pin_memory()
    hio = torch.empty(n, dtype=torch.float32).pin_memory()
    hin.uniform_(-1, 1)
    hio.uniform_(-1, 1)
    pcie, t_floor = pcie_rates(hin, hio, dev if dev is not None else torch.device('cuda', 0))
    redop.check(redop.MPI_Reduce_local(hin, hio, n, H.MPI_FLOAT, H.MPI_SUM))
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        redop.check(redop.MPI_Reduce_local(hin, hio, n, H.MPI_FLOAT, H.MPI_SUM))
    te = (time.perf_counter() - t0) / reps
    result['end_to_end_host'] = dict(gibs=round(3 * n * 4 / GIB / te, 2),
                                     ms_per_call=round(te * 1e3, 2),
                                     frac_of_pcie=round(t_floor / te, 4), pcie=pcie,
                                     note='pinned host buffers: the kernel reads and writes '
                                          'them over PCIe (zero-copy); never `value`; '
                                          'frac_of_pcie = measured PCIe floor of the same '
                                          'traffic / call time')
    # SURVEY.md §8(d)'s end-to-end as written: hipMemcpyAsync H2D(in, inout),
    # the kernel, D2H(inout) from the same page-locked buffers, one stream,
    # whole 1 GiB operands (no chunk pipelining), timed as a whole
    d = dev if dev is not None else torch.device('cuda', 0)
    din = torch.empty(n, dtype=torch.float32, device=d)
    dio = torch.empty(n, dtype=torch.float32, device=d)
    cs = torch.cuda.Stream(d)

    def copy_call():
        with torch.cuda.stream(cs):
            din.copy_(hin, non_blocking=True)
            dio.copy_(hio, non_blocking=True)
            redop.check(redop.reduce_local_async(din, dio, n, H.MPI_FLOAT, H.MPI_SUM, cs))
            hio.copy_(dio, non_blocking=True)
        cs.synchronize()
    copy_call()
    t0 = time.perf_counter()
    for _ in range(reps):
        copy_call()
    tc = (time.perf_counter() - t0) / reps
    result['end_to_end_host']['memcpy_kernel_memcpy'] = dict(
        gibs=round(3 * n * 4 / GIB / tc, 2), ms_per_call=round(tc * 1e3, 2),
        frac_of_pcie=round(t_floor / tc, 4),
        note='SURVEY 8(d) end-to-end as written: hipMemcpyAsync H2D of both operands, the '
             'kernel, hipMemcpyAsync D2H of inout, from the same page-locked buffers on one '
             'stream, whole operands; the zero-copy call above is the library\'s own form')
    del hin, hio, din, dio
    pin_ = np.random.default_rng(0x5EED0007).random(n, dtype=np.float32)
    pio_ = np.random.default_rng(0x5EED0008).random(n, dtype=np.float32)
    prev = redop.get_pageable()
    pg = {}
    try:
        for label, threads in (('workers', prev['threads'] or 8), ('staged', 0)):
            redop.check(redop.set_pageable(threads, prev['chunk_bytes']))
            redop.check(redop.MPI_Reduce_local(pin_, pio_, n, H.MPI_FLOAT, H.MPI_SUM))
            t0 = time.perf_counter()
            for _ in range(reps):
                redop.check(redop.MPI_Reduce_local(pin_, pio_, n, H.MPI_FLOAT, H.MPI_SUM))
            tp = (time.perf_counter() - t0) / reps
            pg[label] = dict(gibs=round(3 * n * 4 / GIB / tp, 2), ms_per_call=round(tp * 1e3, 2),
                             frac_of_pcie=round(t_floor / tp, 4))
    finally:
        redop.check(redop.set_pageable(prev['threads'], prev['chunk_bytes']))
    pg['workers_x_chunk'] = '%d x %d MiB' % (prev['threads'] or 8, prev['chunk_bytes'] >> 20)
    pg['form'] = os.environ.get('MPIX_REDOP_PAGEABLE_MODE', 'wave')
    pg['vs_pinned'] = round(result['end_to_end_host']['ms_per_call'] / pg['workers']['ms_per_call'], 4)
    pg['note'] = ('pageable (numpy) host buffers; never `value`; workers = the library\'s host '
                  'threads (wave form: all copy one chunk into page-locked memory while one '
                  'zero-copy kernel combines the previous one), staged = hipMemcpyAsync through '
                  'device scratch; vs_pinned = pinned call time / workers call time')
    result['end_to_end_pageable'] = pg


def size_sweep(inb, inout, n, stream, nbytes_alg):
    sweep = []
    for mib in (16, 32, 64, 128, 256, 512, 1024):
        m = mib * (1 << 20) // 4
        if m > n:
            break
        avg, _, _ = event_time_per_launch(
            lambda: redop.check(redop.reduce_local_async(inb, inout, m, H.MPI_FLOAT,
                                                         H.MPI_SUM, stream)), 20, stream)
        sweep.append(dict(mib=mib, kernel_ms=round(avg, 4),
                          GBs=round(3 * m * 4 / (avg * 1e-3) / 1e9, 1)))
    # the chunked sweep replayed from a HIP graph: the launch-bound small
    # chunks lose the per-call host launch cost
    graphed = []
    gs = torch.cuda.Stream()
    for ck in (64 << 10, 256 << 10, 1 << 20, 4 << 20):
        m = ck // 4
        nch = min(n // m, 4096)
        g = torch.cuda.CUDAGraph()
        gs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(gs):
            with torch.cuda.graph(g, stream=gs):
                for k in range(nch):
                    redop.check(redop.reduce_local_async(inb[k * m:], inout[k * m:], m,
                                                         H.MPI_FLOAT, H.MPI_SUM, gs))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        graphed.append(dict(chunk_bytes=ck, calls=nch, GiBs=round(3 * m * 4 * nch / tt / GIB, 1)))
        del g
    return dict(size_kernel=sweep, chunked_hipgraph_replay=graphed)


# ------------------------------------------------------------------ N > 1
def progress(rank, what):
    """one stderr line per leg from rank 0 (long N > 1 runs show they move)"""
    if rank == 0:
        sys.stderr.write('[bench %s] %s\n' % (time.strftime('%H:%M:%S'), what))
        sys.stderr.flush()


def schedule_ran(cc, requested, kind='rs'):
    """which schedule the last collective on communicator `cc` actually ran
    (MPIX_Comm_get_state): a requested pull whose windows failed verification
    on some rank, or a shape a variant does not cover, runs the schedule with
    the same bits instead -- its time must never be reported under the
    requested name.  Returns the fields a leg carries; 'error' is set when
    the requested schedule did not run (the leg is then not timed)."""
    st = cc.state()
    ran = st['last_rs'] if kind == 'rs' else st['last_allreduce']
    out = dict(schedule_requested=requested, schedule_ran=ran,
               window_retries=st['window_retries'], pulls_enabled=st['pulls_enabled'])
    if ran != requested:
        out['error'] = 'fell back to %s' % ran
    return out


def rh_expected_block(sends, rank, recvcount):
    """rank's block of MPI_Reduce_scatter_block by recursive halving, as the
    reference schedule associates it (…recursive_halving.c:110-229): the
    non-power-of-two fold (odd rank 2i+1 adds rank 2i's vector), then per
    step with mask = pof2/2 .. 1 every new rank adds its partner's partial
    (one IEEE fp32 add each, so the tree alone fixes the bits)"""
    P = len(sends)
    pof2 = 1
    while pof2 * 2 <= P:
        pof2 *= 2
    rem = P - pof2
    parts = [sends[2 * i + 1] + sends[2 * i] for i in range(rem)] + \
        [sends[r] for r in range(2 * rem, P)]
    m = pof2 // 2
    while m:
        parts = [parts[q] + parts[q ^ m] for q in range(pof2)]
        m //= 2
    owner = rank // 2 if rank < 2 * rem else rank - rem
    return parts[owner][rank * recvcount:(rank + 1) * recvcount]


class ParityError(RuntimeError):
    """a bit-exactness or closed-form check failed: never a timing problem,
    so the run fails non-zero even when it happens in a secondary leg"""


def rh_expected_block_device(world, rank, recvcount, seed0, dev, own=None):
    """rh_expected_block at the timed size, on the device: block `rank` of
    every rank's vector (fill_uniform with seed0 + q, regenerated here one
    vector at a time; `own` = this rank's send buffer, not regenerated) folded
    in the schedule's association -- the non-power-of-two fold (odd rank
    2i+1 adds rank 2i), then per step with mask = pof2/2 .. 1 every new rank
    adds its partner's partial (one IEEE fp32 add each, commutative, so both
    members of a pair share one sum tensor).  Peak extra memory: one vector
    and the P blocks."""
    total = world * recvcount

    def block(q):
        if q == rank and own is not None:
            return own[rank * recvcount:(rank + 1) * recvcount].clone()
        v = torch.empty(total, dtype=torch.float32, device=dev)
        fill_uniform(v, seed0 + q)
        b = v[rank * recvcount:(rank + 1) * recvcount].clone()
        del v
        return b
    pof2 = 1
    while pof2 * 2 <= world:
        pof2 *= 2
    rem = world - pof2
    parts = []
    for i in range(rem):
        odd = block(2 * i + 1)
        odd += block(2 * i)
        parts.append(odd)
    parts += [block(r) for r in range(2 * rem, world)]
    m = pof2 // 2
    while m:
        for q in range(pof2):
            if q < q ^ m:
                t = parts[q] + parts[q ^ m]
                parts[q] = parts[q ^ m] = t
        m //= 2
    owner = rank // 2 if rank < 2 * rem else rank - rem
    out = parts[owner]
    del parts
    torch.cuda.empty_cache()
    return out


def bits_equal_all_ranks(got, want, dev):
    """torch.equal on the int32 view (NaN payloads and -0 included), MIN over ranks"""
    same = bool(torch.equal(got.view(torch.int32), want.view(torch.int32)))
    return allreduce_scalar(1.0 if same else 0.0, dist.ReduceOp.MIN, dev) == 1.0


def rsb_inputs_host(r, P, recvcount):
    return np.random.default_rng(0x5EED0100 + r).uniform(-1, 1, P * recvcount).astype(np.float32)


def multi_gpu(args, world, rank, dev):
    from mpich_amd import ccl
    result = {'metric': METRIC_RSB, 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
              'unit': 'GB/s', 'higher_is_better': True, 'scaling': 'strong', 'vs_baseline': None,
              'dtype': 'f32', 'data': 'synthetic (uniform [-1,1), seeded per rank)',
              'launcher': 'bench.py' if os.environ.get('MPIX_BENCH_LAUNCHED') else 'external'}
    # the round-1 figure, kept as an extra: N independent 1 GiB local reductions
    leg = reduce_local_leg(args, world, rank, dev)
    n = args.count
    result['reduce_local_replicas'] = dict(
        value_GiBs=round(world * 3 * n * 4 * args.steps / leg['t'] / GIB, 2),
        ms_per_step=round(1e3 * leg['t'] / args.steps, 4),
        kernel_ms_avg_rank0=round(leg['k_avg'], 4),
        note='every rank reduces its own 1 GiB operands, no collective (round-1 N>1 value)')
    del leg
    torch.cuda.empty_cache()

    if dist.get_backend() == 'nccl':
        cc = ccl.comm_create_ccl_from_process_group()
    else:   # 1-GPU rehearsal: the same C++ schedules over gloo through pinned staging
        from mpich_amd import coll
        cc = coll.comm_for(None, True)
    _CCL['comm'] = cc
    total = (args.rsb_bytes // 4) // world * world
    recvcount = total // world
    # parity before timing: fp32 SUM at a reduced size, bit for bit against
    # the schedule's association restated in numpy on every rank, checked
    # with every half-step's combine split onto the second stream (overlap
    # threshold 1 byte) and with none split (0).  A failure in either form
    # fails the run: the shipped default must never be timed unchecked.
    progress(rank, 'value leg: parity gate')
    shipped_overlap = cc.rh_overlap()
    rc_small = (1 << 16) + 3
    sends = [rsb_inputs_host(r, world, rc_small) for r in range(world)]
    ds = torch.from_numpy(sends[rank]).to(dev)
    dr = torch.empty(rc_small, dtype=torch.float32, device=dev)
    expected = rh_expected_block(sends, rank, rc_small).tobytes()
    try:
        for mode in (1, 0):
            cc.set_rh_overlap(mode)
            dr.fill_(float('nan'))
            redop.check(ccl.reduce_scatter_block(ds, dr, rc_small, H.MPI_FLOAT, H.MPI_SUM, cc,
                                                 'recursive_halving'), 'MPIX_Reduce_scatter_block')
            sched = schedule_ran(cc, 'recursive_halving')
            if 'error' in sched:
                raise RuntimeError('value leg: recursive halving requested, ' + sched['error'])
            ok = dr.cpu().numpy().tobytes() == expected
            if allreduce_scalar(1.0 if ok else 0.0, dist.ReduceOp.MIN, dev) != 1.0:
                raise ParityError('recursive-halving RSB differs from the reference association '
                                  '(fp32 SUM, recvcount %d, combine overlap %s) on some rank'
                                   % (rc_small, 'on every half-step' if mode else 'off'))
    finally:
        cc.set_rh_overlap(shipped_overlap)
    del ds, dr, sends

    send = torch.empty(total, dtype=torch.float32, device=dev)
    fill_uniform(send, 0x5EED0100 + rank)
    recv = torch.empty(recvcount, dtype=torch.float32, device=dev)
    ws = torch.empty(ccl.rsb_workspace_bytes(recvcount, H.MPI_FLOAT, cc, 'recursive_halving'),
                     dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def step():
        redop.check(ccl.reduce_scatter_block(send, recv, recvcount, H.MPI_FLOAT, H.MPI_SUM, cc,
                                             'recursive_halving', workspace=ws),
                    'MPIX_Reduce_scatter_block')

    progress(rank, 'value leg: %d warmup + %d timed calls' % (args.warmup, args.steps))
    for _ in range(args.warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t = allreduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX, dev) / args.steps
    # the timed calls' own result, at the timed size, on every rank (VERDICT
    # r05 item 1): `send` never changes, so `recv` holds one call's block;
    # it must equal the recursive-halving association of every rank's seeded
    # vector regenerated on the device (…recursive_halving.c:164-229)
    progress(rank, 'value leg: full-size bit check')
    if os.environ.get('MPIX_BENCH_FAULT_RANK') == str(rank):
        # test hook (tests/test_bench_gpu.py): one flipped bit in this rank's
        # timed result must fail the run with EXIT_PARITY
        recv[recvcount // 2:recvcount // 2 + 1].view(torch.int32).bitwise_xor_(1)
    expected = rh_expected_block_device(world, rank, recvcount, 0x5EED0100, dev, own=send)
    if not bits_equal_all_ranks(recv, expected, dev):
        raise ParityError('the timed recursive-halving RSB result differs from the reference '
                          'association at the timed size (fp32 SUM, recvcount %d) on some rank'
                          % recvcount)
    busbytes = (world - 1) / world * total * 4
    pof2 = 1
    while pof2 * 2 <= world:
        pof2 *= 2
    link_bytes = (pof2 - 1) / pof2 * total * 4      # received over one link across the steps
    # per-step breakdown on rank 0's stream, of one extra
    # call with the combine overlap off (every combine whole on the collective's
    # stream, so its marks bracket the combine kernel alone; same bits)
    cc.set_rh_overlap(0)
    cc.set_step_timing(True)
    step()
    torch.cuda.synchronize()
    cc.set_step_timing(False)
    cc.set_rh_overlap(shipped_overlap)
    steps = cc.step_times()
    progress(rank, 'value leg: defaults A/B')
    if not bits_equal_all_ranks(recv, expected, dev):
        raise ParityError('recursive-halving RSB with the combine overlap off differs from the '
                          'reference association at the timed size on some rank')
    ab = None if args.no_ab else defaults_ab(cc, step, recv, expected, dev, args.ab_reps,
                                             args.ab_rounds)
    del expected
    progress(rank, 'value leg: CPU baseline (the reference schedule\'s host work)')
    cpu = None if args.no_cpu_baseline else rsb_cpu_baseline(world, rank, recvcount, dev)
    comb_ms = sum(s['ms'] for s in steps if s['phase'] == 'combine')
    exch_ms = sum(s['ms'] for s in steps if s['phase'] == 'exchange')
    combined = (pof2 - 1) / pof2 * total            # elements this rank combined (pof2 ranks)
    comb_gbs = 3 * combined * 4 / (comb_ms * 1e-3) / 1e9 if comb_ms > 0 else None
    result.update(
        value=round(busbytes / t / 1e9, 2),
        ms_per_step=round(t * 1e3, 4),
        config={'workload': 'MPI_Reduce_scatter_block(MPI_SUM, MPI_FLOAT), BASELINE configs[3]: '
                            '4 GiB vector per rank, recursive halving, RCCL/xGMI chunk transport',
                'vector_bytes_per_rank': total * 4, 'recvcount': recvcount,
                'parallelism': 'rsb%d (one rank per GPU, libmpix_coll over RCCL)' % world},
        parity=dict(checked=True, recvcount=rc_small, bit_exact_all_ranks=True,
                    combine_overlap_checked=['every half-step split', 'none split'],
                    against='numpy restatement of the recursive-halving association',
                    full_size_bit_exact_all_ranks=True, full_size_recvcount=recvcount,
                    full_size_checked=['the timed calls\' result (shipped overlap %s)'
                                       % ('on' if shipped_overlap else 'off'),
                                       'the step-timing call (overlap off)'] +
                                      (['every defaults_ab variant'] if ab else []),
                    full_size_against='the recursive-halving association of every rank\'s '
                                      'seeded vector regenerated on the device '
                                      '(bench.rh_expected_block_device), torch.equal on the '
                                      'int32 view, MIN over ranks'),
        schedule_ran=sched['schedule_ran'],
        combine_overlap=overlap_note(shipped_overlap),
        roofline={'bound': 'hbm', 'unit': 'GB/s',
                  'achieved': round(comb_gbs, 1) if comb_gbs else None, 'peak': HBM_PEAK_GBS,
                  'frac': round(comb_gbs / HBM_PEAK_GBS, 4) if comb_gbs else None,
                  'traffic': None,
                  'what': 'the HIP combine steps of rank 0 (3 x 4 B per combined element over '
                          'their event-timed device time)',
                  'link': {'bound': 'xgmi', 'achieved': round(link_bytes / t / 1e9, 2),
                           'peak': XGMI_LINK_GBS,
                           'frac': round(link_bytes / t / 1e9 / XGMI_LINK_GBS, 4),
                           'note': 'bytes a rank receives over its one active link across the '
                                   'log2(P) steps / step time'}},
        steps_rank0=steps,
        step_split_rank0=dict(exchange_ms=round(exch_ms, 3), combine_ms=round(comb_ms, 3)),
        defaults_ab=ab)
    if cpu is not None:
        result['cpu_baseline'] = dict(value=round(busbytes / cpu.pop('value_s') / 1e9, 3), **cpu)
    del send, recv, ws
    torch.cuda.empty_cache()
    return result


def host_memory_budget():
    """bytes this node's ranks may still take: MemAvailable, and the cgroup's
    memory.max less its current use when one is set"""
    avail = None
    try:
        for line in open('/proc/meminfo'):
            if line.startswith('MemAvailable:'):
                avail = int(line.split()[1]) * 1024
                break
    except (OSError, ValueError):
        pass
    try:
        mx = open('/sys/fs/cgroup/memory.max').read().strip()
        if mx != 'max':
            cur = int(open('/sys/fs/cgroup/memory.current').read())
            left = int(mx) - cur
            avail = left if avail is None else min(avail, left)
    except (OSError, ValueError):
        pass
    return avail


def rsb_cpu_baseline(world, rank, recvcount, dev, reps=3):
    """The N > 1 line's CPU baseline:
    the reference's own host work for this collective -- recursive halving
    keeps the vector in host temporaries (…recursive_halving.c:80-88), copies
    the send buffer in (:91-96), combines each step's received half with
    MPIR_Reduce_local (:219-221; log2(P) combines of n/2, n/4, ... elements)
    and copies its block out (:232-235) -- timed with the oracle's op_fns.c
    loop (oracle/host_bench.c oracle_bench_rsb_rank) on one pinned core per
    rank, all ranks at once between barriers, the max over ranks.  The
    exchange is not the CPU's work and is not in it, so `value` (bus bytes /
    that time, GB/s) is the most the reference's CPU path could reach with a
    free network.  When the node's host memory cannot hold every rank's
    three full-size host vectors the sample is scaled down by a power of two
    and the times scaled back up (the work is linear streams); `sample` says
    which."""
    from oracle import oracle as orc
    orc.build()
    topo = host_topology()
    phys = topo['physical']
    cpu = phys[rank % len(phys)]
    total = world * recvcount
    need = world * (3 * total + recvcount) * 4
    budget = host_memory_budget()
    scale = 1
    while budget is not None and need // scale > 0.6 * budget and recvcount // (2 * scale) >= 1024:
        scale *= 2
    scale = int(allreduce_scalar(float(scale), dist.ReduceOp.MAX, dev))
    rc = recvcount // scale
    dist.barrier()
    r = orc.bench_rsb_rank(rc, world, rank, cpu, reps, H.MPI_FLOAT, H.MPI_SUM)
    dist.barrier()
    worst = {k: allreduce_scalar(r[k] * scale, dist.ReduceOp.MAX, dev)
             for k in ('copy_in_s', 'combine_s', 'copy_out_s', 'total_s')}
    comb = r['combined_elements'] * scale
    return dict(
        value_s=worst['total_s'], unit='GB/s', cores=world, kind='port',
        cores_per_rank=1,
        sample='MPICH recursive-halving reduce-scatter-block host work per rank (copy in, the '
               'log2(P) MPIR_Reduce_local combines through oracle/redop_oracle.c, copy out) on '
               '%s fp32 per rank, one pinned core per rank, all %d ranks at once, median of %d '
               'calls per rank, max over ranks%s'
               % ('%d x %d' % (world, rc), world, reps,
                  '' if scale == 1 else '; 1/%d of the timed vector (host memory), times x %d'
                  % (scale, scale)),
        ms_per_call=round(worst['total_s'] * 1e3, 3),
        copy_in_ms=round(worst['copy_in_s'] * 1e3, 3),
        combine_ms=round(worst['combine_s'] * 1e3, 3),
        copy_out_ms=round(worst['copy_out_s'] * 1e3, 3),
        combined_elements_per_rank=comb,
        combine_GiBs_rank=round(3 * comb * 4 / GIB / (r['combine_s'] * scale), 3)
        if r['combine_s'] > 0 else None,
        scaled_down_by=scale, host_cpu=topo['model'], nproc=os.cpu_count(),
        affinity_cpus=len(topo['affinity']), physical_cores=len(phys), sockets=topo['sockets'],
        cgroup_cpu_quota=topo['cgroup_cpu_quota'],
        note='value = (P-1)/P x vector bytes / the slowest rank\'s host call time: the bus '
             'bandwidth MPICH\'s CPU schedule could not exceed even with a free network')


AB_VARIANTS = ('overlap_on_policy_on', 'overlap_off_policy_on', 'overlap_on_policy_off',
               'overlap_off_policy_off')


def defaults_ab(cc, step, recv, expected, dev, reps=3, rounds=2):
    """The value leg's two defaults that no earlier run could measure, timed
    against their alternatives on the same buffers, interleaved: the
    recursive-halving combine overlap (1 MiB half-steps and up, the RCCL
    communicators' default, vs off) x libmpix_redop's store policy (the
    default XCD write-through mask vs all non-temporal stores).  Every variant
    first runs one untimed call whose result must equal, bit for bit on every
    rank, `expected` -- the reference association regenerated on the device
    (rh_expected_block_device), not the shipped default's own output; then
    `reps` calls between barrier + synchronize, max
    over ranks.  `rounds` passes, the order rotated each pass; ms_per_step is
    the median over the passes.  The line's `value` stays on the shipped
    default; this only says whether the defaults gain or cost."""
    torch.cuda.synchronize()
    shipped_overlap = cc.rh_overlap()
    pol = redop.get_store_policy()
    pol_on = pol['xcd_mask'] if pol['xcd_mask'] > 0 else 0x88
    setting = {'overlap_on_policy_on': (1 << 20, pol_on), 'overlap_off_policy_on': (0, pol_on),
               'overlap_on_policy_off': (1 << 20, 0), 'overlap_off_policy_off': (0, 0)}
    times = {k: [] for k in AB_VARIANTS}
    parity = {}
    try:
        for rnd in range(rounds):
            order = AB_VARIANTS[rnd % 4:] + AB_VARIANTS[:rnd % 4]
            for name in order:
                ov, mask = setting[name]
                cc.set_rh_overlap(ov)
                redop.check(redop.set_store_policy(mask, 0, 0, 0), 'MPIX_Redop_set_store_policy')
                recv.fill_(float('nan'))
                step()
                torch.cuda.synchronize()
                if not bits_equal_all_ranks(recv, expected, dev):
                    raise ParityError('defaults A/B: %s differs from the reference association '
                                      'at the timed size on some rank' % name)
                parity[name] = True
                dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    step()
                torch.cuda.synchronize()
                dist.barrier()
                times[name].append(allreduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX,
                                                    dev) / reps)
    finally:
        cc.set_rh_overlap(shipped_overlap)
        redop.set_store_policy(-1 if os.environ.get('MPIX_REDOP_WT_XCD') is None
                               else pol['xcd_mask'], pol['every'], pol['phase'], pol['tail_blocks'])
    shipped = '%s_%s' % ('overlap_on' if shipped_overlap else 'overlap_off',
                         'policy_on' if pol['xcd_mask'] > 0 else 'policy_off')
    out = {k: dict(ms_per_step=round(1e3 * float(np.median(v)), 4),
                   ms_each_round=[round(1e3 * x, 4) for x in v],
                   bit_exact_vs_association_all_ranks=parity.get(k, False))
           for k, v in times.items()}
    best = min(AB_VARIANTS, key=lambda k: out[k]['ms_per_step'])
    out.update(shipped=shipped, fastest=best, reps=reps, rounds=rounds,
               overlap_bytes={'on': 1 << 20, 'off': 0}, store_policy_xcd_mask={'on': pol_on, 'off': 0},
               note='value leg calls, interleaved, order rotated per round; median over rounds')
    return out


def _no_shared(e):
    """a leg over symmetric memory when MPIX_Comm_alloc_shared found no
    verified mapping (MPI_ERR_OTHER on every rank, mpix_coll.h): reported,
    not timed, and the other legs go on"""
    return {'error': 'no symmetric memory (%s); leg not timed' % e, 'schedule_ran': None}


def rsb_secondary(args, world, rank, dev, out):
    """the other schedules on the same RCCL communicator: pairwise (all P-1
    links in one group + one multi-input combine), pipelined pairwise, the
    fused IPC pull; each parity-checked first (redscatblk3.c:43-56 closed
    form on device, every rank)"""
    from mpich_amd import ccl
    cc = _CCL['comm']
    total = (args.rsb_bytes // 4) // world * world
    recvcount = total // world
    send = torch.empty(total, dtype=torch.float32, device=dev)
    fill_uniform(send, 0x5EED0100 + rank)
    recv = torch.empty(recvcount, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    # full-size bit references: multipath must reproduce recursive halving's
    # bits, pipelined pairwise and pull those of pairwise (same association)
    redop.check(ccl.reduce_scatter_block(send, recv, recvcount, H.MPI_FLOAT, H.MPI_SUM, cc,
                                         'recursive_halving'), 'MPIX_Reduce_scatter_block')
    refs = {'recursive_halving': recv.clone()}
    same_as = {'recursive_halving_multipath': 'recursive_halving', 'pairwise_pipelined': 'pairwise',
               'pull': 'pairwise', 'recursive_halving_pull': 'recursive_halving',
               'recursive_halving_pull_shared': 'recursive_halving'}
    # the IPC pulls last: a platform that cannot map peer memory loses only them;
    # the last reads its input from symmetric memory (MPIX_Comm_alloc_shared)
    # in place, without the copy into the pull window
    legs = [(a, a, False) for a in ('recursive_halving_multipath', 'pairwise', 'pairwise_pipelined',
                                    'recursive_halving_pull', 'pull')]
    legs.append(('recursive_halving_pull_shared', 'recursive_halving_pull', True))
    shared = None
    for name, algo, on_shared in legs:
        progress(rank, 'reduce-scatter leg %s' % name)
        if on_shared and shared is None:
            try:        # collective: every rank gets the memory, or none does
                shared = cc.shared_tensor(total, torch.float32)
            except redop.RedopError as e:
                out[name] = _no_shared(e)
                continue
            shared.copy_(send)
            torch.cuda.synchronize()
        src = shared if on_shared else send
        rc_small = 4096 + 3
        blk = torch.cat([torch.full((rc_small,), rank + i, dtype=torch.int32, device=dev)
                         for i in range(world)])
        o = torch.empty(rc_small, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()        # inputs ready before the communicator's stream reads them
        redop.check(ccl.reduce_scatter_block(blk, o, rc_small, H.MPI_INT, H.MPI_SUM, cc, algo),
                    'MPIX_Reduce_scatter_block')
        sched = schedule_ran(cc, algo)
        if 'error' in sched:        # every rank agrees on a fallback: nobody times this leg
            out[name] = sched
            continue
        ok = allreduce_scalar(1 if bool(torch.all(o == world * rank + world * (world - 1) // 2))
                              else 0, dist.ReduceOp.MIN, dev)
        if not ok:
            raise ParityError('%s RSB fails the redscatblk3 closed form' % algo)

        def once():
            redop.check(ccl.reduce_scatter_block(src, recv, recvcount, H.MPI_FLOAT, H.MPI_SUM, cc,
                                                 algo), 'MPIX_Reduce_scatter_block')
        once()                          # at the timed size: the pull windows grow here
        sched = schedule_ran(cc, algo)
        if 'error' in sched:
            out[name] = sched
            continue
        bits = None
        if name == 'pairwise':
            refs['pairwise'] = recv.clone()
        elif name in same_as:
            same = bool(torch.equal(recv.view(torch.int32), refs[same_as[name]].view(torch.int32)))
            if not allreduce_scalar(1 if same else 0, dist.ReduceOp.MIN, dev):
                raise ParityError('%s RSB differs from %s at the timed size' % (name, same_as[name]))
            bits = same_as[name]
        reps = max(3, min(10, args.steps))
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            once()
        torch.cuda.synchronize()
        dist.barrier()
        t = allreduce_scalar((time.perf_counter() - t0) / reps, dist.ReduceOp.MAX, dev)
        if algo == 'recursive_halving_multipath':
            # every directed link of a rank carries 1/(P/2) of each step's half
            pof2 = 1
            while pof2 * 2 <= world:
                pof2 *= 2
            mp = pof2 >= 4 and pof2 == world
            link_bytes = (pof2 - 1) / pof2 * total * 4 / (world // 2 if mp else 1)
            links = world - 1 if mp else 1
        else:   # pairwise family and the pulls: one block per peer link, all links at once
            link_bytes = total * 4 / world
            links = world - 1
        cc.set_step_timing(True)        # one more call: rank 0's per-step device times
        once()
        torch.cuda.synchronize()
        cc.set_step_timing(False)
        steps = cc.step_times()
        sched = schedule_ran(cc, algo)      # the timed calls ran it too
        out[name] = dict(sched, parity_redscatblk3_all_ranks=True, ms=round(t * 1e3, 3),
                         bit_identical_to=bits, steps_rank0=steps,
                         busbw_GBs=round((world - 1) / world * total * 4 / t / 1e9, 2),
                         per_link_GBs=round(link_bytes / t / 1e9, 2), links_active=links,
                         frac_of_xgmi_link=round(link_bytes / t / 1e9 / XGMI_LINK_GBS, 4))
    if shared is not None:
        cc.free_shared(shared.data_ptr())
    del send, recv, refs, shared
    torch.cuda.empty_cache()


def allreduce_secondary(args, world, rank, dev, res):
    """MPI_Allreduce fp32 SUM, 1 GiB per rank: the reference's
    reduce-scatter + allgather schedule (libmpix_coll over RCCL point-to-point
    + the HIP combine, the reference association) next to RCCL's own
    all_reduce (ncclAllReduce, the reference's MPIR_Allreduce_intra_ccl route,
    rccl.c:223) as the comparator"""
    from mpich_amd import ccl
    cc = _CCL['comm']
    m = 100003          # allred.c sum_test_1 closed form (in = i, sol = i*P), on device
    x = torch.arange(m, dtype=torch.int32, device=dev)
    y = torch.empty_like(x)
    torch.cuda.synchronize()
    redop.check(ccl.allreduce(x, y, m, H.MPI_INT, H.MPI_SUM, cc, 'reduce_scatter_allgather'),
                'MPIX_Allreduce')
    if not allreduce_scalar(1 if bool(torch.all(y == x * world)) else 0, dist.ReduceOp.MIN, dev):
        raise ParityError('allreduce fails the allred.c sum_test_1 closed form')
    n = min(1 << 28, args.rsb_bytes // 4)          # 1 GiB per rank at the default size
    send = torch.empty(n, dtype=torch.float32, device=dev)
    fill_uniform(send, 0x5EED0200 + rank)
    recv = torch.empty_like(send)
    ws = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    res.update(parity_allred_sum_test_1_all_ranks=True, bytes_per_rank=n * 4, P=world)
    sh_in = sh_out = None
    asked = {'c_reduce_scatter_allgather': 'reduce_scatter_allgather',
             'c_rsag_multipath': 'rsag_multipath', 'c_pull': 'pull', 'c_pull_shared': 'pull'}
    for name, fn in (('c_reduce_scatter_allgather',
                      lambda: redop.check(ccl.allreduce(send, recv, n, H.MPI_FLOAT, H.MPI_SUM, cc,
                                                        'reduce_scatter_allgather', workspace=ws),
                                          'MPIX_Allreduce')),
                     ('c_rsag_multipath',
                      lambda: redop.check(ccl.allreduce(send, recv, n, H.MPI_FLOAT, H.MPI_SUM, cc,
                                                        'rsag_multipath', workspace=ws),
                                          'MPIX_Allreduce')),
                     ('rccl_all_reduce', lambda: (recv.copy_(send), dist.all_reduce(recv))),
                     ('c_pull',
                      lambda: redop.check(ccl.allreduce(send, recv, n, H.MPI_FLOAT, H.MPI_SUM, cc,
                                                        'pull'), 'MPIX_Allreduce')),
                     ('c_pull_shared',     # input and result in symmetric memory: no window copy
                      lambda: redop.check(ccl.allreduce(sh_in, sh_out, n, H.MPI_FLOAT, H.MPI_SUM,
                                                        cc, 'pull'), 'MPIX_Allreduce'))):
        if name == 'rccl_all_reduce' and dist.get_backend() != 'nccl':
            continue
        progress(rank, 'allreduce leg %s' % name)
        if name == 'c_pull_shared':
            try:
                sh_in = cc.shared_tensor(n, torch.float32)
                sh_out = cc.shared_tensor(n, torch.float32)
            except redop.RedopError as e:
                res[name] = _no_shared(e)
                continue
            sh_in.copy_(send)
            torch.cuda.synchronize()
        fn()
        sched = schedule_ran(cc, asked[name], 'ar') if name in asked else {}
        if 'error' in sched:
            res[name] = sched
            continue
        if name == 'c_reduce_scatter_allgather':
            ref = recv.clone()
        elif name in ('c_rsag_multipath', 'c_pull', 'c_pull_shared'):  # same association
            got = sh_out if name == 'c_pull_shared' else recv
            same = bool(torch.equal(got.view(torch.int32), ref.view(torch.int32)))
            if not allreduce_scalar(1 if same else 0, dist.ReduceOp.MIN, dev):
                raise ParityError('%s allreduce differs from reduce_scatter_allgather' % name)
            res['%s_bit_identical_all_ranks' % name[2:]] = True
        reps = max(3, min(10, args.steps))
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t = allreduce_scalar((time.perf_counter() - t0) / reps, dist.ReduceOp.MAX, dev)
        if name in asked:
            sched = schedule_ran(cc, asked[name], 'ar')
        res[name] = dict(sched, ms=round(t * 1e3, 3),
                         busbw_GBs=round(2 * (world - 1) / world * n * 4 / t / 1e9, 2))
    for t in (sh_in, sh_out):
        if t is not None:
            cc.free_shared(t.data_ptr())
    del send, recv, ws, ref, sh_in, sh_out
    torch.cuda.empty_cache()


_CCL = {}


class _Emitter:
    """prints rank 0's one JSON line exactly once, from whichever thread
    (main, or the watchdog) gets there first"""

    def __init__(self, rank, result):
        import threading
        self.rank, self.result, self.done = rank, result, False
        self.lock = threading.Lock()

    def emit(self, note=None):
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.rank != 0:
                return
            r = dict(self.result)
            if note:
                r['extras_watchdog'] = note
                r.setdefault('extras_error', 'secondary figures not finished: ' + note)
            print(json.dumps(r, default=str), flush=True)


def _watchdog(seconds, emit, note=True, code=0):
    """A hung collective.  Value leg (note=False, code 2): rank 0 prints the
    failed line as it stands and every rank exits non-zero.  Secondary legs
    (note=True): the value leg already passed its parity gate and was timed,
    so rank 0 prints the line with the headline and the hang recorded
    (`extras_watchdog`, `extras_error`), and every rank leaves with `code`
    (0: the N-rank value stands; the secondary figures are extras)"""
    import threading

    def fire():
        emit.emit('secondary collectives exceeded %.0f s; headline kept, rank exits' % seconds
                  if note else None)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def run_secondary(result, legs):
    """Run the secondary legs ((key, fn(part)) pairs) in order into
    result[key], stopping at the first that raises (the peers may be stuck
    in that leg: no further collective).  Returns (failure or None, exit
    code): an exception or timing trouble in an extra keeps the checked
    value and exits 0 (`extras_error`); a ParityError -- a wrong result is
    never an extra -- also sets the top-level `error` and exits
    EXIT_PARITY."""
    for key, fn in legs:
        part = result[key] = {}
        try:
            fn(part)
        except Exception as e:
            part['error'] = '%s: %s' % (type(e).__name__, e)
            failed = '%s: %s' % (key, part['error'])
            result['extras_error'] = failed
            if isinstance(e, ParityError):
                result['error'] = 'secondary leg failed its parity check: ' + failed
                return failed, EXIT_PARITY
            return failed, 0
    return None, 0


def world_plan(args, env=None):
    """Who runs the ranks, decided before anything touches a GPU.

    Returns ('single', 1), ('launch', N) -- this process starts the N ranks
    itself -- or ('rank', N) under an external launcher (torchrun sets
    WORLD_SIZE); raises SystemExit with the reason when --gpus and the
    environment disagree, so an N-GPU request never yields a 1-GPU line."""
    env = os.environ if env is None else env
    ws = env.get('WORLD_SIZE')
    if ws is not None:
        world = int(ws)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%d (launcher and request '
                             'disagree)' % (args.gpus, world))
        return ('rank', world) if world > 1 else ('single', 1)
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit('bench.py: --gpus must be >= 1')
    return ('launch', n) if n > 1 else ('single', 1)


def count_devices(env=None):
    """GPUs the ranks will see, counted in a short-lived child process: the
    launcher parent must stay off the GPU (it starts the ranks with
    subprocess, and a process that initialised HIP must not be the one that
    outlives them), and torch.cuda.device_count() may initialise the HIP
    runtime -- it does whenever amdsmi cannot enumerate and it falls back to
    hipGetDeviceCount.  The child inherits `env`, so HIP_VISIBLE_DEVICES and
    its relatives count as they will in the ranks.  0 if the child fails."""
    import subprocess
    env = os.environ if env is None else env
    try:
        p = subprocess.run([sys.executable, '-c', 'import torch; print(torch.cuda.device_count())'],
                           env=dict(env), capture_output=True, text=True, timeout=300)
        return int(p.stdout.strip().splitlines()[-1]) if p.returncode == 0 else 0
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return 0


def check_devices(world, env=None, launcher=True):
    """one GPU per rank, unless the 1-GPU rehearsal knob shares device 0 (or
    the dry run touches none).  The launcher counts through count_devices, so
    it never initialises HIP (tests/test_launcher_gpu.py checks that on a
    GPU); a rank under an external launcher is about to use its GPU anyway"""
    env = os.environ if env is None else env
    if env.get('MPIX_BENCH_SAME_DEVICE') == '1':
        return
    have = count_devices(env) if launcher else torch.cuda.device_count()
    if have < world:
        raise SystemExit('bench.py: %d ranks need %d GPUs, this node shows %d' % (world, world, have))


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Start N fresh rank processes of this script (subprocess, never exec:
    this process has not touched the GPU and stays off it), one per GPU, with
    the RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* rendezvous torchrun would give
    them -- the in-library bootstrap of the reference (rccl.c:33-43: unique id
    on rank 0, broadcast, ncclCommInitRank) then runs inside the ranks through
    torch.distributed.  Rank 0's stdout is relayed line by line; the run fails
    (non-zero) if any rank does, the others are then stopped, and it also
    fails unless rank 0 printed exactly one JSON line with n_gpus == N."""
    import signal
    import subprocess
    port = os.environ.get('MASTER_PORT') or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK='0', MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=port, MPIX_BENCH_LAUNCHED='1')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.abspath(__file__)] + argv,
                                      env=env, stdout=subprocess.PIPE if r == 0 else None))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = {s: signal.signal(s, lambda sig, frm: (stop(), sys.exit(128 + sig)))
           for s in (signal.SIGTERM, signal.SIGINT)}
    lines = []
    import threading

    def relay():
        for raw in procs[0].stdout:
            line = raw.decode(errors='replace')
            sys.stdout.write(line)
            sys.stdout.flush()
            if line.lstrip().startswith('{'):
                lines.append(line)
    t = threading.Thread(target=relay, daemon=True)
    t.start()
    rc, failed = 0, None
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and failed is None:
                failed, rc = procs.index(p), c
                stop()      # a peer stuck in a collective with the failed rank
        if live:
            time.sleep(0.2)
    t.join(timeout=10)
    for s, h in old.items():
        signal.signal(s, h)
    if failed is not None:
        sys.stderr.write('bench.py: rank %d exited with status %d\n' % (failed, rc))
        return rc if rc > 0 else 1
    try:
        got = json.loads(lines[-1]) if len(lines) == 1 else None
    except ValueError:
        got = None
    if not got or got.get('n_gpus') != n:
        sys.stderr.write('bench.py: rank 0 printed %d JSON line(s), none an n_gpus=%d line\n'
                         % (len(lines), n))
        return 1
    return 0


def dry_run(world, rank, args=None):
    """the launch path without a GPU: ranks rendezvous over gloo, count
    themselves with an all-reduce, run the N > 1 line's CPU baseline (the
    reference schedule's host work, unless --no-cpu-baseline) and rank 0
    prints the line's skeleton"""
    seen = 1
    cpu = None
    if world > 1:
        dist.init_process_group('gloo')
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.barrier()
        if args is not None and not args.no_cpu_baseline:
            total = (args.rsb_bytes // 4) // world * world
            cpu = rsb_cpu_baseline(world, rank, total // world, None)
            cpu = dict(value=round((world - 1) / world * total * 4 / cpu.pop('value_s') / 1e9, 3),
                       **cpu)
    if rank == 0:
        line = {'metric': METRIC_RSB if world > 1 else METRIC, 'value': None,
                'n_gpus': world, 'ranks_seen': seen, 'dry_run': True,
                'defaults_ab': ({k: None for k in AB_VARIANTS} if world > 1 else None),
                'launcher': 'bench.py' if os.environ.get('MPIX_BENCH_LAUNCHED')
                else ('external' if world > 1 else None)}
        if world > 1:
            line['parity'] = {'full_size_bit_exact_all_ranks': None}
            line['cpu_baseline'] = cpu
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if seen == world else 1


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    mode, world = world_plan(args)
    if not args.dry_run and world > 1:
        check_devices(world, launcher=mode == 'launch')
    if mode == 'launch':
        return launch_ranks(world, argv)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.dry_run:
        return dry_run(world, rank, args)
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on
    # device 0 and a gloo control plane + transport; RCCL refuses two ranks on
    # one device (profiles/r01_rccl_probe.txt)
    if os.environ.get('MPIX_BENCH_SAME_DEVICE') == '1':
        local = 0
    backend = os.environ.get('MPIX_BENCH_BACKEND', 'nccl')
    if world > 1:
        torch.cuda.set_device(local)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    assert redop.lib().MPIX_Redop_init() == 0
    if world == 1:
        single_gpu(args, dev)
        return 0
    # a hung value leg (communicator bootstrap, a collective that never
    # completes) still ends the run with rank 0's error line and a non-zero status
    failed_line = {'metric': METRIC_RSB, 'value': None, 'unit': 'GB/s', 'n_gpus': world}
    first = _Emitter(rank, dict(failed_line, error='value leg (reduce-scatter over RCCL) did not '
                                                   'finish within %.0f s' % args.value_timeout))
    dog0 = _watchdog(args.value_timeout, first, note=False, code=2)
    try:
        result = multi_gpu(args, world, rank, dev)
    except Exception as e:      # the value leg failed: say so at the top level, exit non-zero
        first.result = dict(failed_line, error='%s: %s' % (type(e).__name__, e))
        first.emit()
        sys.stdout.flush()
        os._exit(EXIT_PARITY if isinstance(e, ParityError) else 1)
    dog0.cancel()
    with first.lock:            # the watchdog fired meanwhile: its line stands
        if first.done:
            return 2
        first.done = True
    emit = _Emitter(rank, result)
    dog = _watchdog(args.extras_timeout, emit)
    result['extras_timeout_s'] = args.extras_timeout
    failed, code = (None, 0) if args.no_extras else run_secondary(
        result, ((k, lambda part, fn=fn: fn(args, world, rank, dev, part))
                 for k, fn in (('reduce_scatter_block_other', rsb_secondary),
                               ('allreduce', allreduce_secondary))))
    emit.emit()
    if failed:
        sys.stdout.flush()
        sys.stderr.write('bench.py: secondary leg failed: %s\n' % failed)
        sys.stderr.flush()
        os._exit(code)
    dist.barrier()
    if dist.get_backend() == 'nccl':
        _CCL.pop('comm').free()
    else:
        from mpich_amd import coll
        coll.free_comms()
    dist.destroy_process_group()
    dog.cancel()
    return 0


if __name__ == '__main__':
    sys.exit(main())
