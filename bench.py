#!/usr/bin/env python3
"""Benchmark: device-resident MPI_Reduce_local (fp32 SUM, 1 GiB) on MI355X.

BASELINE.json metric "GiB/s device-resident MPI_Reduce_local (fp32 SUM,
1 GiB) vs HBM roofline", on configs[1]: count = 2^28 MPI_FLOAT per operand,
both operands resident in HBM before the timed region.  One step = one
MPIX_Reduce_local call (the synchronous MPIR_Reduce_local drop-in) over the
whole buffer; GiB/s = algorithmic bytes 3 * count * 4 (read in, read inout,
write inout) / wall time.

N > 1 (torchrun, one rank per GPU): every rank reduces its own 1 GiB shard
(no data-path collective: the path is element-wise), value = all ranks'
bytes / max-over-ranks time ("weak" scaling).  Those runs also time the
MPI_Reduce_scatter_block schedules (BASELINE config 4: recursive halving
with a per-step breakdown, pairwise, fused IPC pull) and the allreduce as
secondary figures.

Also reported (not `value`): kernel-only rate from HIP events on the launch
stream -> `roofline`; a measured STREAM triad on the same GPU; the
host-resident end-to-end rate (pinned host operands, the kernel reads and
writes them over PCIe); and the `cpu_baseline` -- the oracle (clean-room C
restatement of MPICH's op loop) timed on this host's cores on a bounded
sample of the same 1 GiB workload, plus BASELINE config 1 (16 MiB) beside it.
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
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=50)
    p.add_argument('--warmup', type=int, default=5)
    p.add_argument('--count', type=int, default=1 << 28, help='fp32 elements per operand')
    p.add_argument('--cpu-seconds', type=float, default=20.0,
                   help='bounded CPU-baseline sample duration per leg')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-extras', action='store_true',
                   help='skip triad / end-to-end / sweep side measurements')
    p.add_argument('--sweep', action='store_true', help='config 2 chunk/size sweep')
    p.add_argument('--rsb', action='store_true', help='time reduce_scatter_block even at N=1')
    p.add_argument('--rsb-bytes', type=int, default=4 << 30, help='RSB vector bytes per rank')
    p.add_argument('--extras-timeout', type=float, default=300.0,
                   help='watchdog (s) over the N>1 collective figures and teardown')
    p.add_argument('--pmc', default=os.path.join(ROOT, 'profiles', 'r01_pmc_summary.json'),
                   help='PMC traffic summary (from tools/pmc_summary.py) to quote as traffic')
    return p.parse_args()


def bench_lib():
    path = os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so')
    L = ctypes.CDLL(path)
    L.mpix_bench_triad.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p]
    L.mpix_bench_call_latency.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double)]
    L.mpix_bench_chunked_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]
    return L


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
            out.append(dict(chunk_bytes=ck, error=rc))
            continue
        out.append(dict(chunk_bytes=ck, calls=nch, GiBs=round(3 * nch * ck / total.value / GIB, 1),
                        us_per_call=round(1e6 * total.value / nch, 2),
                        issue_us_per_call=round(1e6 * issue.value / nch, 2)))
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
        out.append(dict(count=n, median_us=round(med.value, 2), p90_us=round(p90.value, 2),
                        checked=ok))
    return out


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


def cpu_baseline(seconds, count):
    """The oracle (clean-room C restatement of MPICH's op_fns.c loop) on a
    bounded sample of the SAME workload: MPI_Reduce_local(MPI_SUM, MPI_FLOAT)
    on `count`-element (1 GiB) host operands, repeated for ~seconds/2 on one
    core (MPICH's path is one thread per rank) and ~seconds/2 on all cores
    of this process's share.  BASELINE config 1 (16 MiB, cache-resident on
    this host) is reported beside it."""
    import numpy as np
    from oracle import oracle as orc
    orc.build()
    ncores = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else os.cpu_count()
    threads_all = max(1, min(16, ncores))

    def leg(n, nth, budget):
        rng = np.random.default_rng(0x5EED0001)
        a = rng.uniform(-1, 1, n).astype(np.float32)
        b = rng.uniform(-1, 1, n).astype(np.float32)
        t_list = []
        t_end = time.perf_counter() + budget
        while time.perf_counter() < t_end or len(t_list) < 3:
            t0 = orc.wtime()
            orc.reduce_local(b, a, n, H.MPI_FLOAT, H.MPI_SUM, nthreads=nth)
            t_list.append(orc.wtime() - t0)
        t_list.sort()
        med = t_list[len(t_list) // 2]
        return dict(gibs=round(3 * n * 4 / GIB / med, 3), best=round(3 * n * 4 / GIB / t_list[0], 3),
                    reps=len(t_list), threads=nth)

    one = leg(count, 1, seconds * 0.45)
    allc = leg(count, threads_all, seconds * 0.35)
    c1 = leg(4194304, 1, seconds * 0.2)
    model = ''
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                model = line.split(':', 1)[1].strip()
                break
    except OSError:
        pass
    return dict(
        value=one['gibs'], unit='GiB/s', cores=1, kind='port',
        sample='same workload (MPI_Reduce_local MPI_SUM MPI_FLOAT, %d elements = %d MiB per '
               'operand, host-resident) through oracle/redop_oracle.c, 1 thread, %d calls, median'
               % (count, count * 4 >> 20, one['reps']),
        best=one['best'],
        allcores=dict(value=allc['gibs'], threads=threads_all, reps=allc['reps'],
                      note='disjoint slices, one thread per core of this process share'),
        config1_16MiB_1core=dict(value=c1['gibs'], reps=c1['reps'],
                                 note='BASELINE config 1; 48 MiB per call is cache-resident on '
                                      'this host'),
        host_cpu=model, nproc=os.cpu_count(), affinity_cpus=ncores)


def load_pmc(path, count):
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    k = d.get('kernels', {}).get('reduce_local_fp32_sum')
    if not k or k.get('count') != count:
        return None
    return k.get('hbm_bytes_per_launch')


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # rehearsal knobs for a 1-GPU box (not used by the driver): every rank on
    # device 0 and a gloo control plane; RCCL-transport figures then error out
    # (caught) and only the flow, the replicas and the IPC pull are exercised
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

    n = args.count
    nbytes_alg = 3 * n * 4
    inout = torch.empty(n, dtype=torch.float32, device=dev)
    inb = torch.empty(n, dtype=torch.float32, device=dev)
    fill_uniform(inout, 0x5EED0001 + 2 * rank)
    fill_uniform(inb, 0x5EED0002 + 2 * rank)
    torch.cuda.synchronize()

    def step():
        redop.check(redop.MPI_Reduce_local(inb, inout, n, H.MPI_FLOAT, H.MPI_SUM))

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    if world > 1:
        t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
    ms_per_step = 1e3 * t / args.steps
    value = world * nbytes_alg * args.steps / t / GIB

    # kernel-only: the same launch, async on torch's stream, timed by events
    stream = torch.cuda.current_stream()
    kreps = max(10, min(args.steps, 50))
    k_avg, k_med, k_min = event_time_per_launch(
        lambda: redop.check(redop.reduce_local_async(inb, inout, n, H.MPI_FLOAT, H.MPI_SUM,
                                                     stream)), kreps, stream)
    achieved = nbytes_alg / (k_avg * 1e-3) / 1e9
    result = {
        'metric': METRIC,
        'value': round(value, 2),
        'unit': 'GiB/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_per_step, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic (uniform [-1,1), seeded per rank)',
        'config': {
            'workload': 'MPI_Reduce_local(MPI_SUM, MPI_FLOAT) device-resident, BASELINE configs[1] '
                        'at its 1 GiB point',
            'count': n, 'bytes_per_operand': 4 * n, 'algorithmic_bytes_per_step': nbytes_alg,
            'parallelism': 'replicas' if world == 1 else 'dp%d shards (no collective)' % world,
            'launch': redop.get_launch(),
        },
        'roofline': {
            'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBS, 4),
            'traffic': load_pmc(args.pmc, n),
            'kernel_ms_avg': round(k_avg, 4), 'kernel_ms_median_batch': round(k_med, 4),
            'kernel_ms_min_batch': round(k_min, 4), 'kernel_launches_timed': 3 * kreps,
            'algorithmic_bytes_per_launch': nbytes_alg,
        },
    }

    if not args.no_extras and rank == 0:
        # STREAM triad on the same GPU (three separate 1 GiB fp32 arrays)
        try:
            B = bench_lib()
            a3 = torch.empty(n, dtype=torch.float32, device=dev)
            tri_avg, tri_med, _ = event_time_per_launch(
                lambda: B.mpix_bench_triad(a3.data_ptr(), inb.data_ptr(), inout.data_ptr(),
                                           ctypes.c_float(0.5), n, stream.cuda_stream),
                kreps, stream)
            triad = nbytes_alg / (tri_avg * 1e-3) / 1e9
            result['roofline']['triad_measured_GBs'] = round(triad, 1)
            result['roofline']['frac_of_triad'] = round(achieved / triad, 4)
            del a3
            # small-message regime of the same entry point: per-call latency
            try:
                result['sync_call_latency'] = sync_call_latency(B, dev)
            except Exception as e:      # secondary figure: never lose the headline line
                result['sync_call_latency'] = dict(error='%s: %s' % (type(e).__name__, e))
            try:
                result['chunked_async_c'] = chunked_async_c(
                    B, inb, inout, n, stream,
                    (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20) if args.sweep
                    else (64 << 10, 1 << 20, 16 << 20))
            except Exception as e:      # secondary figure
                result['chunked_async_c'] = dict(error='%s: %s' % (type(e).__name__, e))
        except OSError as e:
            result['roofline']['triad_measured_GBs'] = None
            result['roofline']['triad_error'] = str(e)
        # host-resident end-to-end: pinned host in/inout -> MPIX_Reduce_local
        # stages H2D + kernel + D2H (3 x 1 GiB over PCIe)
        hn = n
        hin = torch.empty(hn, dtype=torch.float32).pin_memory()
        hio = torch.empty(hn, dtype=torch.float32).pin_memory()
        hin.uniform_(-1, 1)
        hio.uniform_(-1, 1)
        redop.check(redop.MPI_Reduce_local(hin, hio, hn, H.MPI_FLOAT, H.MPI_SUM))
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            redop.check(redop.MPI_Reduce_local(hin, hio, hn, H.MPI_FLOAT, H.MPI_SUM))
        te = (time.perf_counter() - t0) / reps
        result['end_to_end_host'] = dict(gibs=round(3 * hn * 4 / GIB / te, 2),
                                         ms_per_call=round(te * 1e3, 2),
                                         note='pinned host buffers: the kernel reads and writes '
                                              'them over PCIe (zero-copy); never `value`')
        del hin, hio
        # the same from pageable (numpy) buffers: host workers feeding pinned
        # slots (the default above 256 MiB), and the hipMemcpyAsync staging
        try:
            pin_ = np.random.default_rng(0x5EED0007 + rank).random(hn, dtype=np.float32)
            pio_ = np.random.default_rng(0x5EED0008 + rank).random(hn, dtype=np.float32)
            prev = redop.get_pageable()
            pg = {}
            for label, threads in (('workers', prev['threads'] or 8), ('staged', 0)):
                redop.check(redop.set_pageable(threads, prev['chunk_bytes']))
                redop.check(redop.MPI_Reduce_local(pin_, pio_, hn, H.MPI_FLOAT, H.MPI_SUM))
                t0 = time.perf_counter()
                for _ in range(reps):
                    redop.check(redop.MPI_Reduce_local(pin_, pio_, hn, H.MPI_FLOAT, H.MPI_SUM))
                tp = (time.perf_counter() - t0) / reps
                pg[label] = dict(gibs=round(3 * hn * 4 / GIB / tp, 2), ms_per_call=round(tp * 1e3, 2))
            redop.check(redop.set_pageable(prev['threads'], prev['chunk_bytes']))
            pg['workers_x_chunk'] = '%d x %d MiB' % (prev['threads'] or 8, prev['chunk_bytes'] >> 20)
            pg['note'] = 'pageable (numpy) host buffers; never `value`'
            result['end_to_end_pageable'] = pg
            del pin_, pio_
        except Exception as e:      # secondary figure
            result['end_to_end_pageable'] = dict(error='%s: %s' % (type(e).__name__, e))

    if args.sweep and rank == 0:
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
        chunks = []
        for ck in (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30):
            m = ck // 4
            nch = n // m
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            for k in range(nch):
                redop.check(redop.reduce_local_async(inb[k * m:], inout[k * m:], m, H.MPI_FLOAT,
                                                     H.MPI_SUM, stream))
            torch.cuda.synchronize()
            tt = time.perf_counter() - t0
            chunks.append(dict(chunk_bytes=ck, calls=nch, GiBs=round(nbytes_alg / tt / GIB, 1)))
        # the same chunked sweep replayed from a HIP graph (torch.cuda.graph):
        # the launch-bound small chunks lose the per-call host launch cost
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
        result['sweep'] = dict(size_kernel=sweep, chunked_1gib_async=chunks,
                               chunked_hipgraph_replay=graphed)

    del inout, inb
    torch.cuda.empty_cache()

    # The headline is complete here.  Everything after it (collective
    # figures, teardown) runs under a watchdog: if a secondary collective
    # hangs on some rank, rank 0 still prints the line (with what it has)
    # and every rank leaves, instead of the job dying silently at the
    # driver's limit.
    emit = _Emitter(rank, result)
    dog = None
    if world > 1 or args.rsb:
        dog = _watchdog(args.extras_timeout, emit)
        result['extras_timeout_s'] = args.extras_timeout
        if os.environ.get('MPIX_BENCH_STALL_RANK') == str(rank):
            time.sleep(1e6)     # rehearsal knob: a rank that never arrives
        # filled in place, so a watchdog line carries the figures already taken
        for key, fn in (('reduce_scatter_block', rsb_bench), ('allreduce', allreduce_bench)):
            part = result[key] = {}
            try:
                fn(args, world, rank, dev, part)
            except Exception as e:  # secondary figure: never lose the headline line
                part['error'] = '%s: %s' % (type(e).__name__, e)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result['cpu_baseline'] = cpu_baseline(args.cpu_seconds, args.count)
    emit.emit()
    if world > 1:
        try:
            dist.barrier()
            if _CCL.get('comm') is not None:
                _CCL.pop('comm').free()
            dist.destroy_process_group()
        except Exception as e:  # a peer already left (its error is in the line)
            print('teardown: %s: %s' % (type(e).__name__, e), file=sys.stderr, flush=True)
    if dog is not None:
        dog.cancel()


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
                for k in ('reduce_scatter_block', 'allreduce'):
                    part = dict(r.get(k) or {})
                    part.setdefault('error', 'not finished: ' + note)
                    r[k] = part
            print(json.dumps(r, default=str), flush=True)


def _watchdog(seconds, emit):
    import threading

    def fire():
        emit.emit('secondary collectives exceeded %.0f s; headline kept, rank exits' % seconds)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def rsb_bench(args, world, rank, dev, out):
    """BASELINE config 4: MPI_Reduce_scatter_block fp32 SUM, fixed vector per
    rank (strong scaling): the reference's recursive-halving schedule and
    the pairwise one over RCCL/xGMI (all links at once), and the fused
    pull + combine kernel over hipIpc-mapped peer buffers."""
    from mpich_amd import coll
    if world == 1 or not dist.is_initialized():
        out['note'] = 'P=1 is a local copy (coll_api.txt:402-411); see value for the combine'
        return out
    total = args.rsb_bytes // 4
    recvcount = total // world
    total = recvcount * world
    send = torch.empty(total, dtype=torch.float32, device=dev)
    fill_uniform(send, 0x5EED0100 + rank)
    recv = torch.empty(recvcount, dtype=torch.float32, device=dev)
    ws = (torch.empty(total * 4, dtype=torch.uint8, device=dev),
          torch.empty(total * 4, dtype=torch.uint8, device=dev))
    pof2 = 1
    while pof2 * 2 <= world:
        pof2 *= 2
    p2p_ok = dist.get_backend() == 'nccl'     # the gloo rehearsal cannot move device tensors
    for algo in ('recursive_halving', 'pairwise', 'pull'):
        if algo != 'pull' and not p2p_ok:
            out[algo] = dict(skipped='needs the nccl (RCCL) backend')
            continue
        try:
            fn = coll.ALGORITHMS[algo]
            kw = dict(extent=4)
            if algo != 'pull':
                kw['workspace'] = ws if algo == 'recursive_halving' else ws[0]
            # parity first: redscatblk3.c:43-56 closed form (MPI_INT SUM), on device
            rc_small = 4096 + 3
            blk = torch.cat([torch.full((rc_small,), rank + i, dtype=torch.int32, device=dev)
                             for i in range(world)])
            o = torch.empty(rc_small, dtype=torch.int32, device=dev)
            fn(blk, o, rc_small, H.MPI_INT, H.MPI_SUM, extent=4)
            torch.cuda.synchronize()
            ok = allreduce_scalar(1 if bool(torch.all(o == world * rank + world * (world - 1) // 2))
                                  else 0, dist.ReduceOp.MIN, dev)

            def once():
                fn(send, recv, recvcount, H.MPI_FLOAT, H.MPI_SUM, **kw)
            once()
            reps = max(3, min(10, args.steps))
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            torch.cuda.synchronize()
            dist.barrier()
            t = (time.perf_counter() - t0) / reps
            t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
            busbytes = (world - 1) / world * total * 4
            if algo == 'recursive_halving':
                # bytes a rank receives over its one active link across the steps
                link_bytes = (pof2 - 1) / pof2 * total * 4
                links = 1
            else:                                       # pairwise / pull: all links at once
                link_bytes = total * 4 / world          # one block per peer link
                links = world - 1
            out[algo] = dict(parity_redscatblk3_all_ranks=bool(ok), ms=round(t * 1e3, 3),
                             busbw_GBs=round(busbytes / t / 1e9, 2),
                             per_link_GBs=round(link_bytes / t / 1e9, 2), links_active=links,
                             frac_of_xgmi_link=round(link_bytes / t / 1e9 / 153.0, 4))
            if algo == 'recursive_halving':
                # per-step breakdown, rank 0's stream
                tl = []
                dist.barrier()
                fn(send, recv, recvcount, H.MPI_FLOAT, H.MPI_SUM, timer=tl, **kw)
                torch.cuda.synchronize()
                out[algo]['steps_rank0'] = tl[0].result()

        except Exception as e:          # keep the other algorithms' figures
            out[algo] = dict(error='%s: %s' % (type(e).__name__, e))
    del ws
    torch.cuda.empty_cache()
    # the same schedules as C++ host code (libmpix_coll.so) on their own RCCL
    # communicator: no Python between the steps
    cc = ccl_comm() if p2p_ok else None
    for algo in ('recursive_halving', 'pairwise', 'pairwise_pipelined'):
        key = 'c_' + algo
        if cc is None:
            out[key] = dict(skipped='no RCCL communicator (%s)' % _CCL.get('error', 'gloo'))
            continue
        try:
            from mpich_amd import ccl
            rc_small = 4096 + 3
            blk = torch.cat([torch.full((rc_small,), rank + i, dtype=torch.int32, device=dev)
                             for i in range(world)])
            o = torch.empty(rc_small, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            redop.check(ccl.reduce_scatter_block(blk, o, rc_small, H.MPI_INT, H.MPI_SUM, cc, algo),
                        'MPIX_Reduce_scatter_block')
            ok = allreduce_scalar(1 if bool(torch.all(o == world * rank + world * (world - 1) // 2))
                                  else 0, dist.ReduceOp.MIN, dev)

            def once():
                redop.check(ccl.reduce_scatter_block(send, recv, recvcount, H.MPI_FLOAT, H.MPI_SUM,
                                                     cc, algo), 'MPIX_Reduce_scatter_block')
            once()
            reps = max(3, min(10, args.steps))
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            torch.cuda.synchronize()
            dist.barrier()
            t = (time.perf_counter() - t0) / reps
            t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
            busbytes = (world - 1) / world * total * 4
            if algo == 'recursive_halving':
                link_bytes, links = (pof2 - 1) / pof2 * total * 4, 1
            else:
                link_bytes, links = total * 4 / world, world - 1
            out[key] = dict(parity_redscatblk3_all_ranks=bool(ok), ms=round(t * 1e3, 3),
                            busbw_GBs=round(busbytes / t / 1e9, 2),
                            per_link_GBs=round(link_bytes / t / 1e9, 2), links_active=links,
                            frac_of_xgmi_link=round(link_bytes / t / 1e9 / 153.0, 4))
        except Exception as e:
            out[key] = dict(error='%s: %s' % (type(e).__name__, e))
    del send, recv
    torch.cuda.empty_cache()
    out.update(P=world, bytes_per_rank=total * 4, recvcount=recvcount,
               xgmi_link_GBs_assumed=153.0)
    return out


_CCL = {}


def ccl_comm():
    """one libmpix_coll RCCL communicator per process (MPIR_RCCLcomm_init,
    rccl.c:21-52: rank 0's unique id broadcast over the process group).
    Every rank always reaches the collective init, so a failure cannot leave
    the others waiting in ncclCommInitRank."""
    if 'comm' not in _CCL and 'error' not in _CCL:
        try:
            from mpich_amd import ccl
            _CCL['comm'] = ccl.comm_create_ccl_from_process_group()
        except Exception as e:
            _CCL['error'] = '%s: %s' % (type(e).__name__, e)
    return _CCL.get('comm')


def allreduce_bench(args, world, rank, dev, res):
    """MPI_Allreduce fp32 SUM, 1 GiB per rank: the reference's
    reduce-scatter + allgather schedule on RCCL point-to-point + the HIP
    combine (bit-identical to the reference association), next to RCCL's own
    all_reduce (torch.distributed, ncclAllReduce -- the reference's
    MPIR_Allreduce_intra_ccl route, rccl.c:223) as the comparator."""
    from mpich_amd import coll
    if world == 1 or not dist.is_initialized():
        res['note'] = 'P=1 is a local copy'
        return res
    if dist.get_backend() != 'nccl':
        res['skipped'] = 'needs the nccl (RCCL) backend'
        return res
    # parity: allred.c sum_test_1 closed form (in = i, sol = i*P), on device
    m = 100003
    x = torch.arange(m, dtype=torch.int32, device=dev)
    y = torch.empty_like(x)
    coll.allreduce(x, y, m, H.MPI_INT, H.MPI_SUM, extent=4)
    torch.cuda.synchronize()
    ok = allreduce_scalar(1 if bool(torch.all(y == x * world)) else 0, dist.ReduceOp.MIN, dev)
    n = (1 << 30) // 4
    send = torch.empty(n, dtype=torch.float32, device=dev)
    fill_uniform(send, 0x5EED0200 + rank)
    recv = torch.empty_like(send)
    ws = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    res.update(parity_allred_sum_test_1_all_ranks=bool(ok), bytes_per_rank=n * 4, P=world)
    for name, fn in (('mpich_schedule_hip_combine',
                      lambda: coll.allreduce(send, recv, n, H.MPI_FLOAT, H.MPI_SUM, extent=4,
                                             workspace=ws)),
                     ('mpich_schedule_rd_allgather',
                      lambda: coll.allreduce(send, recv, n, H.MPI_FLOAT, H.MPI_SUM, extent=4,
                                             workspace=ws, allgather='recursive_doubling')),
                     ('rccl_all_reduce', lambda: (recv.copy_(send), dist.all_reduce(recv)))):
        fn()
        reps = max(3, min(10, args.steps))
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t = (time.perf_counter() - t0) / reps
        t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
        res[name] = dict(ms=round(t * 1e3, 3),
                         busbw_GBs=round(2 * (world - 1) / world * n * 4 / t / 1e9, 2))
    cc = ccl_comm()
    if cc is None:
        res['c_reduce_scatter_allgather'] = dict(skipped=_CCL.get('error', 'no communicator'))
    else:
        from mpich_amd import ccl

        def c_ar():
            redop.check(ccl.allreduce(send, recv, n, H.MPI_FLOAT, H.MPI_SUM, cc,
                                      'reduce_scatter_allgather', workspace=ws), 'MPIX_Allreduce')
        try:
            c_ar()
            reps = max(3, min(10, args.steps))
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                c_ar()
            torch.cuda.synchronize()
            dist.barrier()
            t = (time.perf_counter() - t0) / reps
            t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
            res['c_reduce_scatter_allgather'] = dict(
                ms=round(t * 1e3, 3), busbw_GBs=round(2 * (world - 1) / world * n * 4 / t / 1e9, 2))
        except Exception as e:
            res['c_reduce_scatter_allgather'] = dict(error='%s: %s' % (type(e).__name__, e))
        # MPI_Reduce to rank 0 (reduce_scatter_gather, libmpix_coll over RCCL):
        # reduce.c KAT first (in[i] = i on every rank, i*P at the root)
        try:
            m = 100003
            x = torch.arange(m, dtype=torch.int32, device=dev)
            y = torch.full_like(x, -1)
            redop.check(ccl.reduce(x, y if rank == 0 else None, m, H.MPI_INT, H.MPI_SUM, 0, cc,
                                   'reduce_scatter_gather'), 'MPIX_Reduce')
            torch.cuda.synchronize()
            ok = allreduce_scalar(1 if rank != 0 or bool(torch.all(y == x * world)) else 0,
                                  dist.ReduceOp.MIN, dev)

            def c_red():
                redop.check(ccl.reduce(send, recv if rank == 0 else None, n, H.MPI_FLOAT,
                                       H.MPI_SUM, 0, cc, 'reduce_scatter_gather'), 'MPIX_Reduce')
            c_red()
            reps = max(3, min(10, args.steps))
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                c_red()
            torch.cuda.synchronize()
            dist.barrier()
            t = (time.perf_counter() - t0) / reps
            t = allreduce_scalar(t, dist.ReduceOp.MAX, dev)
            res['c_reduce_to_root0'] = dict(
                parity_reduce_c_all_ranks=bool(ok), ms=round(t * 1e3, 3),
                busbw_GBs=round(n * 4 / t / 1e9, 2),   # nccl-tests: reduce busbw = algbw
                algorithm='reduce_scatter_gather')
        except Exception as e:
            res['c_reduce_to_root0'] = dict(error='%s: %s' % (type(e).__name__, e))
    del send, recv, ws
    torch.cuda.empty_cache()
    return res


if __name__ == '__main__':
    main()
