#!/usr/bin/env python3
"""Where a synchronous 1 GiB MPIX_Reduce_local call spends the time beyond its
kernel (~16 us per call over the kernel, against 8.8 us
for a 1-element call).

run:    sync_gap.py run OUT.json [reps]
        K synchronous calls back to back from C (libmpix_bench's
        mpix_bench_call_loop_ts), each call's host entry / return stamped on
        CLOCK_MONOTONIC and CLOCK_BOOTTIME.  Run it under
        rocprofv3 --kernel-trace --output-format csv.
report: sync_gap.py report OUT.json KERNEL_TRACE.csv
        lines the calls up with the trace (the clock whose offset puts each
        kernel inside its call) and splits each call into
          launch   host entry -> kernel start
          kernel   the k_contig dispatch
          to_blit  kernel end -> the stream's completion write
                   (__amd_rocclr_streamOpsWrite) starts
          blit     that write's own duration
          wake     write end -> host return (spin sees the word)
          between  host return -> next call's entry (the loop itself)
"""
import ctypes
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out, reps):
    import torch
    from mpich_amd import handles as H
    from mpich_amd import redop
    n = 1 << 28
    dev = torch.device('cuda', 0)
    a = torch.empty(n, dtype=torch.float32, device=dev).uniform_(-1, 1)
    b = torch.empty(n, dtype=torch.float32, device=dev).uniform_(-1, 1)
    torch.cuda.synchronize()
    B = ctypes.CDLL(os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so'))
    B.mpix_bench_call_loop_ts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_uint64)]
    fn = ctypes.cast(redop.lib().MPIX_Reduce_local, ctypes.c_void_p).value
    t = (ctypes.c_uint64 * (4 * reps))()
    for _ in range(2):          # warm-up pass, then the recorded one
        rc = B.mpix_bench_call_loop_ts(fn, b.data_ptr(), a.data_ptr(), n, H.as_c_int(H.MPI_FLOAT),
                                       H.as_c_int(H.MPI_SUM), reps, t)
        assert rc == 0, rc
    calls = [dict(mono_in=t[4 * i], mono_out=t[4 * i + 1], boot_in=t[4 * i + 2],
                  boot_out=t[4 * i + 3]) for i in range(reps)]
    json.dump(dict(reps=reps, count=n, calls=calls), open(out, 'w'))
    per = [(c['mono_out'] - c['mono_in']) / 1e3 for c in calls]
    print(json.dumps(dict(calls=reps, median_call_us=round(statistics.median(per), 2))))


def report(host_json, trace_csv, out=None):
    h = json.load(open(host_json))
    calls = h['calls']
    rows = list(csv.DictReader(open(trace_csv)))
    ev = []
    for r in rows:
        name = r.get('Kernel_Name') or r.get('KernelName') or ''
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        ev.append((s, e, name))
    ev.sort()
    ks = [x for x in ev if 'k_contig' in x[2]]
    blits = [x for x in ev if 'streamOpsWrite' in x[2]]
    # the recorded pass = the last len(calls) big kernels
    big = [x for x in ks if x[1] - x[0] > 100000][-len(calls):]
    best = None
    for clk in ('mono', 'boot'):
        inside = sum(c[clk + '_in'] <= k[0] and k[1] <= c[clk + '_out'] for c, k in zip(calls, big))
        if best is None or inside > best[1]:
            best = (clk, inside)
    clk = best[0]
    parts = {k: [] for k in ('launch', 'kernel', 'to_blit', 'blit', 'wake', 'call', 'between')}
    for i, (c, k) in enumerate(zip(calls, big)):
        bl = next((b for b in blits if b[0] >= k[1]), None)
        parts['launch'].append((k[0] - c[clk + '_in']) / 1e3)
        parts['kernel'].append((k[1] - k[0]) / 1e3)
        if bl and bl[1] <= c[clk + '_out'] + 1000:
            parts['to_blit'].append((bl[0] - k[1]) / 1e3)
            parts['blit'].append((bl[1] - bl[0]) / 1e3)
            parts['wake'].append((c[clk + '_out'] - bl[1]) / 1e3)
        else:
            parts['wake'].append((c[clk + '_out'] - k[1]) / 1e3)
        parts['call'].append((c[clk + '_out'] - c[clk + '_in']) / 1e3)
        if i + 1 < len(calls):
            parts['between'].append((calls[i + 1][clk + '_in'] - c[clk + '_out']) / 1e3)
    summ = {k: dict(median_us=round(statistics.median(v), 2), mean_us=round(statistics.mean(v), 2),
                    n=len(v)) for k, v in parts.items() if v}
    res = dict(clock=clk, kernels_inside_calls=best[1], calls=len(calls), split=summ,
               overhead_us_median=round(summ['call']['median_us'] - summ['kernel']['median_us'], 2),
               note='per synchronous 1 GiB fp32 SUM call; launch = host entry to kernel start, '
                    'to_blit + blit = the stream completion write after the kernel, wake = its '
                    'end to the host seeing the word and returning')
    if out:
        json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    if sys.argv[1] == 'run':
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        report(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
