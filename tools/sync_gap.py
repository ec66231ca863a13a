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
        splits the time between consecutive kernels on the GPU's own clock
        (kernel, end -> completion write, the write, write -> next kernel)
        and reads the host's per-call time beside it
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
    """the split of one call, from the GPU's own timestamps (exact, one clock)
    plus the host's per-call time (another clock: only differences of it are
    used, never compared with the GPU's)"""
    h = json.load(open(host_json))
    calls = h['calls']
    ev = []
    for r in csv.DictReader(open(trace_csv)):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    ev.sort()
    # the recorded pass: the last len(calls) big kernels, each followed by its
    # stream completion write (__amd_rocclr_streamOpsWrite)
    big = [i for i, x in enumerate(ev) if 'k_contig' in x[2] and x[1] - x[0] > 100000]
    big = big[-len(calls):]
    parts = {k: [] for k in ('kernel', 'end_to_signal', 'signal', 'signal_to_next_kernel',
                             'gpu_period', 'host_call', 'host_period')}
    for j, i in enumerate(big):
        k = ev[i]
        parts['kernel'].append((k[1] - k[0]) / 1e3)
        sig = ev[i + 1] if i + 1 < len(ev) and 'streamOpsWrite' in ev[i + 1][2] else None
        if sig:
            parts['end_to_signal'].append((sig[0] - k[1]) / 1e3)
            parts['signal'].append((sig[1] - sig[0]) / 1e3)
        if j + 1 < len(big):
            nxt = ev[big[j + 1]]
            parts['gpu_period'].append((nxt[0] - k[0]) / 1e3)
            if sig:
                parts['signal_to_next_kernel'].append((nxt[0] - sig[1]) / 1e3)
    for j, c in enumerate(calls):
        parts['host_call'].append((c['mono_out'] - c['mono_in']) / 1e3)
        if j + 1 < len(calls):
            parts['host_period'].append((calls[j + 1]['mono_in'] - c['mono_in']) / 1e3)
    med = {k: round(statistics.median(v), 2) for k, v in parts.items() if v}
    res = dict(calls=len(calls), median_us=med,
               overhead_us=round(med['host_call'] - med['kernel'], 2),
               gpu_idle_between_kernels_us=round(med['gpu_period'] - med['kernel'], 2),
               note='one synchronous 1 GiB fp32 SUM MPIX_Reduce_local per call, called back to '
                    'back from C. GPU clock: kernel, end_to_signal (kernel end -> the stream\'s '
                    'completion write starts: end-of-kernel release + dispatch), signal (that '
                    'write, a blit kernel), signal_to_next_kernel (host sees the word, returns, '
                    'enters the next call, launches; the kernel starts). host_call - kernel = '
                    'the per-call overhead against the kernel alone.')
    if out:
        json.dump(res, open(out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    if sys.argv[1] == 'run':
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        report(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
