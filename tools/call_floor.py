"""Per-call floor of the stream-ordered entry, issue and GPU sides apart
(VERDICT r03 item 3): bursts of `burst` back-to-back MPIX_Reduce_local_async
calls (64 KiB and 1-element fp32 SUM) and of empty kernels, host issue time
and burst time including its drain, per call; the host cost of issuing an
empty kernel by argument-block size; and the synchronous 1-element call.
Prints one JSON line.  usage: python3 tools/call_floor.py [--burst 64]"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--burst', type=int, default=64)
    ap.add_argument('--rounds', type=int, default=200)
    a = ap.parse_args()
    B = ctypes.CDLL(os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so'))
    B.mpix_bench_issue_burst.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int,
                                                                  ctypes.c_int, ctypes.c_void_p,
                                                                  ctypes.c_int, ctypes.c_int,
                                                                  ctypes.c_void_p]
    B.mpix_bench_call_latency.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double)]
    L = redop.lib()
    assert L.MPIX_Redop_init() == 0
    fa = ctypes.cast(L.MPIX_Reduce_local_async, ctypes.c_void_p).value
    fs = ctypes.cast(L.MPIX_Reduce_local, ctypes.c_void_p).value
    s = torch.cuda.Stream()
    # bench.py's decomposition first, in a process that has done nothing else
    import bench
    xb = torch.ones(1 << 20, dtype=torch.float32, device='cuda')
    yb = torch.zeros(1 << 20, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    parts_fresh = bench.call_floor_parts(bench.bench_lib(), xb, yb, s)
    keys = ['reduce_issue_us', 'reduce_burst_us', 'empty_issue_us', 'empty_burst_us',
            'empty_args8_issue_us', 'empty_args64_issue_us', 'empty_args128_issue_us',
            'empty_args256_issue_us', 'empty_args1024_issue_us', 'empty_args2048_issue_us']
    out = dict(burst=a.burst, rounds=a.rounds,
               env={k: v for k, v in os.environ.items() if k.startswith(('HIP_', 'MPIX_'))})
    rows = []
    for count in (1, 16384, 262144):
        x = torch.ones(count, dtype=torch.float32, device='cuda')
        y = torch.zeros(count, dtype=torch.float32, device='cuda')
        torch.cuda.synchronize()
        o = (ctypes.c_double * 10)()
        rc = B.mpix_bench_issue_burst(fa, x.data_ptr(), y.data_ptr(), count, H.MPI_FLOAT, H.MPI_SUM,
                                      ctypes.c_void_p(s.cuda_stream), a.burst, a.rounds, o)
        assert rc == 0, rc
        med, p90 = ctypes.c_double(), ctypes.c_double()
        rc = B.mpix_bench_call_latency(fs, x.data_ptr(), y.data_ptr(), count, H.MPI_FLOAT,
                                       H.MPI_SUM, 2000, ctypes.byref(med), ctypes.byref(p90))
        assert rc == 0, rc
        rows.append(dict(count=count, sync_median_us=round(med.value, 2),
                         **{k: round(v, 3) for k, v in zip(keys, o)}))
    out['rows'] = rows
    # steady state: n back-to-back 64 KiB calls (the bench's chunked_async_c
    # loop) for growing n -- where the per-call time leaves the burst figure,
    # the host is waiting for room in the stream's queue
    B.mpix_bench_chunked_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]
    m = 16384
    x = torch.ones(m * 16384, dtype=torch.float32, device='cuda')
    y = torch.zeros(m * 16384, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    steady = []
    for ncalls in (64, 256, 1024, 4096, 16384):
        issue, total = ctypes.c_double(), ctypes.c_double()
        rc = B.mpix_bench_chunked_async(fa, x.data_ptr(), y.data_ptr(), m * ncalls, m, 4,
                                        H.MPI_FLOAT, H.MPI_SUM, ctypes.c_void_p(s.cuda_stream),
                                        ctypes.byref(issue), ctypes.byref(total))
        assert rc == 0, rc
        steady.append(dict(calls=ncalls, issue_us_per_call=round(1e6 * issue.value / ncalls, 3),
                           us_per_call=round(1e6 * total.value / ncalls, 3)))
    out['steady_64KiB'] = steady
    out['parts_fresh'] = parts_fresh
    out['parts_after'] = bench.call_floor_parts(bench.bench_lib(), xb, yb, s)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
