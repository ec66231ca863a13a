"""The store policy (MPIX_Redop_set_store_policy, XCD mask 0x88 by default)
under concurrent HBM traffic.  It was found on an idle
GPU running one kernel; in the collectives its neighbours are RCCL kernels
and inbound xGMI writes.  Stand-in here: a second stream doing back-to-back
device-to-device hipMemcpyAsync of 1 GiB (as RCCL's copy kernels do, at the
full rate the device gives them) while the combine runs.

Per (kernel, concurrent copy on/off, policy 0 / 0x88), alternating, `reps`
launches timed with HIP events on the combine's stream: k_contig fp32 SUM on
1 GiB operands (the headline kernel) and the 7-input k_contig_multi of the
pairwise reduce-scatter at P = 8 (1 GiB inout, seven 1 GiB inputs would be
8 GiB -- here seven 256 MiB inputs over a 256 MiB inout).  The copy stream's
own rate is reported beside.  Bits are unaffected by the policy
(tests/test_store_policy.py); only the speed is measured.

usage: python3 tools/policy_concurrent.py [--reps 10] [--rounds 4] > out.json
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpich_amd import handles as H  # noqa: E402
from mpich_amd import redop  # noqa: E402


def timed(fn, reps, stream):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=4)
    ap.add_argument('--traffic', default='full,16,64',
                    help="concurrent copy kinds: 'full' (torch D2D copy, the device's rate) "
                         "and/or workgroup counts of the throttled copy kernel")
    a = ap.parse_args()
    import ctypes
    B = ctypes.CDLL(os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so'))
    B.mpix_bench_trickle_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_int, ctypes.c_void_p]
    assert redop.lib().MPIX_Redop_init() == 0
    dev = torch.device('cuda', 0)
    n = 1 << 28                                  # 1 GiB fp32
    x = torch.rand(n, device=dev)
    y = torch.rand(n, device=dev)
    m = 1 << 26                                  # 256 MiB
    ins = [torch.rand(m, device=dev) for _ in range(7)]
    acc = torch.rand(m, device=dev)
    csrc = torch.empty(n, dtype=torch.float32, device=dev)
    cdst = torch.empty(n, dtype=torch.float32, device=dev)
    # the copies on a high-priority stream: a hardware queue of its own (two
    # streams of one priority may share one of the GPU_MAX_HW_QUEUES queues and
    # then run one after the other); row['overlapped'] checks it on the GPU clock
    ks, cs = torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=-1)
    torch.cuda.synchronize()
    kernels = {
        'contig_fp32_sum_1GiB': (lambda: redop.check(redop.reduce_local_async(
            x, y, n, H.MPI_FLOAT, H.MPI_SUM, ks)), 3 * n * 4),
        'multi7_fp32_sum_256MiB': (lambda: redop.check(redop.reduce_local_multi_async(
            ins, acc, m, H.MPI_FLOAT, H.MPI_SUM, ks)), 9 * m * 4),
    }
    def copier(kind):
        if kind == 'full':
            return lambda: cdst.copy_(csrc)
        nb = int(kind)
        return lambda: B.mpix_bench_trickle_copy(cdst.data_ptr(), csrc.data_ptr(), n * 4, nb,
                                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    kinds = ['none'] + a.traffic.split(',')
    # each copier's own rate, alone
    alone = {}
    for kind in kinds[1:]:
        cms = timed(copier(kind), 5, torch.cuda.current_stream())
        alone[kind] = dict(ms=round(cms, 4), GBs=round(2 * n * 4 / (cms * 1e-3) / 1e9, 1))
    res = dict(copy_alone=alone, rows=[])
    default = redop.get_store_policy()
    try:
        for rnd in range(a.rounds):
            for kname, (fn, nbytes) in kernels.items():
                for copy_on in kinds:
                    pols = (0, 0x88) if rnd % 2 == 0 else (0x88, 0)
                    for pol in pols:
                        redop.check(redop.set_store_policy(pol, 0, 0, 0))
                        fn()
                        torch.cuda.synchronize()
                        ncopies = 0
                        t0 = torch.cuda.Event(enable_timing=True)
                        t0.record(torch.cuda.current_stream())
                        ks.wait_stream(torch.cuda.current_stream())
                        cs.wait_stream(torch.cuda.current_stream())
                        if copy_on != 'none':
                            # enough copies to outlast the timed launches
                            per = alone[copy_on]['ms']
                            ncopies = max(4, int(3 * a.reps * nbytes / 6.5e9 / per) + 4)
                            c0 = torch.cuda.Event(enable_timing=True)
                            c1 = torch.cuda.Event(enable_timing=True)
                            cp = copier(copy_on)
                            with torch.cuda.stream(cs):
                                c0.record(cs)
                                for _ in range(ncopies):
                                    cp()
                                c1.record(cs)
                        k0 = torch.cuda.Event(enable_timing=True)
                        k1 = torch.cuda.Event(enable_timing=True)
                        with torch.cuda.stream(ks):
                            k0.record(ks)
                            ms = timed(fn, a.reps, ks)
                            k1.record(ks)
                        torch.cuda.synchronize()
                        row = dict(round=rnd, kernel=kname, concurrent_copy=copy_on,
                                   xcd_mask=pol, kernel_ms=round(ms, 4),
                                   kernel_GBs=round(nbytes / (ms * 1e-3) / 1e9, 1))
                        row['kernels_span_ms'] = [round(t0.elapsed_time(k0), 3),
                                                  round(t0.elapsed_time(k1), 3)]
                        if copy_on != 'none':
                            cms = c0.elapsed_time(c1) / ncopies
                            row['copy_ms_each'] = round(cms, 4)
                            # both windows on one clock: the kernels must sit
                            # inside the copies' window, or nothing overlapped
                            row['copies_span_ms'] = [round(t0.elapsed_time(c0), 3),
                                                     round(t0.elapsed_time(c1), 3)]
                            row['overlapped'] = (t0.elapsed_time(c0) < t0.elapsed_time(k0) and
                                                 t0.elapsed_time(k1) < t0.elapsed_time(c1))
                        res['rows'].append(row)
    finally:
        dm = default['xcd_mask']
        redop.set_store_policy(dm if dm >= -1 else -1, default['every'], default['phase'],
                               default['tail_blocks'])
    # summary: median kernel time per (kernel, copy, policy) and the policy's gain
    summ = {}
    for r in res['rows']:
        summ.setdefault((r['kernel'], r['concurrent_copy'], r['xcd_mask']), []).append(r['kernel_ms'])
    out = []
    for kname in kernels:
        for copy_on in kinds:
            off = sorted(summ[(kname, copy_on, 0)])
            on = sorted(summ[(kname, copy_on, 0x88)])
            mo, mn = off[len(off) // 2], on[len(on) // 2]
            cps = [r['copy_ms_each'] for r in res['rows']
                   if r['kernel'] == kname and r['concurrent_copy'] == copy_on and 'copy_ms_each' in r]
            out.append(dict(kernel=kname, concurrent_copy=copy_on, policy_off_ms=mo,
                            policy_0x88_ms=mn, gain=round(mo / mn - 1, 4),
                            copy_GBs_during=round(2 * n * 4 / (sorted(cps)[len(cps) // 2] * 1e-3)
                                                  / 1e9, 1) if cps else None))
    res['summary'] = out
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
