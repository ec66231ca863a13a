"""HBM rate of the multi-input kernels on one GPU: the tree fold
(MPIX_Reduce_local_tree_async, k slots -> one output) and the in-order fold
(MPIX_Reduce_local_multi_async, inout + k inputs), fp32 SUM, k blocks of
`--mib` MiB each.  Bytes per launch: tree (k + 1) x block, multi (k + 2) x
block.  Prints one JSON line.  Usage: python tools/tree_probe.py [--mib 256]"""
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


def timed(fn, s, reps=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--mib', type=int, default=256)
    ap.add_argument('--out', default=None)
    ap.add_argument('--xcd', type=lambda x: int(x, 0), default=None,
                    help='store policy XCD mask (MPIX_Redop_set_store_policy); default: the library\'s')
    a = ap.parse_args()
    if a.xcd is not None:
        redop.check(redop.set_store_policy(a.xcd, 0, 0, 0))
    n = a.mib * (1 << 20) // 4
    s = torch.cuda.Stream()
    rows = []
    with torch.cuda.stream(s):
        for k in (2, 4, 8, 16):
            blocks = [torch.rand(n, device='cuda') for _ in range(k)]
            out = torch.empty(n, device='cuda')
            acc = torch.empty(n, device='cuda')
            torch.cuda.synchronize()
            ptrs = [b.data_ptr() for b in blocks]

            def tree():
                redop.check(redop.reduce_local_tree_async(ptrs, out.data_ptr(), n, H.MPI_FLOAT,
                                                          H.MPI_SUM, stream=s.cuda_stream),
                            'tree')

            def multi():
                redop.check(redop.reduce_local_multi_async(ptrs[1:], acc.data_ptr(), n,
                                                           H.MPI_FLOAT, H.MPI_SUM,
                                                           stream=s.cuda_stream), 'multi')
            tt, tm = timed(tree, s), timed(multi, s)
            bt, bm = (k + 1) * n * 4, (k + 1) * n * 4      # multi: inout + k-1 inputs
            rows.append(dict(k=k, block_MiB=a.mib, tree_ms=round(tt * 1e3, 4),
                             tree_GBs=round(bt / tt / 1e9, 1), multi_ms=round(tm * 1e3, 4),
                             multi_GBs=round(bm / tm / 1e9, 1)))
            del blocks, out, acc
            torch.cuda.empty_cache()
    # the pull allgather's gather kernel: 7 segments of `mib` MiB in one launch
    # against 7 back-to-back hipMemcpyAsync (device to device), local HBM
    L = redop.lib()
    vp = ctypes.c_void_p
    L.MPIX_Copy_multi_async.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                        ctypes.POINTER(ctypes.c_ssize_t), ctypes.c_int, vp]
    n = a.mib * (1 << 20) // 4
    with torch.cuda.stream(s):
        src = [torch.rand(n, device='cuda') for _ in range(7)]
        dst = [torch.empty(n, device='cuda') for _ in range(7)]
        torch.cuda.synchronize()
        srcs = (vp * 7)(*[t.data_ptr() for t in src])
        dsts = (vp * 7)(*[t.data_ptr() for t in dst])
        nb = (ctypes.c_ssize_t * 7)(*([n * 4] * 7))

        def multi():
            assert L.MPIX_Copy_multi_async(srcs, dsts, nb, 7, vp(s.cuda_stream)) == 0

        def memcpys():
            for x, y in zip(src, dst):
                y.copy_(x, non_blocking=True)
        tc, tm = timed(multi, s), timed(memcpys, s)
        assert all(torch.equal(x, y) for x, y in zip(src, dst))
        copy_row = dict(segments=7, segment_MiB=a.mib, copy_multi_ms=round(tc * 1e3, 4),
                        copy_multi_GBs=round(2 * 7 * n * 4 / tc / 1e9, 1),
                        memcpy_ms=round(tm * 1e3, 4),
                        memcpy_GBs=round(2 * 7 * n * 4 / tm / 1e9, 1))
        del src, dst
    line = json.dumps({'tree_probe': rows, 'copy_multi': copy_row,
                       'store_policy': redop.get_store_policy()})
    print(line)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
