"""Host-side cost of one asynchronous MPIX_Reduce_local_async call, split
into its parts (pointer classification, kernel issue, stream round trip) by
libmpix_bench.so's mpix_bench_launch_floor.  Prints one JSON line.
Usage: python tools/launch_floor.py [out.json]"""
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
    B = ctypes.CDLL(os.path.join(ROOT, 'mpich_amd', 'libmpix_bench.so'))
    B.mpix_bench_launch_floor.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int,
                                                                   ctypes.c_int, ctypes.c_void_p,
                                                                   ctypes.c_int, ctypes.c_void_p]
    L = redop.lib()
    fn = ctypes.cast(L.MPIX_Reduce_local_async, ctypes.c_void_p).value
    s = torch.cuda.Stream()
    rows = []
    keys = ['hipPointerGetAttributes_us', 'hipPointerGetAttribute_type_us', 'empty_launch_issue_us',
            'reduce_async_issue_us', 'empty_launch_roundtrip_us', 'reduce_async_roundtrip_us', 'empty_launch_112B_args_us']
    for count in (1, 16384, 262144):
        a = torch.ones(count, dtype=torch.float32, device='cuda')
        b = torch.ones(count, dtype=torch.float32, device='cuda')
        torch.cuda.synchronize()
        out = (ctypes.c_double * 7)()
        rc = B.mpix_bench_launch_floor(fn, a.data_ptr(), b.data_ptr(), count, H.MPI_FLOAT,
                                       H.MPI_SUM, ctypes.c_void_p(s.cuda_stream), 20000, out)
        if rc:
            raise RuntimeError('mpix_bench_launch_floor rc=%d' % rc)
        rows.append(dict(count=count, **{k: round(v, 3) for k, v in zip(keys, out)}))
    line = json.dumps({'launch_floor': rows})
    print(line)
    if len(sys.argv) > 1:
        with open(sys.argv[1], 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
