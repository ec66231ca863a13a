"""Small-call figures of bench.py alone (sync_call_latency, chunked_async_c
at 64 KiB / 1 MiB / 16 MiB), for comparing HIP runtime settings (env) in
separate processes.  One JSON line: {"env": ..., "sync": [...], "chunked": [...]}."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mpich_amd import redop  # noqa: E402

KNOBS = ('HIP_FORCE_DEV_KERNARG', 'DEBUG_CLR_KERNARG_HDP_FLUSH_WA', 'ROC_USE_FGS_KERNARG',
         'DEBUG_HIP_KERNARG_COPY_OPT')


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    assert redop.lib().MPIX_Redop_init() == 0
    B = bench.bench_lib()
    n = 1 << 28
    inb = torch.zeros(n, dtype=torch.float32, device=dev)
    inout = torch.zeros(n, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    sync = bench.sync_call_latency(B, dev)
    chunked = bench.chunked_async_c(B, inb, inout, n, stream, (64 << 10, 1 << 20, 16 << 20))
    print(json.dumps(dict(env={k: os.environ.get(k) for k in KNOBS if os.environ.get(k)},
                          sync=sync, chunked=chunked)), flush=True)


if __name__ == '__main__':
    main()
