"""The N > 1 bench's rank setup at one rank: torch's RCCL process group and
libmpix_coll's own RCCL communicator in the same process.

bench.py's ranks (N > 1, no rehearsal knobs) call
`dist.init_process_group('nccl', device_id=...)` and then
`ccl.comm_create_ccl_from_process_group()` (the unique id broadcast over that
group, as `MPIR_RCCLcomm_init` does, rccl.c:33-43), so two users of RCCL share
one process.  RCCL refuses two ranks on one device, so the one-GPU box runs the
same setup at world size 1: both collectives, then both teardowns in the bench's
order.  It also records which librccl the process mapped -- libmpix_coll's
`librccl.so.1` resolves to the copy torch already loaded (one RCCL per process).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import json, os, sys
sys.path.insert(0, %(root)r)
import torch
import torch.distributed as dist
from mpich_amd import ccl, redop
from mpich_amd import handles as H
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
dist.init_process_group('nccl', device_id=dev, init_method='tcp://127.0.0.1:%(port)d',
                        rank=0, world_size=1)
t = torch.ones(1 << 20, device=dev)
dist.all_reduce(t)
assert redop.lib().MPIX_Redop_init() == 0
c = ccl.comm_create_ccl_from_process_group()
n = 1 << 22
x = torch.rand(n, device=dev)
y = torch.empty_like(x)
z = torch.empty_like(x)
torch.cuda.synchronize()
assert ccl.reduce_scatter_block(x, y, n, H.MPI_FLOAT, H.MPI_SUM, c) == 0
assert ccl.allreduce(x, z, n, H.MPI_FLOAT, H.MPI_SUM, c) == 0
torch.cuda.synchronize()
ok = bool(torch.equal(x, y) and torch.equal(x, z))
dist.all_reduce(t)          # torch's group still works after ours ran
torch.cuda.synchronize()
ok = ok and bool((t == 1).all())
dist.barrier()
assert c.free() == 0
dist.destroy_process_group()
maps = set()
for line in open('/proc/self/maps'):
    p = line.split()[-1]
    if 'librccl' in p:
        maps.add(os.path.realpath(p))
print(json.dumps(dict(ok=ok, rccl=sorted(maps))))
'''


@pytest.mark.gpu
def test_torch_process_group_and_ccl_comm_share_a_process():
    sys.path.insert(0, ROOT)
    import bench
    code = SCRIPT % dict(root=ROOT, port=bench.free_port())
    env = {k: v for k, v in os.environ.items()
           if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT', 'MASTER_ADDR')}
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=150,
                       env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d['ok'], d
    assert len(d['rccl']) == 1, d      # one RCCL library in the process
