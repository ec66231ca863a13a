"""Pull-window growth on one GPU shared by P processes (the N > 1 bench flow
rehearsed on a 1-GPU box): how often does a window fail verification, and
what does the failing mapping show instead?  One round = a fresh spawn of P
ranks that (like bench.py) allocates and frees large tensors, runs a staged
recursive-halving RSB, then pulls at a small size (first window) and at
`--mib` MiB per rank (the window grows), checking every result bit for bit
against the redscatblk3.c closed form.  MPIX_COLL_TRACE=1 is on; each rank's
trace goes to <out>/r<round>_rank<r>.txt.  Prints one JSON line per round.

  python3 tools/win_grow_probe.py --ranks 4 --rounds 5 --mib 512 --out gpurun_out/wg
"""
import argparse
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPI_INT, MPI_FLOAT, MPI_SUM = 0x4c000405, 0x4c00040a, 0x58000003


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _closed(world, rank, n, it):
    return world * rank + world * (world - 1) // 2 + world * it


def _worker(rank, world, port, out, rnd, mib):
    sys.path.insert(0, ROOT)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['MPIX_COLL_TRACE'] = '1'
    torch.cuda.set_device(0)
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    tr = open(os.path.join(out, 'r%d_rank%d.txt' % (rnd, rank)), 'w')
    os.dup2(tr.fileno(), 2)
    from mpich_amd import coll
    # what bench.py does before the pulls: large allocations freed again
    a = torch.empty(1 << 28, dtype=torch.float32, device='cuda')
    b = torch.empty(1 << 28, dtype=torch.float32, device='cuda')
    del a, b
    torch.cuda.empty_cache()
    n_big = (mib << 20) // 4 // world
    send = torch.empty(world * n_big, dtype=torch.float32, device='cuda').uniform_(-1, 1)
    recv = torch.empty(n_big, dtype=torch.float32, device='cuda')
    torch.cuda.synchronize()
    coll.reduce_scatter_block(send, recv, n_big, MPI_FLOAT, MPI_SUM, algorithm='recursive_halving')
    ref = recv.clone()
    bad = []
    for it, (algo, n) in enumerate((('recursive_halving_pull', 4099), ('recursive_halving_pull', n_big),
                                   ('pull', n_big))):
        blk = torch.cat([torch.full((n,), rank + i + it, dtype=torch.int32, device='cuda')
                         for i in range(world)])
        o = torch.empty(n, dtype=torch.int32, device='cuda')
        torch.cuda.synchronize()
        coll.reduce_scatter_block(blk, o, n, MPI_INT, MPI_SUM, algorithm=algo)
        torch.cuda.synchronize()
        if not bool(torch.all(o == _closed(world, rank, n, it))):
            bad.append('%s@%d' % (algo, n))
        del blk, o
    coll.reduce_scatter_block(send, recv, n_big, MPI_FLOAT, MPI_SUM, algorithm='recursive_halving_pull')
    torch.cuda.synchronize()
    if not torch.equal(recv.view(torch.int32), ref.view(torch.int32)):
        bad.append('rh_pull_bits')
    with open(os.path.join(out, 'r%d_bad%d.txt' % (rnd, rank)), 'w') as f:
        f.write(' '.join(bad))
    dist.barrier()
    coll.free_comms()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ranks', type=int, default=4)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--mib', type=int, default=512)
    ap.add_argument('--out', default='gpurun_out/wg')
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for rnd in range(a.rounds):
        mp.spawn(_worker, args=(a.ranks, _port(), a.out, rnd, a.mib), nprocs=a.ranks, join=True)
        lines = []
        for r in range(a.ranks):
            lines += [ln.strip() for ln in open(os.path.join(a.out, 'r%d_rank%d.txt' % (rnd, r)))
                      if 'window' in ln]
        bad = [open(os.path.join(a.out, 'r%d_bad%d.txt' % (rnd, r))).read() for r in range(a.ranks)]
        print(json.dumps(dict(round=rnd, failed_attempts=sum('all 0' in ln for ln in lines),
                              wrong_reads=[ln for ln in lines if 'reads' in ln][:8],
                              bad=[b for b in bad if b])), flush=True)


if __name__ == '__main__':
    main()
