"""P processes on one GPU: every round each rank frees its buffer, makes a new
one of the same size, fills it with 1000 * (rank + 1) + round, exports it and
all-gathers the handles (gloo); every rank then opens each peer's handle,
reads the first word and checks it, then closes the mappings (policy
'close') or keeps them until the peer's buffer id changes (policy 'lazy':
close all of that peer's mappings, then open); 'nofree' closes like 'close'
but never frees a buffer (each round makes a new one beside the old).  Shows whether a freshly
opened handle can alias another peer's or an earlier allocation.  Usage:
python tools/ipc_multi_probe.py P out.json"""
import ctypes
import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp


class Handle(ctypes.Structure):
    _fields_ = [('reserved', ctypes.c_char * 64)]


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, policy, outdir):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    hip = ctypes.CDLL('libamdhip64.so.7')
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    hip.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(Handle), ctypes.c_void_p]
    hip.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    log = []
    maps = {}       # peer -> (buffer id, mapped base)
    p = None
    for rnd in range(5):
        if p is not None:
            dist.barrier()              # peers done reading the old buffer
            if policy != 'nofree':      # nofree: old buffers stay allocated
                assert hip.hipFree(p) == 0
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(16 << 20)) == 0
        val = 1000 * (rank + 1) + rnd
        t = torch.full((4,), val, dtype=torch.int32, device='cuda')
        assert hip.hipMemcpy(p, ctypes.c_void_p(t.data_ptr()), ctypes.c_size_t(16), 3) == 0
        torch.cuda.synchronize()
        h = Handle()
        rc_get = hip.hipIpcGetMemHandle(ctypes.byref(h), p)
        bid = ctypes.c_ulonglong()
        rc_bid = hip.hipPointerGetAttribute(ctypes.byref(bid), 7, p)
        hip.hipGetLastError()       # a failed call's error must not reach torch's next check
        mine = (ctypes.string_at(ctypes.addressof(h), 64), bid.value, p.value) if rc_get == 0 \
            else None
        if rc_get:
            log.append(dict(rnd=rnd, export_rc=rc_get, bid_rc=rc_bid, va=hex(p.value)))
        allrec = [None] * world
        dist.all_gather_object(allrec, mine)
        for q in range(world):
            if q == rank or allrec[q] is None:
                continue
            raw, qbid, qva = allrec[q]
            cached = maps.get(q)
            if policy == 'lazy' and cached is not None and cached[0] == qbid:
                base = cached[1]
                how = 'cached'
            else:
                if cached is not None:
                    hip.hipIpcCloseMemHandle(ctypes.c_void_p(cached[1]))
                    hip.hipGetLastError()
                    maps.pop(q)
                hh = Handle()
                ctypes.memmove(ctypes.addressof(hh), raw, 64)
                b = ctypes.c_void_p()
                rc = hip.hipIpcOpenMemHandle(ctypes.byref(b), hh, 1)
                hip.hipGetLastError()
                if rc:
                    log.append(dict(rnd=rnd, peer=q, open_rc=rc))
                    continue
                base = b.value
                how = 'opened'
                if policy == 'lazy':
                    maps[q] = (qbid, base)
            got = torch.zeros(4, dtype=torch.int32, device='cuda')
            hip.hipMemcpy(ctypes.c_void_p(got.data_ptr()), ctypes.c_void_p(base), ctypes.c_size_t(16), 3)
            torch.cuda.synchronize()
            g = int(got[0])
            log.append(dict(rnd=rnd, peer=q, expect=1000 * (q + 1) + rnd, got=g, how=how,
                            peer_va=hex(qva), mapped=hex(base), ok=g == 1000 * (q + 1) + rnd))
            if policy in ('close', 'nofree'):
                hip.hipIpcCloseMemHandle(ctypes.c_void_p(base))
                hip.hipGetLastError()
    with open(os.path.join(outdir, '%s_%d.json' % (policy, rank)), 'w') as f:
        json.dump(log, f)
    dist.barrier()
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1])
    out = sys.argv[2]
    d = os.path.dirname(out) or '.'
    res = {}
    for policy in ('close', 'lazy', 'nofree'):
        mp.spawn(worker, args=(world, _port(), policy, d), nprocs=world, join=True)
        logs = [json.load(open(os.path.join(d, '%s_%d.json' % (policy, r)))) for r in range(world)]
        bad = [dict(rank=r, **e) for r, lg in enumerate(logs) for e in lg if not e.get('ok')]
        bad.sort(key=lambda e: (e['rnd'], e['rank']))
        res[policy] = dict(reads=sum(len(lg) for lg in logs), bad=bad[:20], nbad=len(bad),
                           sample=logs[0][:6])
    line = json.dumps({'ipc_multi_probe': res, 'P': world})
    print(line)
    with open(out, 'w') as f:
        f.write(line + '\n')


if __name__ == '__main__':
    main()
