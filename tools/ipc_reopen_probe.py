"""Two processes on one GPU: the exporter makes an allocation, fills it with
its round number, exports it; the importer opens the handle, reads the first
word, closes it.  The exporter then frees the allocation and makes a new one
(same size, so usually the same address and the same handle bytes) and the
round repeats.  Shows whether a re-opened handle maps the NEW allocation or
a stale one, with and without closing in between.  Prints one JSON line."""
import ctypes
import json
import multiprocessing as mproc
import sys


class Handle(ctypes.Structure):             # hipIpcMemHandle_t, passed BY VALUE to open
    _fields_ = [('reserved', ctypes.c_char * 64)]


def _hip():
    import torch
    torch.cuda.init()
    hip = ctypes.CDLL('libamdhip64.so.7')     # torch's runtime, already loaded
    hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
    hip.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(Handle), ctypes.c_void_p]
    hip.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    return hip


def exporter(q_out, q_in, rounds):
    hip = _hip()
    import torch
    for r in range(rounds):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(16 << 20)) == 0
        t = torch.full((4,), r + 1, dtype=torch.int32, device='cuda')
        assert hip.hipMemcpy(p, ctypes.c_void_p(t.data_ptr()), ctypes.c_size_t(16), 3) == 0
        h = Handle()
        assert hip.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
        q_out.put((r, p.value, ctypes.string_at(ctypes.addressof(h), 64)))   # .reserved stops at a NUL
        q_in.get(timeout=60)            # importer done with this round
        assert hip.hipFree(p) == 0
    q_out.put(None)


def importer(q_in, q_out, close_each, res):
    hip = _hip()
    import torch
    seen = []
    mapped = {}
    while True:
        m = q_in.get(timeout=60)
        if m is None:
            break
        r, va, raw = m
        h = Handle()
        ctypes.memmove(ctypes.addressof(h), raw, 64)
        base = mapped.get(raw)
        rc_open = None
        if base is None:
            b = ctypes.c_void_p()
            rc_open = hip.hipIpcOpenMemHandle(ctypes.byref(b), h, 1)
            if rc_open:
                seen.append(dict(round=r, open_rc=rc_open))
                q_out.put(1)
                continue
            base = b.value
            if not close_each:
                mapped[raw] = base
        t = torch.zeros(4, dtype=torch.int32, device='cuda')
        rc_cp = hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(base),
                              ctypes.c_size_t(16), 3)
        torch.cuda.synchronize()
        seen.append(dict(round=r, expect=r + 1, got=int(t[0]), open_rc=rc_open, copy_rc=rc_cp,
                         va=hex(va), mapped_at=hex(base or 0)))
        if close_each:
            seen[-1]['close_rc'] = hip.hipIpcCloseMemHandle(ctypes.c_void_p(base))
        q_out.put(1)
    res.put(seen)


def run(close_each):
    ctx = mproc.get_context('spawn')
    a, b, res = ctx.Queue(), ctx.Queue(), ctx.Queue()
    pe = ctx.Process(target=exporter, args=(a, b, 4))
    pi = ctx.Process(target=importer, args=(a, b, close_each, res))
    pe.start()
    pi.start()
    seen = res.get(timeout=120)
    pe.join(60)
    pi.join(60)
    return seen


if __name__ == '__main__':
    out = {'close_and_reopen_each_round': run(True), 'keep_first_mapping': run(False)}
    line = json.dumps(out)
    print(line)
    if len(sys.argv) > 1:
        open(sys.argv[1], 'w').write(line + '\n')
