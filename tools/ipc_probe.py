"""Does a freed and re-made device allocation come back with the same IPC
handle bytes and address, and does HIP_POINTER_ATTRIBUTE_BUFFER_ID tell the
two apart?  (What the pull schedules' peer-mapping cache keys on.)  Prints one
JSON line."""
import ctypes
import json

import torch  # noqa: F401  (one HIP runtime per process: torch's)

hip = ctypes.CDLL('libamdhip64.so.7')     # torch's runtime, already loaded under this SONAME
HIP_POINTER_ATTRIBUTE_BUFFER_ID = 7     # hip/driver_types.h: CONTEXT = 1, ..., BUFFER_ID


def main():
    torch.cuda.init()
    idx = HIP_POINTER_ATTRIBUTE_BUFFER_ID
    rows = []
    for i in range(4):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(64 << 20)) == 0
        h = ctypes.create_string_buffer(64)
        rc = hip.hipIpcGetMemHandle(h, p)
        bid = ctypes.c_ulonglong(0)
        rb = hip.hipPointerGetAttribute(ctypes.byref(bid), idx, p)
        rows.append(dict(i=i, ptr=hex(p.value), handle_rc=rc, handle=h.raw.hex(),
                         buffer_id_rc=rb, buffer_id=bid.value))
        assert hip.hipFree(p) == 0
    same_handle = len({r['handle'] for r in rows}) < len(rows)
    print(json.dumps({'ipc_probe': rows, 'attr_index': idx, 'handle_bytes_repeat': same_handle,
                      'buffer_ids_distinct': len({r['buffer_id'] for r in rows}) == len(rows)}))


if __name__ == '__main__':
    main()
