"""The support predicates and the performance knobs are CPU-only queries:
MPIR_Typerep_reduce_is_supported's counterpart runs for every reduce_local.c
call, host buffers and count 0 included (reduce_local.c:66-76), in processes
that may never touch a GPU or that fork afterwards.  They must not start the
HIP runtime (read_env() used to query the XCD count).

Checked by interposition: a stub library defining every hip* entry point
libmpix_redop.so imports (each one counts its calls) is loaded RTLD_GLOBAL
ahead of it in a fresh interpreter without torch, so the library's
references bind to the stubs; the fat-binary registration hooks (__hip*) stay
with the real runtime.  A positive control (MPIX_Redop_init, which must make
HIP calls) proves the stubs are the ones bound."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'mpich_amd', 'libmpix_redop.so')


def _hip_imports():
    out = subprocess.run(['nm', '-D', '--undefined-only', LIB], capture_output=True, text=True,
                         check=True).stdout
    names = set()
    for line in out.splitlines():
        sym = line.split()[-1].split('@')[0]
        if sym.startswith('hip'):
            names.add(sym)
    return sorted(names)


@pytest.fixture(scope='module')
def shim(tmp_path_factory):
    names = _hip_imports()
    assert 'hipGetDeviceCount' in names and 'hipPointerGetAttributes' in names
    d = tmp_path_factory.mktemp('hipshim')
    src = d / 'shim.c'
    body = ['#include <stdint.h>', 'volatile long shim_hits = 0;',
            'const char *shim_last = "";']
    for n in names:
        ret = 'const char *' if n == 'hipGetErrorString' else 'int'
        val = '"stub"' if ret != 'int' else '100'
        body.append('%s %s(void) { shim_hits++; shim_last = "%s"; return %s; }' % (ret, n, n, val))
    src.write_text('\n'.join(body) + '\n')
    so = d / 'libhipshim.so'
    subprocess.run(['gcc', '-shared', '-fPIC', '-O1', '-o', str(so), str(src)], check=True)
    return str(so)


def _probe(shim, calls):
    code = textwrap.dedent('''
        import ctypes, sys
        S = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_GLOBAL)
        L = ctypes.CDLL(sys.argv[2], mode=ctypes.RTLD_GLOBAL)
        hits = ctypes.c_long.in_dll(S, 'shim_hits')
        last = ctypes.c_char_p.in_dll(S, 'shim_last')
        i, a, vp = ctypes.c_int, ctypes.c_ssize_t, ctypes.c_void_p
        FLOAT, SUM, MAXLOC, TWOINT = 0x4c00040a, 0x58000003, 0x5800000c, 0x4c000816
        x = [i() for _ in range(4)]
        y = [a() for _ in range(3)]
        {calls}
        print(hits.value, last.value.decode())
        ''').format(calls=textwrap.indent(calls, ''))
    p = subprocess.run([sys.executable, '-c', code, shim, LIB], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    hits, _, last = p.stdout.strip().partition(' ')
    return int(hits), last


def test_queries_and_knobs_make_no_hip_call(shim):
    calls = '\n'.join([
        'L.MPIX_Redop_is_supported.argtypes = [i, a, i]',
        'assert L.MPIX_Redop_is_supported(SUM, 1 << 20, FLOAT) == 1',
        'assert L.MPIX_Redop_is_supported(SUM, 0, FLOAT) == 1',
        'assert L.MPIX_Redop_is_supported(MAXLOC, 7, TWOINT) == 1',
        'L.MPIX_Redop_is_supported_buffers.argtypes = [i, a, i, vp, vp]',
        'assert L.MPIX_Redop_is_supported_buffers(SUM, 0, FLOAT, None, None) == 1',
        'assert L.MPIX_Redop_has_gpu_path(SUM, FLOAT) == 1',
        'assert L.MPIX_Redop_op_dt_check(SUM, FLOAT) == 1',
        'assert L.MPIX_Datatype_extent(FLOAT) == 4',
        'assert L.MPIX_Redop_get_store_policy(*[ctypes.byref(v) for v in x]) == 0',
        'assert x[0].value == -1, x[0].value          # default not settled before a launch',
        'assert L.MPIX_Redop_set_store_policy(0x81, 0, 0, 0) == 0',
        'assert L.MPIX_Redop_set_store_policy(-1, 0, 0, 0) == 0',
        'assert L.MPIX_Redop_get_sync_store_policy(ctypes.byref(x[0])) == 0',
        'assert x[0].value == -1, x[0].value          # sync default unsettled too',
        'assert L.MPIX_Redop_set_sync_store_policy(0x22) == 0',
        'assert L.MPIX_Redop_set_sync_store_policy(-1) == 0',
        'assert L.MPIX_Redop_get_support(ctypes.byref(x[0]), *[ctypes.byref(v) for v in y]) == 0',
        'L.MPIX_Redop_set_support.argtypes = [i, a, a, a]',
        'assert L.MPIX_Redop_set_support(x[0], y[0], y[1], y[2]) == 0',
        'assert L.MPIX_Redop_get_pageable(ctypes.byref(x[0]), ctypes.byref(y[0])) == 0',
        'L.MPIX_Redop_set_pageable.argtypes = [i, a]',
        'assert L.MPIX_Redop_set_pageable(x[0], y[0]) == 0',
        'assert L.MPIX_Redop_get_launch(*[ctypes.byref(v) for v in x[:3]]) == 0',
        'assert L.MPIX_Redop_set_launch(x[0], x[2]) == 0',
        'assert L.MPIX_Redop_set_fortran_booleans(1, 0) == 0',
        'L.MPIX_Reduce_local.argtypes = [vp, vp, a, i, i]',
        'assert L.MPIX_Reduce_local(None, None, 0, FLOAT, SUM) == 0     # count 0',
        'assert L.MPIX_Reduce_local(None, None, -1, FLOAT, SUM) != 0    # bad count',
        # batch: argument and overlap errors are found before any HIP call
        'P = ctypes.c_void_p * 2; C = ctypes.c_ssize_t * 2',
        'assert L.MPIX_Reduce_local_batch_async(P(1 << 20, 2 << 20), P(4096, 4100), C(4, 4), 2,'
        ' FLOAT, SUM, None) == 1      # MPI_ERR_BUFFER',
        'assert L.MPIX_Reduce_local_batch_async(P(1 << 20, 2 << 20), P(4096, 8192), C(0, 0), 2,'
        ' FLOAT, SUM, None) == 0      # nothing to do',
    ])
    hits, last = _probe(shim, calls)
    assert hits == 0, 'HIP entered through %s' % last


def test_positive_control_init_is_intercepted(shim):
    hits, last = _probe(shim, 'L.MPIX_Redop_init()')
    assert hits > 0 and last.startswith('hip'), (hits, last)
