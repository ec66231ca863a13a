"""Register and scratch budget of the built gfx950 code objects (CPU: reads
the AMDGPU metadata of mpich_amd/csrc/build/inst_*.o, no GPU).

Every kernel of the library must run without scratch (a spill to private
memory is HBM traffic the roofline does not count, and a call stack in a
streaming kernel halves its occupancy), and the contiguous kernels -- the
headline and the config-3 rows -- must stay well under the 128-VGPR cap of
`__launch_bounds__(1024)`: the Annex G complex product sat at 128 with 32
bytes of scratch at four packets per lane until its slow path stopped reusing
the tile's registers ("Store policy"); at one packet per lane
(round 5) it is the plain per-element form again, its recovery inlined."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, 'mpich_amd', 'csrc', 'build')
OBJDUMP = '/opt/rocm/lib/llvm/bin/llvm-objdump'
READELF = '/opt/rocm/lib/llvm/bin/llvm-readelf'


def _kernels(obj):
    """[(name, vgpr_count, private_segment_fixed_size, kernarg_segment_size or -1 when
    the runtime's hidden arguments are part of it)] of the gfx950 code object in obj"""
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, os.path.basename(obj))
        shutil.copy(obj, src)
        subprocess.run([OBJDUMP, '--offloading', src], cwd=d, check=True, capture_output=True)
        dev = [f for f in os.listdir(d) if 'gfx950' in f]
        assert dev, 'no gfx950 code object in %s' % obj
        notes = subprocess.run([READELF, '--notes', os.path.join(d, dev[0])], check=True,
                               capture_output=True, text=True).stdout
    out = []
    for b in notes.split('  - .agpr_count')[1:]:
        m = re.search(r'\.name:\s+(\S+)', b)
        v = re.search(r'\.vgpr_count:\s+(\d+)', b)
        p = re.search(r'\.private_segment_fixed_size:\s+(\d+)', b)
        k = re.search(r'\.kernarg_segment_size:\s+(\d+)', b)
        if m and v and p and k:
            out.append((m.group(1), int(v.group(1)), int(p.group(1)),
                        -1 if '.value_kind:     hidden_' in b else int(k.group(1))))
    return out


@pytest.fixture(scope='module')
def kernels():
    if not (os.path.exists(OBJDUMP) and os.path.exists(READELF)):
        pytest.skip('ROCm llvm tools not found')
    objs = [os.path.join(BUILD, f + '.o') for f in ('inst_int', 'inst_fp', 'inst_pair')]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip('library objects not built (run __graft_entry__.build())')
    ks = []
    for o in objs:
        ks += _kernels(o)
    return ks


def test_no_kernel_uses_scratch(kernels):
    assert len(kernels) > 1000
    spilled = [(n, v, p) for n, v, p, _ in kernels if p]
    assert not spilled, spilled[:5]


def test_contiguous_kernels_under_the_vgpr_cap(kernels):
    contig = [(n, v) for n, v, _, _ in kernels if n.startswith('_ZN4mpix8k_contig')]
    assert len(contig) >= 200
    worst = max(contig, key=lambda x: x[1])
    assert worst[1] <= 96, worst


def test_contiguous_kernels_carry_no_hidden_arguments(kernels):
    """the combine kernels (contiguous, 32-byte, batch, element-wise, vector
    and iov targets, multi-input; not the tree forms, measured slower so) get
    their grid and block sizes as arguments:
    reading gridDim / blockDim would append the runtime's hidden-argument
    block (k_contig: 360 instead of 112 bytes), written by the host on every
    launch (bench.py call_floor_parts: up to 1 us per call)"""
    contig = [(n, k) for n, _, _, k in kernels if n.startswith('_ZN4mpix8k_contig')]
    assert len(contig) >= 200
    assert max(k for _, k in contig) <= 128, max(contig, key=lambda x: x[1])
    # -1: the metadata lists hidden_* arguments
    for prefix in ('_ZN4mpix8k_contig', '_ZN4mpix10k_contig32', '_ZN4mpix7k_batch',
                   '_ZN4mpix6k_elem', '_ZN4mpix8k_vector', '_ZN4mpix9k_vector1',
                   '_ZN4mpix11k_vector_s2', '_ZN4mpix5k_iov', '_ZN4mpix14k_contig_multi',
                   '_ZN4mpix12k_elem_multi'):
        ks = [(n, k) for n, _, _, k in kernels if n.startswith(prefix)]
        assert ks, prefix
        assert all(k >= 0 for _, k in ks), [n for n, k in ks if k < 0][:3]
