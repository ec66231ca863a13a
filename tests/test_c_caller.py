"""A pure-C program compiled against include/mpix_redop.h and linked with
libmpix_redop.so (tests/c/reduce_local_c.c).  Compiling it is a CPU check of
the C boundary; running it needs the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(out):
    subprocess.check_call([
        'gcc', '-std=c11', '-O2', '-Wall', '-Werror', '-D__HIP_PLATFORM_AMD__',
        '-I/opt/rocm/include', '-I' + os.path.join(ROOT, 'include'),
        os.path.join(ROOT, 'tests', 'c', 'reduce_local_c.c'),
        '-L' + os.path.join(ROOT, 'mpich_amd'), '-lmpix_redop', '-L/opt/rocm/lib', '-lamdhip64',
        '-Wl,-rpath,' + os.path.join(ROOT, 'mpich_amd'), '-Wl,-rpath,/opt/rocm/lib', '-o', out])


def test_c_caller_compiles_and_links(tmp_path):
    build(str(tmp_path / 'reduce_local_c'))


@pytest.mark.gpu
def test_c_caller_runs(tmp_path):
    exe = str(tmp_path / 'reduce_local_c')
    build(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'No Errors' in r.stdout
