"""The launch grid cap: HIP rejects a dispatch of more than
UINT32_MAX work-items, so mpix::grid_for caps the grid at
floor((2^32 - 1) / block) blocks and the kernels stride over the rest.
Host-only: tests/c/grid_cap_check.cpp built with g++ against the same
header the launchers use (mpich_amd/csrc/redop_dispatch.h)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_grid_cap_host(tmp_path):
    exe = str(tmp_path / 'grid_cap_check')
    subprocess.run(['g++', '-O2', '-std=c++17', '-Wall', '-D__HIP_PLATFORM_AMD__',
                    '-I/opt/rocm/include', '-I' + os.path.join(ROOT, 'mpich_amd', 'csrc'),
                    '-o', exe, os.path.join(ROOT, 'tests', 'c', 'grid_cap_check.cpp')], check=True)
    p = subprocess.run([exe], capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
    assert 'grid cap: ok' in p.stdout
