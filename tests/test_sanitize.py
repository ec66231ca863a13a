"""Host-side sanitizer runs (MPICH's --enable-g=asan,ubsan,tsan
equivalent for this path): the host C++ of libmpix_redop.so and
libmpix_coll.so built with AddressSanitizer + UndefinedBehaviorSanitizer
and, separately, ThreadSanitizer (mpich_amd/csrc/sanitize.mk), driven by the
pure-C program tests/c/coll_host_sanitize.c -- every reduce-scatter /
allreduce / reduce / scan schedule on the in-process host transport with
P = 1..8 threads, results checked against the reference tests' closed forms,
plus the argument and legality paths.  CPU only; no GPU is touched."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'mpich_amd', 'csrc')


@pytest.mark.parametrize('san', ['asan', 'tsan'])
def test_host_code_under_sanitizer(san):
    subprocess.run(['make', '-s', '-f', 'sanitize.mk', 'SAN=' + san], cwd=CSRC, check=True,
                   timeout=600)
    env = dict(os.environ)
    env['ASAN_OPTIONS'] = 'abort_on_error=0:halt_on_error=1:detect_leaks=1'
    env['UBSAN_OPTIONS'] = 'halt_on_error=1:print_stacktrace=1'
    env['TSAN_OPTIONS'] = 'halt_on_error=1:exitcode=66'
    p = subprocess.run([os.path.join(CSRC, 'build', san, 'coll_host_sanitize')], env=env,
                       capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-6000:])
    assert 'coll_host_sanitize: 0 errors' in p.stdout
    assert 'Sanitizer' not in p.stderr, p.stderr[-6000:]
