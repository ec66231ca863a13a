"""bench.py's own host logic on CPU: the numpy restatement of the
recursive-halving association that gates the N > 1 value (checked here
against the oracle's simulation of reduce_scatter_block_intra_recursive_halving.c),
and the watchdogs that turn a hung leg into rank 0's error line plus a
non-zero exit status."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize('world', [2, 3, 4, 5, 6, 7, 8])
def test_rh_expected_block_matches_oracle(oracle, world):
    import bench
    rc = 1031
    sends = [bench.rsb_inputs_host(r, world, rc) for r in range(world)]
    exp = oracle.rsb_recursive_halving([s.view(np.uint8) for s in sends], rc, 0x4c00040a, 0x58000003)
    for r in range(world):
        assert bench.rh_expected_block(sends, r, rc).tobytes() == exp[r].tobytes(), r


def _run(code):
    return subprocess.run([sys.executable, '-c', textwrap.dedent(code)], cwd=ROOT,
                          capture_output=True, text=True, timeout=60)


def test_value_leg_watchdog_prints_error_and_exits_2():
    p = _run("""
        import time, bench
        e = bench._Emitter(0, {'metric': 'm', 'value': None, 'error': 'value leg did not finish'})
        bench._watchdog(0.3, e, note=False, code=2)
        time.sleep(10)
        """)
    assert p.returncode == 2
    assert '"error": "value leg did not finish"' in p.stdout
    assert 'extras_watchdog' not in p.stdout


def test_extras_watchdog_keeps_headline_and_exits_3():
    p = _run("""
        import time, bench
        e = bench._Emitter(0, {'metric': 'm', 'value': 1.5})
        bench._watchdog(0.3, e)
        time.sleep(10)
        """)
    assert p.returncode == 3
    assert '"value": 1.5' in p.stdout and 'extras_watchdog' in p.stdout and '"error"' in p.stdout


def test_emitter_prints_once_and_only_on_rank0():
    p = _run("""
        import bench
        e = bench._Emitter(0, {'v': 1})
        e.emit(); e.emit('late')
        bench._Emitter(1, {'v': 2}).emit()
        """)
    assert p.returncode == 0
    assert p.stdout.strip().splitlines() == ['{"v": 1}']
