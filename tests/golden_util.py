"""Helpers shared by the CPU (oracle) and GPU parity tests: load the golden
vectors committed under tests/golden/ and compare results per case mode."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load_cases():
    with open(os.path.join(GOLDEN, 'kat_manifest.json')) as f:
        man = json.load(f)
    vec = np.load(os.path.join(GOLDEN, 'kat_vectors.npz'), allow_pickle=False)
    out = []
    for c in man['cases']:
        c = dict(c)
        c['inputs'] = vec[c['id'] + '_in']
        c['expected'] = vec[c['id'] + '_out']
        out.append(c)
    return out


def layout_dtype(layout):
    if isinstance(layout, str):
        return np.dtype(layout)
    return np.dtype([tuple(x) for x in layout])


def _float_view(dt):
    """per-element float sub-arrays of a dtype, for NaN-equivalence checks"""
    if dt.kind == 'c':
        return np.dtype('<f%d' % (dt.itemsize // 2))
    return dt


def mismatches(case, got):
    """number of elements where `got` (uint8 bytes) differs from the case's
    expected bytes, under the case's comparison mode."""
    exp = case['expected']
    got = np.asarray(got, np.uint8)
    assert got.shape == exp.shape
    mode = case['cmp']
    dt = layout_dtype(case['layout'])
    if mode == 'bytes':
        g = got.reshape(-1, dt.itemsize)
        e = exp.reshape(-1, dt.itemsize)
        return int(np.any(g != e, axis=1).sum())
    if mode == 'nan_equiv':
        fv = _float_view(dt)
        g = got.view(fv)
        e = exp.view(fv)
        gn, en = np.isnan(g), np.isnan(e)
        bad = (g.view(np.uint8).reshape(len(g), -1) != e.view(np.uint8).reshape(len(e), -1)).any(1)
        bad = np.where(gn | en, gn != en, bad)
        return int(bad.sum())
    if mode == 'fields':
        g = got.view(dt)
        e = exp.view(dt)
        bad = np.zeros(len(g), bool)
        for f in ('v', 'l'):
            bad |= g[f] != e[f]
        return int(bad.sum())
    raise ValueError(mode)


def fold(case, reduce_fn):
    """acc = inputs[0]; acc = reduce_local(in=inputs[r], inout=acc) for r>0.
    reduce_fn(in_bytes, inout_bytes, count, datatype, op) -> rc, in place."""
    ins = case['inputs']
    acc = ins[0].copy()
    for r in range(1, case['nranks']):
        src = ins[r].copy()
        rc = reduce_fn(src, acc, case['count'], case['datatype'], case['op'])
        if rc:
            return rc, acc
    return 0, acc
