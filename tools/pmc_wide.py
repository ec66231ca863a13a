#!/usr/bin/env python3
"""HBM traffic of the 32-byte-unit kernels (round 4): MPI_LONG_DOUBLE_INT
MAXLOC and MPI_C_LONG_DOUBLE_COMPLEX SUM at 1 GiB per operand, once on
16-byte-aligned operands (k_contig32: whole-line packet loads and an
adjacent-lane swap) and once with both operands 8 bytes off the 16-byte grid
(k_elem: a unit per lane, its two packets 32 bytes apart).  Run under
`rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE` (one
counter block per pass), then summarise:

  python3 tools/pmc_wide.py                      # the workload (prints kernel ms)
  python3 tools/pmc_wide.py --summarise F.csv W.csv OUT.json [RUN.json]
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = (('MPI_LONG_DOUBLE_INT', 'MPI_MAXLOC'), ('MPI_C_LONG_DOUBLE_COMPLEX', 'MPI_SUM'))
NBYTES = 1 << 30
REPS = 5


def workload():
    import torch
    from mpich_amd import handles as H
    from mpich_amd import redop
    from bench import event_time_per_launch
    dev = torch.device('cuda', 0)
    a = torch.empty(NBYTES + 64, dtype=torch.uint8, device=dev)
    b = torch.empty(NBYTES + 64, dtype=torch.uint8, device=dev)
    a.view(torch.int8).random_(0, 3)
    b.view(torch.int8).random_(0, 3)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    rows = []
    for tn, on in CASES:
        dt, op = getattr(H, tn), getattr(H, on)
        ext = redop.datatype_extent(dt)
        for off in (0, 8):      # 8: both operands off the 16-byte grid -> k_elem
            n = (NBYTES - 64) // ext
            ia, ib = a[off:], b[off:]
            assert ia.data_ptr() % 16 == off and ib.data_ptr() % 16 == off

            def call():
                redop.check(redop.reduce_local_async(ib, ia, n, dt, op, s))
            call()
            avg, _, _ = event_time_per_launch(call, REPS, s, rounds=1)
            rows.append(dict(type=tn, op=on, offset=off, count=n, extent=ext,
                             kernel='k_contig32' if off == 0 else 'k_elem',
                             kernel_ms=round(avg, 4),
                             alg_GBs=round(3 * n * ext / (avg * 1e-3) / 1e9, 1)))
    torch.cuda.synchronize()
    print(json.dumps(dict(rows=rows)), flush=True)


def per_dispatch(path, counter):
    """[(kernel, grid, value)] in dispatch order"""
    out = []
    for r in csv.DictReader(open(path)):
        if r.get('Counter_Name', counter) != counter:
            continue
        out.append((r['Kernel_Name'], int(r['Grid_Size']), float(r['Counter_Value'])))
    return out


def summarise(fetch_csv, write_csv, out_path, run_json=None):
    f = per_dispatch(fetch_csv, 'FETCH_SIZE')
    w = per_dispatch(write_csv, 'WRITE_SIZE')
    rows = []
    runs = json.load(open(run_json))['rows'] if run_json else None
    groups = {}
    for name, grid, v in f:
        if name.startswith(('k_contig32', 'k_elem')):
            groups.setdefault((name, grid), [[], []])[0].append(v)
    for name, grid, v in w:
        if name.startswith(('k_contig32', 'k_elem')):
            groups.setdefault((name, grid), [[], []])[1].append(v)
    alg = 3 * NBYTES
    for (name, grid), (fv, wv) in groups.items():
        if not fv or not wv:
            continue
        fk, wk = statistics.median(fv), statistics.median(wv)
        rows.append(dict(kernel=name, grid=grid, launches=[len(fv), len(wv)],
                         fetch_kib_raw=fk, write_kib=wk,
                         read_over_2GiB_raw=round(fk * 1024 / (2 * NBYTES), 4),
                         read_over_2GiB_gfx950_corrected=round(2 * fk * 1024 / (2 * NBYTES), 4),
                         write_over_1GiB=round(wk * 1024 / NBYTES, 4),
                         hbm_over_algorithmic_corrected=round((2 * fk + wk) * 1024 / alg, 4)))
    out = dict(what='FETCH_SIZE / WRITE_SIZE per launch of the 32-byte-unit kernels, separate '
                    'rocprofv3 --pmc passes of tools/pmc_wide.py (1 GiB per operand; algorithmic '
                    '2 GiB read + 1 GiB written)',
               correction='MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE in KiB; on gfx950 '
                          'FETCH_SIZE counts half the bytes of 16-byte streaming reads (corrected '
                          'column doubles it; the raw column is kept since k_elem reads half '
                          'lines per instruction)',
               kernels=rows, timing=runs)
    with open(out_path, 'w') as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == '--summarise':
        summarise(*sys.argv[2:])
    else:
        workload()
