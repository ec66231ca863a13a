#!/usr/bin/env python3
"""HBM traffic of the multi-input and tree combines: summarise separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes of
`tools/multi_probe.py --mib M --ks K --tree-ks T` (every combine is launched
once untimed, then 3 batches of 10, in the order of --ks, then --tree-ks).

  python3 tools/pmc_multi.py FETCH.csv WRITE.csv OUT.json [--mib 256] [--ks ..] [--tree-ks ..]

Per k: median FETCH_SIZE (KiB, doubled: gfx950 counts half the bytes of
16-byte streaming reads, MI355X_MICROARCH.md) and WRITE_SIZE per launch
against the algorithmic bytes ((k + 2) S read+written for the multi-input
fold, (k + 1) S for the tree into a separate output)."""
import argparse
import csv
import json
import statistics

PER_K = 31      # multi_probe.py: one untimed call + 3 x 10 timed launches


def dispatches(path, counter, prefix):
    rows = [r for r in csv.DictReader(open(path))
            if r.get('Counter_Name', counter) == counter and r['Kernel_Name'].startswith(prefix)]
    rows.sort(key=lambda r: int(r.get('Dispatch_Id', 0)))
    return [float(r['Counter_Value']) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch')
    ap.add_argument('write')
    ap.add_argument('out')
    ap.add_argument('--mib', type=int, default=256)
    ap.add_argument('--ks', default='1,2,3,4,7,15')
    ap.add_argument('--tree-ks', default='2,4,8,16')
    a = ap.parse_args()
    S = a.mib << 20
    res = []
    for kind, prefix, ks, streams in (('multi', 'k_contig_multi', a.ks, lambda k: k + 2),
                                      ('tree', 'k_contig_tree', a.tree_ks, lambda k: k + 1)):
        f = dispatches(a.fetch, 'FETCH_SIZE', prefix)
        w = dispatches(a.write, 'WRITE_SIZE', prefix)
        for i, k in enumerate(int(x) for x in ks.split(',')):
            fk = statistics.median(f[i * PER_K:(i + 1) * PER_K])
            wk = statistics.median(w[i * PER_K:(i + 1) * PER_K])
            alg = streams(k) * S
            res.append(dict(kind=kind, k=k, launches=[len(f[i * PER_K:(i + 1) * PER_K]),
                                                      len(w[i * PER_K:(i + 1) * PER_K])],
                            fetch_kib_raw=fk, write_kib=wk,
                            hbm_over_algorithmic=round((2 * fk + wk) * 1024 / alg, 4)))
    out = dict(what='HBM bytes per launch of the multi-input and tree combines (fp32 SUM, %d MiB '
                    'per operand), separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of '
                    'tools/multi_probe.py, gfx950-corrected' % a.mib, rows=res)
    with open(a.out, 'w') as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
