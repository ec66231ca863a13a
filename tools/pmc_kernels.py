"""Per-kernel summary of a rocprofv3 --pmc counter-collection CSV: for every
kernel name (and VGPR count, which tells the instantiations of one template
apart when the names are cut), the median over its dispatches of each
counter, and per-wave figures (counter / SQ_WAVES).  Used for the soft-float
kernels' instruction counts (round 6).

usage: pmc_kernels.py COUNTER_CSV [--what TEXT] > summary.json
"""
import argparse
import csv
import json
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--what', default='')
    a = ap.parse_args()
    # (kernel, vgprs) -> dispatch -> counter -> value (summed over the
    # per-XCD / per-SE rows a counter may have)
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for r in csv.DictReader(open(a.csv)):
        key = (r['Kernel_Name'], r.get('VGPR_Count', ''))
        per[key][r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
    out = {'what': a.what, 'kernels': []}
    for (name, vgpr), disp in sorted(per.items()):
        counters = sorted({c for d in disp.values() for c in d})
        med = {c: statistics.median(d[c] for d in disp.values() if c in d) for c in counters}
        row = {'kernel': name, 'vgpr_count': vgpr, 'dispatches': len(disp), 'median': med}
        waves = med.get('SQ_WAVES')
        if waves:
            row['per_wave'] = {c: round(v / waves, 2) for c, v in med.items()
                               if c.startswith('SQ_') and c != 'SQ_WAVES'}
        out['kernels'].append(row)
    json.dump(out, __import__('sys').stdout, indent=1)


if __name__ == '__main__':
    main()
