#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of a bench.py run into profiles/.

Inputs (rocprofv3 --output-format csv):
  --kt    <dir>/<name>_kernel_stats.csv   (--kernel-trace --stats pass)
  --fetch <dir>/<name>_counter_collection.csv  (--pmc FETCH_SIZE pass)
  --write <dir>/<name>_counter_collection.csv  (--pmc WRITE_SIZE pass)
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes
of a wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE
is exact for 16-byte streaming stores.  Counters come from separate passes
(TCC slots: FETCH_SIZE costs 3, WRITE_SIZE 2).
"""
import argparse
import csv
import json
import shutil
import statistics


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r.get('Counter_Name', counter) != counter:
            continue
        out.setdefault(r['Kernel_Name'], []).append((int(r['Grid_Size']), float(r['Counter_Value'])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--kt', required=True)
    ap.add_argument('--fetch', required=True)
    ap.add_argument('--write', required=True)
    ap.add_argument('--kernel', default='k_contig')
    ap.add_argument('--count', type=int, default=1 << 28)
    ap.add_argument('--elem', type=int, default=4)
    ap.add_argument('--out', required=True)
    ap.add_argument('--stats-copy', required=True)
    ap.add_argument('--trace', default=None,
                    help='the kernel-trace CSV of the --kt pass: launches that started from an idle '
                         'GPU (more than 5 us after the previous one ended: the synchronous loop and '
                         "bench.py's idle-start event timing) averaged apart from back-to-back ones")
    ap.add_argument('--traced-line', default=None,
                    help="the traced bench run's own JSON line (its ms_per_step is kept beside the "
                         "traced kernel average: traced kernel <= step time)")
    a = ap.parse_args()
    stats = {r['Name']: r for r in csv.DictReader(open(a.kt))}
    shutil.copy(a.kt, a.stats_copy)
    f = per_kernel(a.fetch, 'FETCH_SIZE')[a.kernel]
    w = per_kernel(a.write, 'WRITE_SIZE')[a.kernel]
    fetch_kib = statistics.median(v for _, v in f)
    write_kib = statistics.median(v for _, v in w)
    hbm = (2 * fetch_kib + write_kib) * 1024
    alg = 3 * a.count * a.elem
    k = stats[a.kernel]
    avg_ns = float(k['AverageNs'])
    summary = dict(
        source='rocprofv3 on MI355X (gfx950), ROCm 7.2, command: python3 bench.py (see '
               'tools/gpu_evidence.sh)',
        kernels={'reduce_local_fp32_sum': dict(
            kernel=a.kernel, count=a.count, launches_traced=int(k['Calls']),
            avg_duration_ns=avg_ns, min_ns=float(k['MinNs']), max_ns=float(k['MaxNs']),
            fetch_size_kib_raw=fetch_kib, write_size_kib=write_kib,
            hbm_bytes_per_launch=int(hbm), algorithmic_bytes_per_launch=alg,
            traffic_over_algorithmic=round(hbm / alg, 5),
            achieved_GBs_from_trace=round(alg / avg_ns, 1),
            frac_from_trace=round(alg / avg_ns / 8000.0, 4),
            correction='hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950 FETCH_SIZE half-count)')})
    if a.trace:
        rows = [r for r in csv.DictReader(open(a.trace)) if r['Kernel_Name'].startswith(a.kernel)]
        rows.sort(key=lambda r: int(r['Start_Timestamp']))
        idle, b2b = [], []
        for i, r in enumerate(rows):
            d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            gap = int(r['Start_Timestamp']) - int(rows[i - 1]['End_Timestamp']) if i else 10 ** 9
            (idle if gap > 5000 else b2b).append(d)
        kk = summary['kernels']['reduce_local_fp32_sum']
        if idle:
            kk['idle_start_launches'] = len(idle)
            kk['idle_start_avg_ns'] = round(sum(idle) / len(idle), 1)
            kk['frac_from_trace_idle_start'] = round(alg / (sum(idle) / len(idle)) / 8000.0, 4)
        if b2b:
            kk['back_to_back_launches'] = len(b2b)
            kk['back_to_back_avg_ns'] = round(sum(b2b) / len(b2b), 1)
    if a.traced_line:
        line = json.loads(open(a.traced_line).read().strip().splitlines()[-1])
        kk = summary['kernels']['reduce_local_fp32_sum']
        kk['traced_run_ms_per_step'] = line.get('ms_per_step')
        kk['traced_run_value'] = line.get('value')
        kk['traced_kernel_within_step'] = (line.get('ms_per_step') is not None and
                                           avg_ns * 1e-6 <= line['ms_per_step'])
    with open(a.out, 'w') as fo:
        json.dump(summary, fo, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main()
